// The synthetic env's per-element step (SyntheticAtariEnv, envs.py): counter-based splitmix64
// values of (seed, step id, env, element), so any launch that knows an env's action can step it.
// Shared by synth_env_kernel (ocppo_rollout.hip) and the policy head's fused env step
// (ocppo_loss.hip): one definition, bitwise the same frames either way.
#pragma once
#include "ocppo_common.h"

namespace ocppo {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float unit24(uint64_t h) {  // exact multiple of 2^-24 in [0, 1)
  return static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
}

// env n's key at step id `step`
__device__ __forceinline__ uint64_t synth_env_key(uint64_t seed, uint64_t step, int64_t n) {
  return splitmix64(splitmix64(splitmix64(seed) + step) + static_cast<uint64_t>(n));
}

// object frames: element k of the newest frame (x, y, w/h fields; y of object 0 follows the
// action), in two parts so that a caller can hash before it knows the action: the action-free
// value, then the action applied (element 1 only)
__device__ __forceinline__ uint32_t synth_env_obj_base(uint64_t key, int64_t k) {
  const uint64_t h = splitmix64(key + static_cast<uint64_t>(k));
  const int field = static_cast<int>(k & 3);
  if (field == 0) return static_cast<uint32_t>(h % 160u);
  if (field == 1) return static_cast<uint32_t>(h % 210u);
  return static_cast<uint32_t>(1u + h % 16u);
}
__device__ __forceinline__ float synth_env_obj_act(uint32_t base, int64_t k, int64_t a) {
  const uint64_t v = (k == 1) ? (base + 7u * static_cast<uint64_t>(a)) % 210u : base;
  return static_cast<float>(v);
}
__device__ __forceinline__ float synth_env_obj(uint64_t key, int64_t k, int64_t a) {
  return synth_env_obj_act(synth_env_obj_base(key, k), k, a);
}

// pixel frames: byte k (row 0 encodes the action)
__device__ __forceinline__ uint8_t synth_env_pixel(uint64_t key, int64_t k, int64_t a) {
  const uint64_t h = splitmix64(key + static_cast<uint64_t>(k));
  uint32_t v = (h % 10u == 0u) ? static_cast<uint32_t>((h >> 8) & 0xFFu) : 0u;
  if (k < 84) v = static_cast<uint32_t>((a * 37) & 0xFF);
  return static_cast<uint8_t>(v);
}

// reward / done of env n and its RecordEpisodeStatistics counters (one thread per env)
__device__ __forceinline__ void synth_env_outcome(uint64_t key, int64_t n,
                                                  float* __restrict__ reward_out,
                                                  float* __restrict__ done_out,
                                                  float* __restrict__ ep) {
  const float ur = unit24(splitmix64(key ^ 0x5DEECE66Dull));
  const float r = ur < 0.005f ? 1.f : (ur < 0.01f ? -1.f : 0.f);
  const float ud = unit24(splitmix64(key ^ 0xB5297A4Dull));
  const float d = ud < (1.0f / 3500.0f) ? 1.f : 0.f;
  reward_out[n] = r;
  done_out[n] = d;
  if (ep) {
    float* e = ep + n * 5;
    const float run_ret = e[0] + r, run_len = e[1] + 1.f;
    if (d != 0.f) {
      e[2] += run_ret;
      e[3] += run_len;
      e[4] += 1.f;
      e[0] = 0.f;
      e[1] = 0.f;
    } else {
      e[0] = run_ret;
      e[1] = run_len;
    }
  }
}

}  // namespace ocppo
