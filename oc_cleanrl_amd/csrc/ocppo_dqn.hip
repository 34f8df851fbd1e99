// DQN path of config 5 (cleanrl/dqn_atari_oc.py): an HBM replay buffer with stable-baselines3
// ReplayBuffer(optimize_memory_usage=True) semantics (:317-325, :369, :377) and the fused TD-target
// + MSE loss forward/backward (:378-382).
//
// Replay layout: obs [size, E, D] in the storage dtype (u8 pixels / bf16 objects: exact),
// actions [size, E] i64, rewards / dones [size, E] f32; state = device int64 {pos, full}.
// `add` writes obs at pos and next_obs at (pos+1) % size (the memory-optimised variant: slot i+1
// holds transition i's next obs); `sample` draws, like SB3, batch indices in [0, pos) or, once
// full, (randint(1, size) + pos) % size (never the slot being overwritten), and an env index
// uniform in [0, E). Random numbers come from a counter-based splitmix64 stream (device counter),
// so sampling is graph-replayable; the law is SB3's, the bits are not numpy's (parity of the
// sampler is by distribution, the TD math is bit-level).
#include "ocppo_common.h"
#include "ocppo_categorical.h"
#include "ocppo_store.h"
#include "ocppo_synth_env.h"

namespace ocppo {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <int SDT, int ODT>
__global__ __launch_bounds__(256) void replay_add_kernel(
    const void* __restrict__ obs, const void* __restrict__ next_obs,
    const int64_t* __restrict__ actions, const float* __restrict__ rewards,
    const float* __restrict__ dones, int64_t E, int64_t D, int64_t* state, int64_t size,
    void* __restrict__ rb_obs, int64_t* __restrict__ rb_act, float* __restrict__ rb_rew,
    float* __restrict__ rb_done, unsigned* ticket) {
  __shared__ int s_last;
  const int64_t pos = __hip_atomic_load(&state[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t nxt = (pos + 1) % size;
  const int64_t total = E * D;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
       g += stride) {
    Elem<ODT>::store(static_cast<typename Elem<ODT>::T*>(rb_obs), pos * total + g,
                     Elem<SDT>::load(static_cast<const typename Elem<SDT>::T*>(obs), g));
    Elem<ODT>::store(static_cast<typename Elem<ODT>::T*>(rb_obs), nxt * total + g,
                     Elem<SDT>::load(static_cast<const typename Elem<SDT>::T*>(next_obs), g));
    if (g < E) {
      rb_act[pos * E + g] = actions[g];
      rb_rew[pos * E + g] = rewards[g];
      rb_done[pos * E + g] = dones[g];
    }
  }
  // every workgroup has read `pos`; the last one to arrive advances it (graph-replay safe)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
    if (s_last) {
      const int64_t p1 = pos + 1;
      if (p1 == size) {
        __hip_atomic_store(&state[1], int64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&state[0], int64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        __hip_atomic_store(&state[0], p1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One thread per (sample, element group); the sample's indices are recomputed per thread from the
// counter-based stream (cheap) so no cross-thread hand-off is needed.
__device__ __forceinline__ void sample_index(uint64_t seed, int64_t ctr, int64_t b, int64_t pos,
                                             int64_t full, int64_t size, int64_t E, int64_t& i,
                                             int64_t& e) {
  const uint64_t h = mix64(mix64(seed ^ 0xD1B54A32D192ED03ull) + static_cast<uint64_t>(ctr) * 0x100000001B3ull +
                           static_cast<uint64_t>(b));
  const uint64_t h2 = mix64(h);
  if (full)
    i = (static_cast<int64_t>(h % static_cast<uint64_t>(size - 1)) + 1 + pos) % size;
  else
    i = static_cast<int64_t>(h % static_cast<uint64_t>(pos > 0 ? pos : 1));
  e = static_cast<int64_t>(h2 % static_cast<uint64_t>(E));
}

template <int ODT>
__global__ __launch_bounds__(256) void replay_sample_kernel(
    uint64_t seed, const int64_t* __restrict__ counter, const int64_t* __restrict__ state,
    int64_t size, int64_t E, int64_t D, const void* __restrict__ rb_obs,
    const int64_t* __restrict__ rb_act, const float* __restrict__ rb_rew,
    const float* __restrict__ rb_done, int64_t B, float* __restrict__ obs_out,
    float* __restrict__ next_out, int64_t* __restrict__ act_out, float* __restrict__ rew_out,
    float* __restrict__ done_out, int64_t* __restrict__ idx_out) {
  const int64_t pos = state[0], full = state[1];
  const int64_t ctr = counter[0];
  const int64_t total = B * D;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
       g += stride) {
    const int64_t b = g / D, k = g - b * D;
    int64_t i, e;
    sample_index(seed, ctr, b, pos, full, size, E, i, e);
    const auto* src = static_cast<const typename Elem<ODT>::T*>(rb_obs);
    obs_out[g] = Elem<ODT>::load(src, (i * E + e) * D + k);
    next_out[g] = Elem<ODT>::load(src, (((i + 1) % size) * E + e) * D + k);
    if (k == 0) {
      act_out[b] = rb_act[i * E + e];
      rew_out[b] = rb_rew[i * E + e];
      done_out[b] = rb_done[i * E + e];
      if (idx_out) {
        idx_out[2 * b] = i;
        idx_out[2 * b + 1] = e;
      }
    }
  }
}

__global__ void counter_add_kernel(int64_t* counter, int64_t n) { counter[0] += n; }

// epsilon-greedy (dqn_atari_oc.py:345-350): epsilon = max(slope * t + start_e, end_e) with
// slope = (end_e - start_e) / duration (linear_schedule, :230-232, in double); ONE coin for all
// envs; random actions uniform in [0, A), else argmax_j q[e, j] (first maximum, like torch).
__global__ __launch_bounds__(256) void epsilon_greedy_kernel(
    const float* __restrict__ q, int64_t E, int A, uint64_t seed, const int64_t* __restrict__ step,
    int64_t step_offset, double start_e, double end_e, double duration,
    int64_t* __restrict__ actions, float* __restrict__ eps_out) {
  const int64_t t = step[0] + step_offset;
  const double slope = (end_e - start_e) / duration;
  double eps = slope * static_cast<double>(t) + start_e;
  eps = eps > end_e ? eps : end_e;
  const uint64_t h = mix64(mix64(seed ^ 0xA0761D6478BD642Full) + static_cast<uint64_t>(t));
  const double coin = static_cast<double>(h >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
  const bool explore = coin < eps;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < E;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    int64_t a;
    if (explore) {
      a = static_cast<int64_t>(mix64(h + static_cast<uint64_t>(e) + 1) % static_cast<uint64_t>(A));
    } else {
      int best = 0;
      float bq = q[e * A];
      for (int j = 1; j < A; ++j) {
        const float v = q[e * A + j];
        if (v > bq || (v != v && bq == bq)) {
          bq = v;
          best = j;
        }
      }
      a = best;
    }
    actions[e] = a;
  }
  if (eps_out && blockIdx.x == 0 && threadIdx.x == 0) eps_out[0] = static_cast<float>(eps);
}

// The acting step's Q head and epsilon-greedy choice in one launch (dqn_atari_oc.py:345-352:
// `q_values = q_network(obs); actions = argmax(q_values)` or a uniform random action with
// probability epsilon): one wave per env, the head's A <= 8 weight rows in registers, the A dot
// products of the hidden row by the policy head's reduce-scatter butterfly, then exactly
// epsilon_greedy_kernel's coin, argmax rule and random action on those values.
template <int CH>
__global__ __launch_bounds__(256) void q_head_eps_kernel(
    const float* __restrict__ hidden, int64_t E, const float* __restrict__ wq,
    const float* __restrict__ bq, int A, uint64_t seed, const int64_t* __restrict__ step,
    int64_t step_offset, double start_e, double end_e, double duration,
    int64_t* __restrict__ actions, float* __restrict__ eps_out, float* __restrict__ q_out) {
  constexpr int H = 256 * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 4 + wv;
  if (e >= E) return;  // wave-uniform
  const int jo = lane >> 3;
  const float bias = jo < A ? bq[jo] : 0.f;
  float4 w[8][CH];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int c = 0; c < CH; ++c)
      w[j][c] = j < A ? reinterpret_cast<const float4*>(wq + static_cast<int64_t>(j) * H)[c * kWave + lane]
                      : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 x[CH];
  head_load_row<CH>(hidden, e, lane, x);
  const float t = head_dots<CH>(x, w, lane) + bias;
  const int64_t ts = step[0] + step_offset;
  const double slope = (end_e - start_e) / duration;
  double eps = slope * static_cast<double>(ts) + start_e;
  eps = eps > end_e ? eps : end_e;
  const uint64_t hh = mix64(mix64(seed ^ 0xA0761D6478BD642Full) + static_cast<uint64_t>(ts));
  const double coin = static_cast<double>(hh >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
  float q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 8 * j));
  int64_t a;
  if (coin < eps) {
    a = static_cast<int64_t>(mix64(hh + static_cast<uint64_t>(e) + 1) % static_cast<uint64_t>(A));
  } else {
    int best = 0;
    float bqv = q[0];
#pragma unroll
    for (int j = 1; j < 8; ++j)
      if (j < A && (q[j] > bqv || (q[j] != q[j] && bqv == bqv))) {
        bqv = q[j];
        best = j;
      }
    a = best;
  }
  if (lane == 0) actions[e] = a;
  const float mine = __shfl(t, 8 * (lane & 7), kWave);  // all lanes take part in the permute
  if (q_out && lane < A) q_out[e * A + lane] = mine;
  if (eps_out && e == 0 && lane == 0) eps_out[0] = static_cast<float>(eps);
}

// Fused TD target + MSE loss, forward and backward w.r.t. q (dqn_atari_oc.py:378-382):
//   target_max = max_a q_next;  td = r + (f32(gamma) * target_max) * (1 - d)
//   old = q[b, a_b];  loss = mean((td - old)^2);  dq[b, j] = j == a_b ? (old - td) * (2/B) : 0
// One workgroup (B is the DQN minibatch, 32 in the reference).
__global__ __launch_bounds__(1024) void td_loss_kernel(const float* __restrict__ q,
                                                       const float* __restrict__ q_next,
                                                       const int64_t* __restrict__ actions,
                                                       const float* __restrict__ rewards,
                                                       const float* __restrict__ dones, int64_t B,
                                                       int A, float gamma, float norm,
                                                       float* __restrict__ dq,
                                                       float* __restrict__ stats) {
  __shared__ float scratch[16];
  float se = 0.f, sq = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += blockDim.x) {
    float m = q_next[b * A];
    for (int j = 1; j < A; ++j) m = fmaxf(m, q_next[b * A + j]);
    const float td = rewards[b] + (gamma * m) * (1.0f - dones[b]);
    const int64_t a = actions[b];
    const float old = q[b * A + a];
    const float diff = td - old;
    se += diff * diff;
    sq += old;
    const float g = (old - td) * norm;  // mse_loss_backward w.r.t. its `target` argument
    for (int j = 0; j < A; ++j) dq[b * A + j] = j == a ? g : 0.f;
  }
  se = block_sum(se, scratch);
  sq = block_sum(sq, scratch);
  if (threadIdx.x == 0) {
    stats[0] = se / static_cast<float>(B);  // losses/td_loss
    stats[1] = sq / static_cast<float>(B);  // losses/q_values (old_val.mean())
  }
}

// ---- one acting step of the DQN loop in ONE launch (dqn_atari_oc.py:345-372) --------------------
// The Q head + epsilon-greedy choice (q_head_eps_kernel's arithmetic), the object-frame synthetic
// env's step on those actions (synth_env_kernel's), the frame-stack store + VecNormalize
// (store_vecnorm_kernel's: store_groups / vecnorm_block) and the replay add of (obs, next_obs,
// action, reward, done) (replay_add_kernel's), as four phases of ONE workgroup separated by
// barriers: every value is the one the four launches write, in the same order; the step's chain of
// four dependent launches (4-5 us each at one env) becomes one. E <= 64 envs (one workgroup).
struct DqnActArgs {
  const float* hidden;
  int64_t E;
  const float* wq;
  const float* bq;
  int A;
  uint64_t seed;
  int64_t* step;
  int64_t step_offset;
  double start_e, end_e, duration;
  int64_t* actions;
  float* eps_out;
  uint64_t env_seed;
  int64_t* env_step_base;
  int64_t env_step_offset, D;
  float* frame;
  float* env_reward;
  float* env_done;
  float* ep;
  int W;
  const void* prev;
  void* out;
  float* net;
  float* done_out;
  float* reward_out;
  int vecnorm;
  double vn_gamma, vn_eps, vn_clip;
  double* ret;
  double* rms;
  int64_t* rb_state;
  int64_t rb_size;
  void* rb_obs;
  int64_t* rb_act;
  float* rb_rew;
  float* rb_done;
  int64_t advance;  // added to *step and *env_step_base at the end (the chunk's last env step)
};
constexpr int kDqnActMaxE = 64;

template <int CH, int ODT>
__global__ __launch_bounds__(256) void dqn_act_step_kernel(DqnActArgs p) {
  __shared__ int64_t s_act[kDqnActMaxE];
  constexpr int H = 256 * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t E = p.E;
  // 1. Q head + epsilon-greedy, one wave per env
  {
    const int jo = lane >> 3;
    const float bias = jo < p.A ? p.bq[jo] : 0.f;
    float4 w[8][CH];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int c = 0; c < CH; ++c)
        w[j][c] = j < p.A ? reinterpret_cast<const float4*>(p.wq + static_cast<int64_t>(j) * H)[c * kWave + lane]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t ts = p.step[0] + p.step_offset;
    const double slope = (p.end_e - p.start_e) / p.duration;
    double eps = slope * static_cast<double>(ts) + p.start_e;
    eps = eps > p.end_e ? eps : p.end_e;
    const uint64_t hh = mix64(mix64(p.seed ^ 0xA0761D6478BD642Full) + static_cast<uint64_t>(ts));
    const double coin = static_cast<double>(hh >> 11) * (1.0 / 9007199254740992.0);  // [0, 1)
    for (int64_t e = wv; e < E; e += 4) {  // wave-uniform
      float4 x[CH];
      head_load_row<CH>(p.hidden, e, lane, x);
      const float t = head_dots<CH>(x, w, lane) + bias;
      float q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 8 * j));
      int64_t a;
      if (coin < eps) {
        a = static_cast<int64_t>(mix64(hh + static_cast<uint64_t>(e) + 1) % static_cast<uint64_t>(p.A));
      } else {
        int best = 0;
        float bqv = q[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)
          if (j < p.A && (q[j] > bqv || (q[j] != q[j] && bqv == bqv))) {
            bqv = q[j];
            best = j;
          }
        a = best;
      }
      if (lane == 0) {
        p.actions[e] = a;
        s_act[e] = a;
      }
    }
    if (p.eps_out && threadIdx.x == 0) p.eps_out[0] = static_cast<float>(eps);
  }
  __syncthreads();
  // 2. the env step on those actions (object frames)
  {
    const uint64_t st = static_cast<uint64_t>(p.env_step_base[0] + p.env_step_offset);
    for (int64_t g = threadIdx.x; g < E * p.D; g += blockDim.x) {
      const int64_t n = g / p.D, k = g - n * p.D;
      const uint64_t key = synth_env_key(p.env_seed, st, n);
      p.frame[g] = synth_env_obj(key, k, s_act[n]);
      if (k == 0) synth_env_outcome(key, n, p.env_reward, p.env_done, p.ep);
    }
  }
  __syncthreads();
  // 3. store (+ VecNormalize)
  if (p.vecnorm) {
    vecnorm_block(p.env_reward, p.env_done, E, p.vn_gamma, p.vn_eps, p.vn_clip, p.ret, p.rms,
                  p.reward_out);
    store_groups<OCPPO_F32, ODT, 1>(0, 1, p.frame, p.env_reward, p.env_done, E, p.W, p.D, p.prev,
                                    p.out, p.net, nullptr, p.done_out, 1.0f, nullptr);
  } else {
    store_groups<OCPPO_F32, ODT, 1>(0, 1, p.frame, p.env_reward, p.env_done, E, p.W, p.D, p.prev,
                                    p.out, p.net, p.reward_out, p.done_out, 1.0f, nullptr);
  }
  __syncthreads();
  // 4. replay add of (prev, out, action, reward_out, done_out) at pos; pos advanced after
  const int64_t pos = p.rb_state[0];
  const int64_t nxt = (pos + 1) % p.rb_size;
  const int64_t total = E * p.W * p.D;
  using T = typename Elem<ODT>::T;
  const T* pv = static_cast<const T*>(p.prev);
  const T* ov = static_cast<const T*>(p.out);
  T* rb = static_cast<T*>(p.rb_obs);
  for (int64_t g = threadIdx.x; g < total; g += blockDim.x) {
    rb[pos * total + g] = pv[g];
    rb[nxt * total + g] = ov[g];
    if (g < E) {
      p.rb_act[pos * E + g] = s_act[g];
      p.rb_rew[pos * E + g] = p.reward_out[g];
      p.rb_done[pos * E + g] = p.done_out[g];
    }
  }
  __syncthreads();  // every thread has read pos
  if (threadIdx.x == 0) {
    const int64_t p1 = pos + 1;
    if (p1 == p.rb_size) {
      p.rb_state[1] = 1;
      p.rb_state[0] = 0;
    } else {
      p.rb_state[0] = p1;
    }
    if (p.advance) {  // both counters were read in phases 1 and 2, before the barriers
      p.step[0] += p.advance;
      p.env_step_base[0] += p.advance;
    }
  }
}

}  // namespace ocppo

using namespace ocppo;

extern "C" size_t ocppo_replay_workspace_bytes(void) { return 256; }

extern "C" int ocppo_dqn_act_step(
    ocppo_stream_t stream, const float* hidden, int64_t E, int64_t H, const float* wq,
    const float* bq, int64_t A, uint64_t seed, int64_t* step, int64_t step_offset,
    double start_e, double end_e, double duration, int64_t* actions, float* epsilon_out,
    uint64_t env_seed, int64_t* env_step_base, int64_t env_step_offset, int64_t D,
    float* frame, float* env_reward, float* env_done, float* ep_state, int64_t W,
    const void* prev_obs, void* obs_out, int obs_dtype, float* net_obs, float* done_out,
    float* reward_out, int vecnorm, double vn_gamma, double vn_epsilon, double vn_clip,
    double* ret_state, double* rms_state, int64_t* rb_state, int64_t rb_size, void* rb_obs,
    int64_t* rb_actions, float* rb_rewards, float* rb_dones, int64_t advance) {
  OCPPO_REQUIRE(E >= 1 && E <= kDqnActMaxE && A >= 1 && A <= 8 && H >= 256 && H % 256 == 0 &&
                    H <= 1024 && D >= 1 && W >= 1 && W <= 64 && rb_size >= 2 && duration > 0,
                "ocppo_dqn_act_step: bad sizes E=%lld H=%lld A=%lld D=%lld W=%lld (E <= %d, A <= "
                "8, H a multiple of 256 <= 1024)", (long long)E, (long long)H, (long long)A,
                (long long)D, (long long)W, kDqnActMaxE);
  OCPPO_REQUIRE(hidden && wq && bq && step && actions && env_step_base && frame && env_reward &&
                    env_done && prev_obs && obs_out && done_out && reward_out && rb_state &&
                    rb_obs && rb_actions && rb_rewards && rb_dones &&
                    (!vecnorm || (ret_state && rms_state)),
                "ocppo_dqn_act_step: null pointer");
  OCPPO_REQUIRE(((reinterpret_cast<uintptr_t>(hidden) | reinterpret_cast<uintptr_t>(wq)) & 15) == 0,
                "ocppo_dqn_act_step: hidden and wq must be 16-B aligned");
  OCPPO_REQUIRE(prev_obs != obs_out && reward_out != env_reward,
                "ocppo_dqn_act_step: prev_obs / obs_out and reward / reward_out must not alias");
  OCPPO_REQUIRE(obs_dtype == OCPPO_F32 || obs_dtype == OCPPO_BF16 || obs_dtype == OCPPO_U8,
                "ocppo_dqn_act_step: bad obs dtype %d", obs_dtype);
  DqnActArgs p{hidden, E, wq, bq, (int)A, seed, step, step_offset, start_e, end_e, duration,
               actions, epsilon_out, env_seed, env_step_base, env_step_offset, D, frame,
               env_reward, env_done, ep_state, (int)W, prev_obs, obs_out, net_obs, done_out,
               reward_out, vecnorm ? 1 : 0, vn_gamma, vn_epsilon, vn_clip, ret_state, rms_state,
               rb_state, rb_size, rb_obs, rb_actions, rb_rewards, rb_dones, advance};
  clear_stale_error();
  hipStream_t s = as_stream(stream);
#define OCPPO_DA(CH, O) \
  hipLaunchKernelGGL((dqn_act_step_kernel<CH, O>), dim3(1), dim3(256), 0, s, p)
#define OCPPO_DA_CH(O)            \
  switch (H / 256) {              \
    case 1: OCPPO_DA(1, O); break; \
    case 2: OCPPO_DA(2, O); break; \
    case 3: OCPPO_DA(3, O); break; \
    default: OCPPO_DA(4, O); break; \
  }
  if (obs_dtype == OCPPO_F32) {
    OCPPO_DA_CH(OCPPO_F32)
  } else if (obs_dtype == OCPPO_BF16) {
    OCPPO_DA_CH(OCPPO_BF16)
  } else {
    OCPPO_DA_CH(OCPPO_U8)
  }
#undef OCPPO_DA_CH
#undef OCPPO_DA
  return check_launch("ocppo_dqn_act_step");
}

extern "C" int ocppo_replay_add(ocppo_stream_t stream, const void* obs, const void* next_obs,
                                int obs_dtype, const int64_t* actions, const float* rewards,
                                const float* dones, int64_t E, int64_t D, int64_t* state,
                                int64_t size, void* rb_obs, int rb_dtype, int64_t* rb_actions,
                                float* rb_rewards, float* rb_dones, void* workspace) {
  OCPPO_REQUIRE(E >= 1 && D >= 1 && size >= 2, "ocppo_replay_add: bad sizes");
  OCPPO_REQUIRE(obs && next_obs && actions && rewards && dones && state && rb_obs && rb_actions &&
                    rb_rewards && rb_dones && workspace,
                "ocppo_replay_add: null pointer");
  OCPPO_REQUIRE((obs_dtype == OCPPO_F32 || obs_dtype == OCPPO_BF16 || obs_dtype == OCPPO_U8) &&
                    (rb_dtype == OCPPO_F32 || rb_dtype == OCPPO_BF16 || rb_dtype == OCPPO_U8),
                "ocppo_replay_add: bad dtypes");
  int64_t g = ceil_div(E * D, 256);
  g = g < 1024 ? g : 1024;
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  unsigned* ticket = static_cast<unsigned*>(workspace);
#define OCPPO_ADD(S, O)                                                                         \
  if (obs_dtype == S && rb_dtype == O) {                                                        \
    hipLaunchKernelGGL((replay_add_kernel<S, O>), dim3(g), dim3(256), 0, s, obs, next_obs,       \
                       actions, rewards, dones, E, D, state, size, rb_obs, rb_actions,          \
                       rb_rewards, rb_dones, ticket);                                           \
    return check_launch("ocppo_replay_add");                                                    \
  }
  OCPPO_ADD(OCPPO_F32, OCPPO_F32)
  OCPPO_ADD(OCPPO_F32, OCPPO_BF16)
  OCPPO_ADD(OCPPO_F32, OCPPO_U8)
  OCPPO_ADD(OCPPO_U8, OCPPO_F32)
  OCPPO_ADD(OCPPO_U8, OCPPO_BF16)
  OCPPO_ADD(OCPPO_U8, OCPPO_U8)
  OCPPO_ADD(OCPPO_BF16, OCPPO_F32)
  OCPPO_ADD(OCPPO_BF16, OCPPO_BF16)
  OCPPO_ADD(OCPPO_BF16, OCPPO_U8)
#undef OCPPO_ADD
  return fail(OCPPO_E_INVALID, "ocppo_replay_add: unsupported dtype pair");
}

extern "C" int ocppo_replay_sample(ocppo_stream_t stream, uint64_t seed, int64_t* counter,
                                   const int64_t* state, int64_t size, int64_t E, int64_t D,
                                   const void* rb_obs, int rb_dtype, const int64_t* rb_actions,
                                   const float* rb_rewards, const float* rb_dones, int64_t B,
                                   float* obs_out, float* next_obs_out, int64_t* actions_out,
                                   float* rewards_out, float* dones_out, int64_t* indices_out) {
  OCPPO_REQUIRE(E >= 1 && D >= 1 && size >= 2 && B >= 1, "ocppo_replay_sample: bad sizes");
  OCPPO_REQUIRE(counter && state && rb_obs && rb_actions && rb_rewards && rb_dones && obs_out &&
                    next_obs_out && actions_out && rewards_out && dones_out,
                "ocppo_replay_sample: null pointer");
  int64_t g = ceil_div(B * D, 256);
  g = g < 4096 ? g : 4096;
  clear_stale_error();
  hipStream_t s = as_stream(stream);
#define OCPPO_SMP(O)                                                                              \
  hipLaunchKernelGGL(replay_sample_kernel<O>, dim3(g), dim3(256), 0, s, seed, counter, state,      \
                     size, E, D, rb_obs, rb_actions, rb_rewards, rb_dones, B, obs_out,             \
                     next_obs_out, actions_out, rewards_out, dones_out, indices_out)
  if (rb_dtype == OCPPO_F32)
    OCPPO_SMP(OCPPO_F32);
  else if (rb_dtype == OCPPO_BF16)
    OCPPO_SMP(OCPPO_BF16);
  else if (rb_dtype == OCPPO_U8)
    OCPPO_SMP(OCPPO_U8);
  else
    return fail(OCPPO_E_INVALID, "ocppo_replay_sample: bad dtype %d", rb_dtype);
#undef OCPPO_SMP
  if (int rc = check_launch("ocppo_replay_sample")) return rc;
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, s, counter, int64_t(1));
  return check_launch("ocppo_replay_sample/counter");
}

extern "C" int ocppo_td_loss_fwd_bwd(ocppo_stream_t stream, const float* q, const float* q_next,
                                     const int64_t* actions, const float* rewards,
                                     const float* dones, int64_t B, int64_t A, double gamma,
                                     float* dq, float* stats) {
  OCPPO_REQUIRE(B >= 1 && A >= 1 && A <= 1024, "ocppo_td_loss_fwd_bwd: bad sizes");
  OCPPO_REQUIRE(q && q_next && actions && rewards && dones && dq && stats,
                "ocppo_td_loss_fwd_bwd: null pointer");
  clear_stale_error();
  // mse_loss backward: norm = 2 / numel (computed in double by ATen, applied in f32)
  const float norm = static_cast<float>(2.0 / static_cast<double>(B));
  hipLaunchKernelGGL(td_loss_kernel, dim3(1), dim3(256), 0, as_stream(stream), q, q_next, actions,
                     rewards, dones, B, (int)A, static_cast<float>(gamma), norm, dq, stats);
  return check_launch("ocppo_td_loss_fwd_bwd");
}

extern "C" int ocppo_epsilon_greedy(ocppo_stream_t stream, const float* q, int64_t E, int64_t A,
                                    uint64_t seed, const int64_t* step, int64_t step_offset,
                                    double start_e, double end_e, double duration,
                                    int64_t* actions, float* epsilon_out) {
  OCPPO_REQUIRE(E >= 1 && A >= 1 && A <= INT32_MAX && duration > 0,
                "ocppo_epsilon_greedy: bad sizes");
  OCPPO_REQUIRE(q && step && actions, "ocppo_epsilon_greedy: null pointer");
  clear_stale_error();
  int64_t g = ceil_div(E, 256);
  g = g < 1024 ? g : 1024;
  hipLaunchKernelGGL(epsilon_greedy_kernel, dim3(g), dim3(256), 0, as_stream(stream), q, E, (int)A,
                     seed, step, step_offset, start_e, end_e, duration, actions, epsilon_out);
  return check_launch("ocppo_epsilon_greedy");
}

extern "C" int ocppo_q_head_epsilon_greedy(ocppo_stream_t stream, const float* hidden, int64_t E,
                                          int64_t H, const float* wq, const float* bq, int64_t A,
                                          uint64_t seed, const int64_t* step, int64_t step_offset,
                                          double start_e, double end_e, double duration,
                                          int64_t* actions, float* epsilon_out, float* q_out) {
  OCPPO_REQUIRE(E >= 1 && A >= 1 && A <= 8 && H >= 256 && H % 256 == 0 && H <= 1024 &&
                    duration > 0 && E <= INT32_MAX,
                "ocppo_q_head_epsilon_greedy: bad sizes E=%lld H=%lld A=%lld (A <= 8, H a "
                "multiple of 256 <= 1024)", (long long)E, (long long)H, (long long)A);
  OCPPO_REQUIRE(hidden && wq && bq && step && actions, "ocppo_q_head_epsilon_greedy: null pointer");
  OCPPO_REQUIRE(((reinterpret_cast<uintptr_t>(hidden) | reinterpret_cast<uintptr_t>(wq)) & 15) == 0,
                "ocppo_q_head_epsilon_greedy: hidden and wq must be 16-B aligned");
  clear_stale_error();
  const dim3 grid(static_cast<unsigned>(ceil_div(E, 4))), block(256);
  hipStream_t s = as_stream(stream);
#define OCPPO_QH(CH)                                                                            \
  hipLaunchKernelGGL(q_head_eps_kernel<CH>, grid, block, 0, s, hidden, E, wq, bq, (int)A, seed, \
                     step, step_offset, start_e, end_e, duration, actions, epsilon_out, q_out)
  switch (H / 256) {
    case 1: OCPPO_QH(1); break;
    case 2: OCPPO_QH(2); break;
    case 3: OCPPO_QH(3); break;
    default: OCPPO_QH(4); break;
  }
#undef OCPPO_QH
  return check_launch("ocppo_q_head_epsilon_greedy");
}
