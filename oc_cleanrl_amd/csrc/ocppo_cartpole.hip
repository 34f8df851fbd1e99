// CartPole-v1 as a device-resident vector env: config 1 (cleanrl/ppo.py:162 builds
// gym.vector.SyncVectorEnv over gym.make("CartPole-v1") + RecordEpisodeStatistics, :81-91).
//
// Dynamics restate gymnasium 0.28.1 (the reference's pin, poetry.lock:1265-1266)
// classic_control/cartpole.py: Euler integration in f64 with the published constants and the
// same operation order, termination at |x| > 2.4 or |theta| > 12 degrees, reward 1.0 per step,
// TimeLimit(max_episode_steps=500) truncation, SyncVectorEnv's same-step auto-reset (the returned
// obs of a done env is its reset obs), obs = float32(state). The reset draw is
// uniform(-0.05, 0.05)^4 from a counter-based stream (seed, env, episode) instead of numpy's
// PCG64, so trajectories are not numpy's (parity of the dynamics is against the oracle's
// restatement; gymnasium itself is not installed).
//
// One thread per env; the state stays in HBM between launches, so a captured rollout graph
// replays it step after step.
#include "ocppo_common.h"

namespace ocppo {

namespace cartpole {
constexpr double kGravity = 9.8;
constexpr double kMassCart = 1.0;
constexpr double kMassPole = 0.1;
constexpr double kTotalMass = kMassPole + kMassCart;
constexpr double kLength = 0.5;
constexpr double kPoleMassLength = kMassPole * kLength;
constexpr double kForceMag = 10.0;
constexpr double kTau = 0.02;
constexpr double kXThreshold = 2.4;
constexpr int64_t kMaxSteps = 500;
}  // namespace cartpole

__device__ __forceinline__ uint64_t cp_mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform(-0.05, 0.05) as numpy computes low + (high - low) * u, u a 53-bit double in [0, 1)
__device__ __forceinline__ void cartpole_reset_state(uint64_t seed, int64_t n, int64_t episode,
                                                     double* st) {
  const uint64_t key = cp_mix(cp_mix(seed) + static_cast<uint64_t>(n) * 0x100000001B3ull) ^
                       cp_mix(static_cast<uint64_t>(episode) + 0x632BE59BD9B4E019ull);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t h = cp_mix(key + static_cast<uint64_t>(i));
    const double u = static_cast<double>(h >> 11) * (1.0 / 9007199254740992.0);
    st[i] = -0.05 + (0.05 - -0.05) * u;
  }
}

__global__ __launch_bounds__(256) void cartpole_step_kernel(
    uint64_t seed, const int64_t* __restrict__ actions, int64_t N, double* __restrict__ state,
    int64_t* __restrict__ counters, float* __restrict__ obs, float* __restrict__ reward_out,
    float* __restrict__ done_out, float* __restrict__ ep) {
  using namespace cartpole;
  const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double st[4] = {state[4 * n], state[4 * n + 1], state[4 * n + 2], state[4 * n + 3]};
  int64_t elapsed = counters[2 * n];
  const int64_t episode = counters[2 * n + 1];
  if (actions == nullptr) {  // env.reset(): every env starts episode `episode`
    cartpole_reset_state(seed, n, episode, st);
    counters[2 * n] = 0;
    counters[2 * n + 1] = episode + 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      state[4 * n + i] = st[i];
      obs[4 * n + i] = static_cast<float>(st[i]);
    }
    if (reward_out) reward_out[n] = 0.f;
    if (done_out) done_out[n] = 0.f;
    return;
  }
  // cartpole.py step(), Euler branch; Python evaluates left to right, no FMA (-ffp-contract=off)
  const double x = st[0], x_dot = st[1], theta = st[2], theta_dot = st[3];
  const double force = actions[n] == 1 ? kForceMag : -kForceMag;
  const double costheta = cos(theta);
  const double sintheta = sin(theta);
  const double temp = (force + kPoleMassLength * (theta_dot * theta_dot) * sintheta) / kTotalMass;
  const double thetaacc =
      (kGravity * sintheta - costheta * temp) /
      (kLength * (4.0 / 3.0 - kMassPole * (costheta * costheta) / kTotalMass));
  const double xacc = temp - kPoleMassLength * thetaacc * costheta / kTotalMass;
  st[0] = x + kTau * x_dot;
  st[1] = x_dot + kTau * xacc;
  st[2] = theta + kTau * theta_dot;
  st[3] = theta_dot + kTau * thetaacc;
  const double theta_thr = 12.0 * 2.0 * 3.141592653589793 / 360.0;
  const bool terminated = st[0] < -kXThreshold || st[0] > kXThreshold || st[2] < -theta_thr ||
                          st[2] > theta_thr;
  elapsed += 1;
  const bool truncated = elapsed >= kMaxSteps;  // TimeLimit(500)
  const bool done = terminated || truncated;
  const float r = 1.0f;  // also on the terminating step (steps_beyond_terminated is None)
  if (ep) {  // RecordEpisodeStatistics: return / length of the episode that just ended
    float* e = ep + n * 5;
    const float run_ret = e[0] + r, run_len = e[1] + 1.f;
    if (done) {
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
  if (done) {  // SyncVectorEnv auto-reset in the same step (gymnasium 0.28)
    cartpole_reset_state(seed, n, episode, st);
    elapsed = 0;
    counters[2 * n + 1] = episode + 1;
  }
  counters[2 * n] = elapsed;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    state[4 * n + i] = st[i];
    obs[4 * n + i] = static_cast<float>(st[i]);
  }
  reward_out[n] = r;
  done_out[n] = done ? 1.f : 0.f;
}

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_cartpole_step(ocppo_stream_t stream, uint64_t seed, const int64_t* actions,
                                   int64_t N, double* state, int64_t* counters, float* obs_out,
                                   float* reward_out, float* done_out, float* ep_state) {
  OCPPO_REQUIRE(N >= 0, "ocppo_cartpole_step: bad size N=%lld", (long long)N);
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(state && counters && obs_out, "ocppo_cartpole_step: null pointer");
  OCPPO_REQUIRE(actions == nullptr || (reward_out && done_out),
                "ocppo_cartpole_step: a step needs reward_out and done_out");
  clear_stale_error();
  hipLaunchKernelGGL(cartpole_step_kernel, dim3(grid_for(N, 256)), dim3(256), 0,
                     as_stream(stream), seed, actions, N, state, counters, obs_out, reward_out,
                     done_out, ep_state);
  return check_launch("ocppo_cartpole_step");
}
