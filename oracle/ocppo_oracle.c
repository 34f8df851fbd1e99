/* ORACLE — plain-C restatement of the reference GAE loop (TEST INFRASTRUCTURE ONLY).
 *
 * cleanrl/ppo_atari_oc.py:533-547 in f32, op by op, compiled with -ffp-contract=off so every
 * product and sum is rounded like PyTorch's separate ATen kernels. Pinned bit-for-bit to
 * tests/golden/gae_*.npz by tests/test_oracle_c.py; used as an independent second restatement
 * next to oracle/ocppo_oracle.py. Never linked into the product library. */
#include <stdint.h>

void oracle_gae(const float* rewards, const float* values, const float* dones,
                const float* next_value, const float* next_done, int64_t T, int64_t N,
                double gamma, double gae_lambda, float* adv, float* ret) {
  const float g = (float)gamma;                /* `args.gamma * tensor`                     */
  const float gl = (float)(gamma * gae_lambda); /* `args.gamma * args.gae_lambda * tensor`   */
  for (int64_t n = 0; n < N; ++n) {
    float last = 0.0f;
    for (int64_t t = T - 1; t >= 0; --t) {
      const float nnt = 1.0f - (t == T - 1 ? next_done[n] : dones[(t + 1) * N + n]);
      const float nv = t == T - 1 ? next_value[n] : values[(t + 1) * N + n];
      float delta = rewards[t * N + n] + (g * nv) * nnt;
      delta = delta - values[t * N + n];
      last = delta + (gl * nnt) * last;
      adv[t * N + n] = last;
      ret[t * N + n] = last + values[t * N + n];
    }
  }
}
