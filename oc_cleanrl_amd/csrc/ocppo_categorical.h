// Categorical(logits) row statistics and the sampling tail shared by the policy-head kernels
// (ocppo_loss.hip: the rollout action head; ocppo_linear.hip: the decoder + head launch), in
// torch's op order so sampled actions stay bit-identical to torch's sampler on the same logits
// (torch/distributions/categorical.py, architectures/ppo.py:89-95).
#pragma once

#include <cfloat>

#include "ocppo_common.h"

namespace ocppo {

// Row statistics of Categorical(logits=l): lse, normalised logits ln = l - lse, probs = softmax(ln)
// (torch/distributions/categorical.py: logits - logits.logsumexp(-1), then logits_to_probs).
template <int AMAX>
__device__ __forceinline__ void categorical_row(const float (&l)[AMAX], int A, float& lse,
                                                float (&ln)[AMAX], float (&p)[AMAX]) {
  float m = l[0];
#pragma unroll
  for (int j = 1; j < AMAX; ++j)
    if (j < A) m = fmaxf(m, l[j]);
  const float mm = (fabsf(m) == INFINITY) ? 0.f : m;  // ATen masks infinite maxima
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) s += expf(l[j] - m);
  lse = logf(s) + mm;
  float m2 = -INFINITY;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) {
      ln[j] = l[j] - lse;
      m2 = fmaxf(m2, ln[j]);
    }
  float s2 = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) {
      p[j] = expf(ln[j] - m2);
      s2 += p[j];
    }
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) p[j] = p[j] / s2;
}

// entropy = -(clamp(ln, min=lowest) * p).sum(-1)   (Categorical.entropy)
template <int AMAX>
__device__ __forceinline__ float categorical_entropy(const float (&ln)[AMAX],
                                                     const float (&p)[AMAX], int A) {
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) acc += fmaxf(ln[j], -FLT_MAX) * p[j];
  return -acc;
}

// Categorical tail for one environment given its A logits (l[7] = value) and Exp(1) noise:
// writes action, log-prob, value, entropy, logits.
__device__ __forceinline__ void head_tail(const float (&l)[8], const float (&nzj)[7], int A,
                                          int64_t n, int64_t* __restrict__ action_out,
                                          float* __restrict__ logprob_out,
                                          float* __restrict__ entropy_out,
                                          float* __restrict__ value_out,
                                          float* __restrict__ logits_out, bool store) {
  float ln[8], p[8], lse;
  categorical_row<8>(l, A, lse, ln, p);
  int best = 0;
  float best_q = p[0] / nzj[0];
#pragma unroll
  for (int j = 1; j < 7; ++j)
    if (j < A) {
      const float q = p[j] / nzj[j];
      if (q > best_q || (q != q && best_q == best_q)) {
        best_q = q;
        best = j;
      }
    }
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < 7; ++j)
    if (j == best) lp = ln[j];
  if (!store) return;
  action_out[n] = best;
  logprob_out[n] = lp;
  value_out[n] = l[7];
  if (entropy_out) entropy_out[n] = categorical_entropy<8>(ln, p, A);
  if (logits_out) {
#pragma unroll
    for (int j = 0; j < 7; ++j)
      if (j < A) logits_out[n * A + j] = l[j];
  }
}

}  // namespace ocppo
