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
__device__ __forceinline__ int head_tail(const float (&l)[8], const float (&nzj)[7], int A,
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
  if (!store) return best;
  action_out[n] = best;
  logprob_out[n] = lp;
  value_out[n] = l[7];
  if (entropy_out) entropy_out[n] = categorical_entropy<8>(ln, p, A);
  if (logits_out) {
#pragma unroll
    for (int j = 0; j < 7; ++j)
      if (j < A) logits_out[n * A + j] = l[j];
  }
  return best;
}

// The policy head's row access for H = 256*CH (lane = float4 columns c*64 + lane of the row) and
// its A+1 (padded to 8) dot products against register-resident weight rows, reduce-scattered so
// that lane 8j ends with value j.
template <int CH>
__device__ __forceinline__ void head_load_row(const float* __restrict__ hidden, int64_t n, int lane,
                                              float4 (&x)[CH]) {
  const float4* h4 = reinterpret_cast<const float4*>(hidden + n * (256 * CH));
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = h4[c * kWave + lane];
}

// The A+1 (padded to 8) dot products of one hidden row against the register-resident weights,
// reduce-scattered so that lane 8j ends with value j (see above).
template <int CH>
__device__ __forceinline__ float head_dots(const float4 (&x)[CH], const float4 (&w)[8][CH],
                                           int lane) {
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    acc[j] = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
      acc[j] += x[c].x * w[j][c].x + x[c].y * w[j][c].y + x[c].z * w[j][c].z + x[c].w * w[j][c].w;
  }
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
  float s4[4], s2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float send = b5 ? acc[i] : acc[i + 4];
    s4[i] = (b5 ? acc[i + 4] : acc[i]) + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = b4 ? s4[i] : s4[i + 2];
    s2[i] = (b4 ? s4[i + 2] : s4[i]) + __shfl_xor(send, 16);
  }
  float t = (b3 ? s2[1] : s2[0]) + __shfl_xor(b3 ? s2[0] : s2[1], 8);
  t += __shfl_xor(t, 4);
  t += __shfl_xor(t, 2);
  t += __shfl_xor(t, 1);
  return t;
}

}  // namespace ocppo
