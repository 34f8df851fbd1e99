// Fused PPO minibatch loss (forward + backward), minibatch advantage statistics and the
// Categorical action head.
//
// Replaces, from the network's raw outputs onward, cleanrl/ppo_atari_oc.py:566-602 (ratio, KL
// stats, clipfrac, advantage normalisation, clipped surrogate, clipped value loss, entropy bonus)
// and torch.distributions.Categorical as used by architectures/ppo.py:89-95, plus the autograd
// backward of all of it down to d loss / d logits and d loss / d value.
//
// Every per-element quantity is computed in f32 in PyTorch's op order (no contraction), and the
// backward follows autograd's formulas: max() splits the gradient 1/2-1/2 on ties, clamp() passes
// it at the bounds, softmax/logsumexp backward as in ATen. Reductions use a fixed order (per-thread
// strided sums, wave butterfly, waves in order, blocks in order), so results are run-to-run
// bit-identical; they differ from ATen's own reduction trees only in the last bits.
//
// Roofline of the loss kernel: HBM/latency bound, (8A + 36) algorithmic bytes per element
// (logits 4A + value 4 + index 8 + action 8 + old logprob/adv/return/value 16 in; dlogits 4A + dv 4
// out). At the configs (M = 4096) one launch moves 344 KB and is launch/latency bound.
#include <cfloat>
#include <cstdlib>
#include <cstring>

#include "ocppo_common.h"
#include "ocppo_categorical.h"
#include "ocppo_philox.h"
#include "ocppo_synth_env.h"

namespace ocppo {

constexpr int kLossThreads = 256;  // one element per thread, 256-element tiles
constexpr int kLossMaxBlocks = 1792;  // grid cap: 7 workgroups per CU (the A <= 6 kernels' occupancy)
constexpr int kNumPartials = 6;    // pg, v, entropy, old_kl, kl, clipfrac
constexpr size_t kTicketBytes = kHandoffTicketBytes;

// Backward of (log_prob(a), entropy()) w.r.t. the raw logits, for upstream grads g_lp and g_h.
template <int AMAX>
__device__ __forceinline__ void categorical_backward(const float (&l)[AMAX], float lse,
                                                     const float (&ln)[AMAX],
                                                     const float (&p)[AMAX], int A, int64_t a,
                                                     float g_lp, float g_h, float (&dl)[AMAX]) {
  const float dplp = -g_h;  // entropy = -sum(p_log_p)
  float dot = 0.f;          // softmax backward: sum_k dprobs_k * p_k, dprobs_k = dplp * ln_k
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) dot += (dplp * ln[j]) * p[j];
  float S = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) {
      const float dprob = dplp * ln[j];
      float d = dplp * p[j];               // through the clamped normalised logits
      d = d + p[j] * (dprob - dot);        // through probs = softmax(ln)
      if (j == a) d = d + g_lp;            // through log_prob's gather
      dl[j] = d;
      S += d;
    }
#pragma unroll
  for (int j = 0; j < AMAX; ++j)  // ln = l - logsumexp(l)
    if (j < A) dl[j] = dl[j] - S * expf(l[j] - lse);
}

// Loss-kernel form of the row statistics: lse (hence ln = l - lse and the log-prob) exactly as
// above, but the probabilities reuse the logsumexp pass, p = exp(l - m) * (1 / s), instead of a
// second softmax over ln: mathematically the same softmax (torch evaluates it as
// softmax(l - lse)), here within an ulp or two of it, for A exps instead of 2A and one division.
// Only the loss uses it (checked to 1e-6 of scale against the reference's autograd fixtures); the
// sampler keeps categorical_row so sampled actions stay bit-identical to torch's.
template <int AMAX>
__device__ __forceinline__ void categorical_row_loss(const float (&l)[AMAX], int A, float& lse,
                                                     float (&ln)[AMAX], float (&p)[AMAX]) {
  float m = l[0];
#pragma unroll
  for (int j = 1; j < AMAX; ++j)
    if (j < A) m = fmaxf(m, l[j]);
  const float mm = (fabsf(m) == INFINITY) ? 0.f : m;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) {
      p[j] = expf(l[j] - m);
      s += p[j];
    }
  lse = logf(s) + mm;
  const float rs = 1.0f / s;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) {
      ln[j] = l[j] - lse;
      p[j] = p[j] * rs;
    }
}

// categorical_backward with exp(l - lse) (logsumexp's backward) taken as the row's p.
template <int AMAX>
__device__ __forceinline__ void categorical_backward_loss(const float (&ln)[AMAX],
                                                          const float (&p)[AMAX], int A,
                                                          int64_t a, float g_lp, float g_h,
                                                          float (&dl)[AMAX]) {
  const float dplp = -g_h;
  float dot = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) dot += (dplp * ln[j]) * p[j];
  float S = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) {
      const float dprob = dplp * ln[j];
      float d = dplp * p[j];
      d = d + p[j] * (dprob - dot);
      if (j == a) d = d + g_lp;
      dl[j] = d;
      S += d;
    }
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) dl[j] = dl[j] - S * p[j];
}

// ---- minibatch advantage statistics ------------------------------------------------------------
// One 256-thread block per minibatch. Each thread first issues all of its index loads, then all
// of its gathered loads (VPT in flight instead of a dependent chain), keeps the values in
// registers, and runs the two passes (mean, then squared deviations) from there -- torch's
// mean() / std() (unbiased) of ppo_atari_oc.py:579 in f32. The same block body serves
// ocppo_minibatch_adv_stats and the statistics blocks of ocppo_minibatch_prepare, so the two
// give bitwise-identical figures.
constexpr int kStatsThreads = 256;
// STRIDE: floats between consecutive samples' advantages (1: the b_adv array;
// field of the 16-B sample records of ocppo_gae_records: 4)
template <int VPT, int STRIDE = 1>
__device__ __forceinline__ void adv_stats_block(const float* __restrict__ adv,
                                                const int64_t* __restrict__ perm, int64_t M,
                                                int64_t mb, float* __restrict__ out,
                                                float* scratch) {
  const int64_t base = mb * M;
  int64_t idx[VPT];
  float x[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t i = threadIdx.x + static_cast<int64_t>(k) * kStatsThreads;
    idx[k] = i < M ? (perm ? perm[base + i] : base + i) : -1;
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) x[k] = idx[k] >= 0 ? adv[idx[k] * STRIDE] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k) s += x[k];
  s = block_sum(s, scratch);
  const float mean = s / static_cast<float>(M);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < VPT; ++k)
    if (idx[k] >= 0) {
      const float d = x[k] - mean;
      q += d * d;
    }
  q = block_sum(q, scratch);
  if (threadIdx.x == 0) {
    out[2 * mb + 0] = mean;
    out[2 * mb + 1] = sqrtf(q / static_cast<float>(M - 1));  // unbiased, torch.std()
  }
}

// Any M: strided loops, values re-gathered for the second pass.
template <int STRIDE = 1>
__device__ __forceinline__ void adv_stats_block_any(const float* __restrict__ adv,
                                                    const int64_t* __restrict__ perm, int64_t M,
                                                    int64_t mb, float* __restrict__ out,
                                                    float* scratch) {
  const int64_t base = mb * M;
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < M; i += kStatsThreads)
    s += adv[(perm ? perm[base + i] : base + i) * STRIDE];
  s = block_sum(s, scratch);
  const float mean = s / static_cast<float>(M);
  float q = 0.f;
  for (int64_t i = threadIdx.x; i < M; i += kStatsThreads) {
    const float d = adv[(perm ? perm[base + i] : base + i) * STRIDE] - mean;
    q += d * d;
  }
  q = block_sum(q, scratch);
  if (threadIdx.x == 0) {
    out[2 * mb + 0] = mean;
    out[2 * mb + 1] = sqrtf(q / static_cast<float>(M - 1));
  }
}

// VPT = 0: the strided form
template <int VPT, int STRIDE = 1>
__device__ __forceinline__ void adv_stats_any_vpt(const float* adv, const int64_t* perm,
                                                  int64_t M, int64_t mb, float* out,
                                                  float* scratch) {
  if constexpr (VPT == 0)
    adv_stats_block_any<STRIDE>(adv, perm, M, mb, out, scratch);
  else
    adv_stats_block<VPT, STRIDE>(adv, perm, M, mb, out, scratch);
}

inline int adv_stats_vpt(int64_t M) {
  return M <= kStatsThreads ? 1 : M <= 4 * kStatsThreads ? 4 : M <= 16 * kStatsThreads ? 16
       : M <= 64 * kStatsThreads ? 64 : 0;
}

template <int VPT>
__global__ __launch_bounds__(kStatsThreads) void adv_stats_kernel(const float* __restrict__ adv,
                                                                  const int64_t* __restrict__ perm,
                                                                  int64_t M, float* __restrict__ out) {
  __shared__ float scratch[kStatsThreads / kWave];
  adv_stats_any_vpt<VPT>(adv, perm, M, blockIdx.x, out, scratch);
}

static void launch_adv_stats(hipStream_t s, const float* adv, const int64_t* perm, int64_t M,
                             int64_t num_mb, float* out) {
  const dim3 grid(static_cast<unsigned>(num_mb)), block(kStatsThreads);
  switch (adv_stats_vpt(M)) {
    case 1: hipLaunchKernelGGL(adv_stats_kernel<1>, grid, block, 0, s, adv, perm, M, out); break;
    case 4: hipLaunchKernelGGL(adv_stats_kernel<4>, grid, block, 0, s, adv, perm, M, out); break;
    case 16: hipLaunchKernelGGL(adv_stats_kernel<16>, grid, block, 0, s, adv, perm, M, out); break;
    case 64: hipLaunchKernelGGL(adv_stats_kernel<64>, grid, block, 0, s, adv, perm, M, out); break;
    default: hipLaunchKernelGGL(adv_stats_kernel<0>, grid, block, 0, s, adv, perm, M, out); break;
  }
}

// Minibatch prepare: the per-sample records of every minibatch gathered into minibatch order
// (SoA), so that each loss launch reads contiguous arrays (no index, no scattered 4-8 B loads),
// AND each minibatch's advantage statistics, in ONE launch: num_mb statistics blocks, each running
// adv_stats_block for one minibatch (its own gathers of b_adv through perm: the figures of
// ocppo_minibatch_adv_stats, bit for bit), then gather_blocks blocks running a plain elementwise
// gather over the flat num_mb * M index space (VPT elements per thread, all index loads, then
// all gathers, then all stores in flight).
template <int VPT, int SVPT>
__global__ __launch_bounds__(256) void minibatch_prepare_kernel(
    const int64_t* __restrict__ perm, int64_t n, int gather_blocks, int64_t M,
    const int64_t* __restrict__ b_act, const float* __restrict__ b_lp,
    const float* __restrict__ b_adv, const float* __restrict__ b_ret,
    const float* __restrict__ b_val, int64_t* __restrict__ mb_act, float* __restrict__ mb_lp,
    float* __restrict__ mb_adv, float* __restrict__ mb_ret, float* __restrict__ mb_val,
    float* __restrict__ stats) {
  // the statistics blocks come first (they gather a whole minibatch each: started early, they
  // overlap the elementwise gather blocks behind them)
  const int nstat = stats ? static_cast<int>(gridDim.x) - gather_blocks : 0;
  if (static_cast<int>(blockIdx.x) < nstat) {  // statistics block of minibatch blockIdx.x
    __shared__ float scratch[kStatsThreads / kWave];
    adv_stats_any_vpt<SVPT>(b_adv, perm, M, blockIdx.x, stats, scratch);
    return;
  }
  const int64_t base = static_cast<int64_t>(blockIdx.x - nstat) * 256 * VPT + threadIdx.x;
  int64_t idx[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t i = base + k * 256;
    idx[k] = i < n ? perm[i] : -1;
  }
  int64_t a[VPT];
  float lp[VPT], ad[VPT], rt[VPT], vl[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t b = idx[k] >= 0 ? idx[k] : 0;
    a[k] = b_act[b];
    lp[k] = b_lp[b];
    ad[k] = b_adv[b];
    rt[k] = b_ret[b];
    vl[k] = b_val[b];
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t i = base + k * 256;
    if (idx[k] >= 0) {
      mb_act[i] = a[k];
      mb_lp[i] = lp[k];
      mb_adv[i] = ad[k];
      mb_ret[i] = rt[k];
      mb_val[i] = vl[k];
    }
  }
}

// The same from the 16-B sample records of ocppo_gae_records ({log-prob, advantage, value,
// action i32}): one 16-B gather per sample instead of five scattered 4-8 B ones; the return is
// advantage + value with GAE's own f32 add, so the statistics and the SoA outputs are bitwise
// those of minibatch_prepare_kernel.
template <int VPT, int SVPT>
__global__ __launch_bounds__(256) void minibatch_prepare_rec_kernel(
    const int64_t* __restrict__ perm, int64_t n, int gather_blocks, int64_t M,
    const float4* __restrict__ rec, int64_t* __restrict__ mb_act, float* __restrict__ mb_lp,
    float* __restrict__ mb_adv, float* __restrict__ mb_ret, float* __restrict__ mb_val,
    float* __restrict__ stats) {
  const int nstat = stats ? static_cast<int>(gridDim.x) - gather_blocks : 0;
  if (static_cast<int>(blockIdx.x) < nstat) {
    __shared__ float scratch[kStatsThreads / kWave];
    adv_stats_any_vpt<SVPT, 4>(reinterpret_cast<const float*>(rec) + 1, perm, M, blockIdx.x,
                               stats, scratch);
    return;
  }
  const int64_t base = static_cast<int64_t>(blockIdx.x - nstat) * 256 * VPT + threadIdx.x;
  int64_t idx[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t i = base + k * 256;
    idx[k] = i < n ? perm[i] : -1;
  }
  float4 r0[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) r0[k] = rec[idx[k] >= 0 ? idx[k] : 0];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int64_t i = base + k * 256;
    if (idx[k] >= 0) {
      mb_act[i] = __float_as_int(r0[k].w);
      mb_lp[i] = r0[k].x;
      mb_adv[i] = r0[k].y;
      mb_ret[i] = r0[k].y + r0[k].z;  // GAE's returns = advantages + values, the same f32 add
      mb_val[i] = r0[k].z;
    }
  }
}

// ---- fused loss ----------------------------------------------------------------------------------
struct LossParams {
  const float* logits;
  const float* new_value;
  const int64_t* mb_inds;
  const int64_t* b_actions;
  const float* b_logprobs;
  const float* b_adv;
  const float* b_ret;
  const float* b_val;
  const float* adv_stats;
  float* dlogits;
  float* dvalue;
  float* stats;
  unsigned* ticket;
  float* partials;   // [gridDim.x][kNumPartials]
  float* gpartials;  // [groups][kNumPartials]
  int64_t M;
  int A;
  int norm_adv, clip_vloss;
  float clip, clip_lo, clip_hi;  // f32(c), f32(1-c), f32(1+c)
  float ent_coef, vf_coef;
  float g_pg, g_h, g_v;  // upstream grads reaching mean(pg), mean(entropy), mean(v_loss_max)
  float inv_m;           // f32(1/M) for the reported means
};

template <int AMAX>
struct LossTileRegs {
  int64_t a;
  float old_lp, adv, R, v_old, v;
  float lg[AMAX];  // this thread's coalesced share of the tile's [cnt*A] logits
};

// Loads tile `tl`'s per-element records (element tid) and logits chunk into registers.
template <int AMAX>
__device__ __forceinline__ void loss_tile_load(const LossParams& P, int A, int64_t tl,
                                               int64_t ntiles, int tid, LossTileRegs<AMAX>& r) {
  r.a = 0;
  r.old_lp = r.adv = r.R = r.v_old = r.v = 0.f;
  if (tl >= ntiles) return;
  const int64_t i0 = tl * kLossThreads;
  const int64_t cnt = (P.M - i0) < kLossThreads ? (P.M - i0) : kLossThreads;
  if (tid < cnt) {
    const int64_t i = i0 + tid;
    const int64_t b = P.mb_inds ? P.mb_inds[i] : i;
    r.a = P.b_actions[b];
    r.old_lp = P.b_logprobs[b];
    r.adv = P.b_adv[b];
    r.R = P.b_ret[b];
    r.v_old = P.b_val[b];
    r.v = P.new_value[i];
  }
  const float* lrow = P.logits + i0 * A;
  const int n = static_cast<int>(cnt) * A;
#pragma unroll
  for (int k = 0; k < AMAX; ++k) {
    const int e = k * kLossThreads + tid;
    r.lg[k] = (k < A && e < n) ? lrow[e] : 0.f;
  }
}

// Block partials (fixed order) -> two-level hand-off -> the minibatch means in the last block.
__device__ __forceinline__ void loss_finish(const LossParams& P, const float (&part)[kNumPartials]) {
  __shared__ float red[kLossThreads / kWave][kNumPartials];
  __shared__ int s_last;
  const int tid = threadIdx.x;
  // per-block partial sums in a fixed order
  const int lane = tid & (kWave - 1), wid = tid / kWave;
#pragma unroll
  for (int k = 0; k < kNumPartials; ++k) {
    const float w = wave_sum(part[k]);
    if (lane == 0) red[wid][k] = w;
  }
  __syncthreads();
  float mine[kNumPartials], s[kNumPartials];
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < kNumPartials; ++k) {
      mine[k] = red[0][k];
      for (int w = 1; w < kLossThreads / kWave; ++w) mine[k] += red[w][k];
    }
  }
  if (!handoff_combine<kNumPartials>(mine, P.ticket, P.partials, P.gpartials, s, &s_last)) return;
  if (tid == 0) {
    const float pg_loss = s[0] * P.inv_m;
    const float v_loss = 0.5f * (s[1] * P.inv_m);
    const float ent = s[2] * P.inv_m;
    const float loss = (pg_loss - P.ent_coef * ent) + v_loss * P.vf_coef;
    P.stats[OCPPO_STAT_LOSS] = loss;
    P.stats[OCPPO_STAT_PG_LOSS] = pg_loss;
    P.stats[OCPPO_STAT_V_LOSS] = v_loss;
    P.stats[OCPPO_STAT_ENTROPY] = ent;
    P.stats[OCPPO_STAT_OLD_APPROX_KL] = s[3] * P.inv_m;
    P.stats[OCPPO_STAT_APPROX_KL] = s[4] * P.inv_m;
    P.stats[OCPPO_STAT_CLIPFRAC] = s[5] * P.inv_m;
    P.stats[OCPPO_STAT_ADV_MEAN] = P.norm_adv ? P.adv_stats[0] : 0.f;
    P.stats[OCPPO_STAT_ADV_STD] = P.norm_adv ? P.adv_stats[1] : 0.f;
  }
}

// One element of the fused loss: forward terms accumulated into part[], and the autograd
// backward of the minibatch loss to this row's logits (dl) and new value (dv).
// adv_mean / adv_den: the minibatch mean and std + 1e-8 (f32, as torch rounds them), read from
// P.adv_stats ONCE per thread by the caller: a load inside the element loop makes the compiler
// drain every outstanding (prefetch) load with it.
template <int AMAX>
__device__ __forceinline__ void loss_element(const LossParams& P, int A, const float (&l)[AMAX],
                                             int64_t a, float old_lp, float adv, float R,
                                             float v_old, float v, float adv_mean, float adv_den,
                                             float (&part)[kNumPartials], float (&dl)[AMAX],
                                             float& dv) {
#ifdef OCPPO_LOSS_PROBE  // bandwidth probe build (tools/): same traffic, trivial arithmetic
  dv = v + R + v_old + adv + old_lp;
  part[0] += dv;
#pragma unroll
  for (int j = 0; j < AMAX; ++j) dl[j] = l[j] + (j == a ? 1.f : 0.f);
  return;
#endif
  float ln[AMAX], p[AMAX];
  float lse;
  categorical_row_loss<AMAX>(l, A, lse, ln, p);
  float new_lp = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j == a) new_lp = ln[j];
  const float H = categorical_entropy<AMAX>(ln, p, A);

  // ratio and no-grad diagnostics (:569-575)
  const float logratio = new_lp - old_lp;
  const float ratio = expf(logratio);
  part[3] += -logratio;
  part[4] += (ratio - 1.0f) - logratio;
  part[5] += fabsf(ratio - 1.0f) > P.clip ? 1.f : 0.f;

  // advantage normalisation (:577-579)
  float advn = adv;
  if (P.norm_adv) advn = (adv - adv_mean) / adv_den;

  // clipped surrogate (:581-583)
  const float nadv = -advn;
  const float pg1 = nadv * ratio;
  const float rc = fminf(fmaxf(ratio, P.clip_lo), P.clip_hi);
  const float pg2 = nadv * rc;
  part[0] += fmaxf(pg1, pg2);

  // value loss (:585-597)
  const float du = v - R;
  const float vu = du * du;
  if (P.clip_vloss) {
    const float dvv = v - v_old;
    const float dvc = fminf(fmaxf(dvv, -P.clip), P.clip);
    const float vcl = v_old + dvc;
    const float dc = vcl - R;
    const float vc = dc * dc;
    part[1] += fmaxf(vu, vc);
    const float gu = vu > vc ? P.g_v : (vu == vc ? P.g_v / 2.f : 0.f);
    const float gc = vc > vu ? P.g_v : (vu == vc ? P.g_v / 2.f : 0.f);
    const float tu = gu * (2.0f * du);
    float tc = gc * (2.0f * dc);
    tc = (dvv >= -P.clip && dvv <= P.clip) ? tc : 0.f;
    dv = tu + tc;
  } else {
    part[1] += vu;
    dv = P.g_v * (2.0f * du);
  }
  part[2] += H;

  // backward of the surrogate to new_logprob
  const float g1 = pg1 > pg2 ? P.g_pg : (pg1 == pg2 ? P.g_pg / 2.f : 0.f);
  const float g2 = pg2 > pg1 ? P.g_pg : (pg1 == pg2 ? P.g_pg / 2.f : 0.f);
  const float dr1 = g1 * nadv;
  const float dr2 = (ratio >= P.clip_lo && ratio <= P.clip_hi) ? g2 * nadv : 0.f;
  const float dratio = dr1 + dr2;
  const float dnew_lp = dratio * ratio;  // exp backward, then logratio = new - old

  categorical_backward_loss<AMAX>(ln, p, A, a, dnew_lp, P.g_h, dl);
}

// AMAX = the compile-time row width; EXACT: A == AMAX (the Atari minimal action-set sizes are
// instantiated exactly, so the per-action loops carry no `j < A` guards), else A <= AMAX at run time.
template <int AMAX, bool EXACT>
__device__ __forceinline__ void ppo_loss_body(const LossParams& P) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [kLossThreads * A]

  const int A = EXACT ? AMAX : P.A;
  const int tid = threadIdx.x;
  float part[kNumPartials] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float adv_mean = P.norm_adv ? P.adv_stats[0] : 0.f;
  const float adv_den = P.norm_adv ? P.adv_stats[1] + 1e-8f : 1.f;
  const int64_t ntiles = (P.M + kLossThreads - 1) / kLossThreads;
  // grid-stride over 256-element tiles (the grid is capped at kLossMaxBlocks so the ticket
  // fan-in stays bounded); each thread accumulates its partials over its tiles in order.
  // Software-pipelined: the next tile's records and logits chunk are loaded into registers
  // before the current tile is computed.
  LossTileRegs<AMAX> nxt;
  loss_tile_load<AMAX>(P, A, blockIdx.x, ntiles, tid, nxt);
  for (int64_t tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
  const int64_t i0 = tl * kLossThreads;
  const int64_t cnt = (P.M - i0) < kLossThreads ? (P.M - i0) : kLossThreads;
  const bool active = tid < cnt;
  const int64_t i = i0 + tid;
  const LossTileRegs<AMAX> cur = nxt;
  const int64_t a = cur.a;
  const float old_lp = cur.old_lp, adv = cur.adv, R = cur.R, v_old = cur.v_old, v = cur.v;
  // stage this tile's logits rows (contiguous [cnt*A] floats, loaded coalesced) in LDS
  const int tile_n = static_cast<int>(cnt) * A;
#pragma unroll
  for (int k = 0; k < AMAX; ++k) {
    const int e = k * kLossThreads + tid;
    if (k < A && e < tile_n) tile[e] = cur.lg[k];
  }
  loss_tile_load<AMAX>(P, A, tl + gridDim.x, ntiles, tid, nxt);
  __syncthreads();

  float dl[AMAX];
  if (active) {
    float l[AMAX];
#pragma unroll
    for (int j = 0; j < AMAX; ++j) l[j] = j < A ? tile[tid * A + j] : 0.f;
    float dv;
    loss_element<AMAX>(P, A, l, a, old_lp, adv, R, v_old, v, adv_mean, adv_den, part, dl, dv);
    P.dvalue[i] = dv;
  }
  __syncthreads();  // everyone has read its logits row; reuse the tile for dlogits
  if (active) {
#pragma unroll
    for (int j = 0; j < AMAX; ++j)
      if (j < A) tile[tid * A + j] = dl[j];
  }
  __syncthreads();
  float* drow = P.dlogits + i0 * A;
  for (int e = tid; e < tile_n; e += kLossThreads) drow[e] = tile[e];
  __syncthreads();  // the next tile restages the LDS tile
  }

  loss_finish(P, part);
}

template <int AMAX, bool EXACT>
__global__ __launch_bounds__(kLossThreads) void ppo_loss_kernel(LossParams P) {
  ppo_loss_body<AMAX, EXACT>(P);
}

// Small exact action sets (A <= 6) fit 72 VGPRs without spilling: ask for 7 waves per SIMD (the
// grid cap, kLossMaxBlocks, is sized for it) instead of the 4 the hand-off's live ranges cost.
template <int AMAX>
__global__ __launch_bounds__(kLossThreads) __attribute__((amdgpu_waves_per_eu(7)))
void ppo_loss_kernel_small(LossParams P) {
  static_assert(AMAX <= 6, "register budget sized for A <= 6");
  ppo_loss_body<AMAX, true>(P);
}

// Streaming form for large minibatches with records already in minibatch order (mb_inds == NULL,
// as ocppo_minibatch_prepare leaves them): each thread owns kLossVec CONSECUTIVE elements, so
// every per-element array moves as one 16-B load or store per lane (actions: two), and the
// [kLossTile, A] logits / dlogits tiles pass through LDS as coalesced 16-B vectors (A per lane).
// 4x fewer tiles, barriers and load instructions per element than ppo_loss_kernel; the arithmetic
// per element is the same loss_element, so dlogits / dvalue are bit-identical to it. The tail tile
// (M % kLossTile elements) takes guarded scalar accesses.
constexpr int kLossVec = 4;
constexpr int kLossTile = kLossThreads * kLossVec;

// Registers of one full tile for one thread: kLossVec consecutive records + its A float4s of the
// tile's logits (coalesced: float4 k*256 + tid of the tile).
template <int A>
struct LossVecRegs {
  int64_t act[kLossVec];
  float olp[kLossVec], adv[kLossVec], ret[kLossVec], vold[kLossVec], vnew[kLossVec];
  float4 lg[A];
};

template <int A>
__device__ __forceinline__ void loss_vec_load(const LossParams& P, int64_t tl, int tid,
                                              LossVecRegs<A>& r) {
  const int64_t e0 = tl * kLossTile + static_cast<int64_t>(tid) * kLossVec;
  const longlong2 a01 = *reinterpret_cast<const longlong2*>(P.b_actions + e0);
  const longlong2 a23 = *reinterpret_cast<const longlong2*>(P.b_actions + e0 + 2);
  r.act[0] = a01.x; r.act[1] = a01.y; r.act[2] = a23.x; r.act[3] = a23.y;
  const float4 x0 = *reinterpret_cast<const float4*>(P.b_logprobs + e0);
  const float4 x1 = *reinterpret_cast<const float4*>(P.b_adv + e0);
  const float4 x2 = *reinterpret_cast<const float4*>(P.b_ret + e0);
  const float4 x3 = *reinterpret_cast<const float4*>(P.b_val + e0);
  const float4 x4 = *reinterpret_cast<const float4*>(P.new_value + e0);
  r.olp[0] = x0.x; r.olp[1] = x0.y; r.olp[2] = x0.z; r.olp[3] = x0.w;
  r.adv[0] = x1.x; r.adv[1] = x1.y; r.adv[2] = x1.z; r.adv[3] = x1.w;
  r.ret[0] = x2.x; r.ret[1] = x2.y; r.ret[2] = x2.z; r.ret[3] = x2.w;
  r.vold[0] = x3.x; r.vold[1] = x3.y; r.vold[2] = x3.z; r.vold[3] = x3.w;
  r.vnew[0] = x4.x; r.vnew[1] = x4.y; r.vnew[2] = x4.z; r.vnew[3] = x4.w;
  const float4* lsrc = reinterpret_cast<const float4*>(P.logits + tl * kLossTile * A);
#pragma unroll
  for (int k = 0; k < A; ++k) r.lg[k] = lsrc[k * kLossThreads + tid];
}

// Tile compute + write-back shared by the full and the tail tiles. `rec` holds the records of
// this thread's kLossVec rows; the tile's logits are in LDS.
template <int A, bool FULL>
__device__ __forceinline__ void loss_vec_tile(const LossParams& P, float* tile, int64_t i0,
                                              int64_t cnt, int tid, const LossVecRegs<A>& rec,
                                              float adv_mean, float adv_den,
                                              float (&part)[kNumPartials]) {
  const int64_t e0 = i0 + static_cast<int64_t>(tid) * kLossVec;
  float dl[kLossVec][A];
  float dv[kLossVec];
#pragma unroll
  for (int r = 0; r < kLossVec; ++r) {
    const int row = tid * kLossVec + r;
    if (FULL || row < cnt) {
      float l[A];
#pragma unroll
      for (int j = 0; j < A; ++j) l[j] = tile[row * A + j];
      loss_element<A>(P, A, l, rec.act[r], rec.olp[r], rec.adv[r], rec.ret[r], rec.vold[r],
                      rec.vnew[r], adv_mean, adv_den, part, dl[r], dv[r]);
    } else {
      dv[r] = 0.f;
#pragma unroll
      for (int j = 0; j < A; ++j) dl[r][j] = 0.f;
    }
  }
  __syncthreads();  // every row has been read: the tile takes dlogits
#pragma unroll
  for (int r = 0; r < kLossVec; ++r)
#pragma unroll
    for (int j = 0; j < A; ++j) tile[(tid * kLossVec + r) * A + j] = dl[r][j];
  __syncthreads();
  float* ddst = P.dlogits + i0 * A;
  if (FULL) {
    *reinterpret_cast<float4*>(P.dvalue + e0) = make_float4(dv[0], dv[1], dv[2], dv[3]);
#pragma unroll
    for (int k = 0; k < A; ++k)
      reinterpret_cast<float4*>(ddst)[k * kLossThreads + tid] =
          reinterpret_cast<const float4*>(tile)[k * kLossThreads + tid];
  } else {
#pragma unroll
    for (int r = 0; r < kLossVec; ++r)
      if (e0 + r < P.M) P.dvalue[e0 + r] = dv[r];
    const int n = static_cast<int>(cnt) * A;
    for (int e = tid; e < n; e += kLossThreads) ddst[e] = tile[e];
  }
}

// One tile per block up to the hand-off's 8192 blocks (M <= 8M elements); larger M walks tiles.
// No software pipelining: co-resident blocks (4 per CU) overlap each other's loads and
// arithmetic, while a loop carrying a prefetch across the tile's stores makes the compiler wait
// for those stores (vmcnt is in order) at every tile.
template <int A>
__global__ __launch_bounds__(kLossThreads) void ppo_loss_vec_kernel(LossParams P) {
  extern __shared__ __attribute__((aligned(16))) float tile[];  // [kLossTile * A]
  const int tid = threadIdx.x;
  float part[kNumPartials] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const float adv_mean = P.norm_adv ? P.adv_stats[0] : 0.f;
  const float adv_den = P.norm_adv ? P.adv_stats[1] + 1e-8f : 1.f;
  const int64_t ntiles = (P.M + kLossTile - 1) / kLossTile;
  LossVecRegs<A> rec;
  for (int64_t tl = blockIdx.x; tl < ntiles; tl += gridDim.x) {
    const int64_t i0 = tl * kLossTile;
    const int64_t cnt = (P.M - i0) < kLossTile ? (P.M - i0) : kLossTile;
    if (tl != blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    if (cnt == kLossTile) {
      loss_vec_load<A>(P, tl, tid, rec);
#pragma unroll
      for (int k = 0; k < A; ++k) reinterpret_cast<float4*>(tile)[k * kLossThreads + tid] = rec.lg[k];
      __syncthreads();
      loss_vec_tile<A, true>(P, tile, i0, cnt, tid, rec, adv_mean, adv_den, part);
    } else {  // the tail tile: guarded scalar accesses
      const int64_t e0 = i0 + static_cast<int64_t>(tid) * kLossVec;
#pragma unroll
      for (int r = 0; r < kLossVec; ++r) {
        const int64_t e = e0 + r;
        const bool ok = e < P.M;
        rec.act[r] = ok ? P.b_actions[e] : 0;
        rec.olp[r] = ok ? P.b_logprobs[e] : 0.f;
        rec.adv[r] = ok ? P.b_adv[e] : 0.f;
        rec.ret[r] = ok ? P.b_ret[e] : 0.f;
        rec.vold[r] = ok ? P.b_val[e] : 0.f;
        rec.vnew[r] = ok ? P.new_value[e] : 0.f;
      }
      const float* lsrc = P.logits + i0 * A;
      const int n = static_cast<int>(cnt) * A;
      for (int e = tid; e < n; e += kLossThreads) tile[e] = lsrc[e];
      __syncthreads();
      loss_vec_tile<A, false>(P, tile, i0, cnt, tid, rec, adv_mean, adv_den, part);
    }
  }
  loss_finish(P, part);
}

// ---- Categorical action head ---------------------------------------------------------------------
// The sampler's Exp(1) values: read from `in`, or -- pn.state set -- drawn here as torch's
// exponential_ would have drawn them (ocppo_philox.h) and, when `out` is set, written there.
struct NoiseSrc {
  const float* in;
  float* out;
  PhiloxNoise pn;
  __device__ __forceinline__ float get(int64_t i) const {
    if (pn.state == nullptr) return in[i];
    const float v = philox_noise(pn, i);
    if (out) out[i] = v;
    return v;
  }
};

template <int AMAX>
__global__ __launch_bounds__(256) void categorical_sample_kernel(
    const float* __restrict__ logits, NoiseSrc noise, int64_t N, int A,
    int64_t* __restrict__ action_out, float* __restrict__ logprob_out,
    float* __restrict__ entropy_out, const float* __restrict__ value_in,
    float* __restrict__ value_out) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float l[AMAX], ln[AMAX], p[AMAX];
#pragma unroll
  for (int j = 0; j < AMAX; ++j) l[j] = j < A ? logits[n * A + j] : 0.f;
  float lse;
  categorical_row<AMAX>(l, A, lse, ln, p);
  // torch.multinomial(probs, 1) fast path: argmax(probs / q), q ~ Exp(1); first index on ties
  int best = 0;
  float best_q = p[0] / noise.get(n * A);
#pragma unroll
  for (int j = 1; j < AMAX; ++j)
    if (j < A) {
      const float q = p[j] / noise.get(n * A + j);
      if (q > best_q || (q != q && best_q == best_q)) {  // argmax propagates NaN like ATen
        best_q = q;
        best = j;
      }
    }
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j == best) lp = ln[j];
  action_out[n] = best;
  logprob_out[n] = lp;
  if (entropy_out) entropy_out[n] = categorical_entropy<AMAX>(ln, p, A);
  if (value_in && value_out) value_out[n] = value_in[n];
}

template <int AMAX>
__global__ __launch_bounds__(256) void categorical_lp_ent_kernel(
    const float* __restrict__ logits, const int64_t* __restrict__ actions, int64_t N, int A,
    float* __restrict__ logprob_out, float* __restrict__ entropy_out) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float l[AMAX], ln[AMAX], p[AMAX];
#pragma unroll
  for (int j = 0; j < AMAX; ++j) l[j] = j < A ? logits[n * A + j] : 0.f;
  float lse;
  categorical_row<AMAX>(l, A, lse, ln, p);
  const int64_t a = actions[n];
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j == a) lp = ln[j];
  if (logprob_out) logprob_out[n] = lp;
  if (entropy_out) entropy_out[n] = categorical_entropy<AMAX>(ln, p, A);
}

template <int AMAX>
__global__ __launch_bounds__(256) void categorical_lp_ent_bwd_kernel(
    const float* __restrict__ logits, const int64_t* __restrict__ actions,
    const float* __restrict__ g_lp, const float* __restrict__ g_h, int64_t N, int A,
    float* __restrict__ dlogits) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float l[AMAX], ln[AMAX], p[AMAX], dl[AMAX];
#pragma unroll
  for (int j = 0; j < AMAX; ++j) l[j] = j < A ? logits[n * A + j] : 0.f;
  float lse;
  categorical_row<AMAX>(l, A, lse, ln, p);
  categorical_backward<AMAX>(l, lse, ln, p, A, actions[n], g_lp ? g_lp[n] : 0.f,
                             g_h ? g_h[n] : 0.f, dl);
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j < A) dlogits[n * A + j] = dl[j];
}

constexpr int kMaxActions = 32;

// ---- fused rollout policy head ---------------------------------------------------------------------
// logits = hidden @ W_actor^T + b_actor, value = hidden @ w_critic + b_critic, then the Categorical
// sample of categorical_sample_kernel. One wave per env: lane l owns hidden[4l + 256k .. +3]
// (16-B loads, 1 KiB per wave instruction) and the same slice of the A+1 weight rows (L2-resident,
// shared by every wave), accumulates A+1 partial dots, and a butterfly reduces them (fixed order).
// Replaces the actor and critic Linear launches + the sampler of architectures/ppo.py:89-95 for a
// rollout step (the GEMMs have only A+1 = 7 output columns).
template <int AMAX>
__global__ __launch_bounds__(256) void policy_head_sample_kernel(
    const float* __restrict__ hidden, int64_t N, int H, const float* __restrict__ wa,
    const float* __restrict__ ba, const float* __restrict__ wc, const float* __restrict__ bc,
    NoiseSrc noise, int A, int64_t* __restrict__ action_out,
    float* __restrict__ logprob_out, float* __restrict__ entropy_out,
    float* __restrict__ value_out, float* __restrict__ logits_out) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t n = static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (n >= N) return;  // wave-uniform
  const float* h = hidden + n * H;
  float acc[AMAX + 1];
#pragma unroll
  for (int j = 0; j <= AMAX; ++j) acc[j] = 0.f;
  if ((H & 3) == 0) {
    for (int k = 4 * lane; k < H; k += 4 * kWave) {
      const float4 x = *reinterpret_cast<const float4*>(h + k);
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) {
          const float4 w = *reinterpret_cast<const float4*>(wa + static_cast<int64_t>(j) * H + k);
          acc[j] += x.x * w.x + x.y * w.y + x.z * w.z + x.w * w.w;
        }
      const float4 w = *reinterpret_cast<const float4*>(wc + k);
      acc[AMAX] += x.x * w.x + x.y * w.y + x.z * w.z + x.w * w.w;
    }
  } else {
    for (int k = lane; k < H; k += kWave) {
      const float x = h[k];
#pragma unroll
      for (int j = 0; j < AMAX; ++j)
        if (j < A) acc[j] += x * wa[static_cast<int64_t>(j) * H + k];
      acc[AMAX] += x * wc[k];
    }
  }
  float l[AMAX];
#pragma unroll
  for (int j = 0; j < AMAX; ++j) l[j] = j < A ? wave_sum(acc[j]) + ba[j] : 0.f;
  const float value = wave_sum(acc[AMAX]) + bc[0];
  if (lane != 0) return;
  float ln[AMAX], p[AMAX], lse;
  categorical_row<AMAX>(l, A, lse, ln, p);
  int best = 0;
  float best_q = p[0] / noise.get(n * A);
#pragma unroll
  for (int j = 1; j < AMAX; ++j)
    if (j < A) {
      const float q = p[j] / noise.get(n * A + j);
      if (q > best_q || (q != q && best_q == best_q)) {
        best_q = q;
        best = j;
      }
    }
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < AMAX; ++j)
    if (j == best) lp = ln[j];
  action_out[n] = best;
  logprob_out[n] = lp;
  value_out[n] = value;
  if (entropy_out) entropy_out[n] = categorical_entropy<AMAX>(ln, p, A);
  if (logits_out) {
#pragma unroll
    for (int j = 0; j < AMAX; ++j)
      if (j < A) logits_out[n * A + j] = l[j];
  }
}

// Fast path of the head for A <= 7 actions and H = 256*CH. Each wave keeps the A+1 weight rows
// in registers (CH*8 float4 per lane) and owns a group of E consecutive environments (E = 1 at
// the config sizes, up to 64 when N is large). Per environment: the hidden row (next one in
// flight), A+1 dot products padded to 8, reduced by a reduce-scatter butterfly -- xor 32 / 16 / 8
// halve the set of values each lane carries (4 + 2 + 1 shuffles), xor 4 / 2 / 1 finish one value
// per 8-lane group -- so lane 8j holds logit j (j = 7: the value); 8 lanes park them in LDS.
// Then lane e runs environment e's categorical (a wave64 VALU op costs the same for 1 or 64
// active lanes, so batching the ~500-instruction tail over E lanes is what makes large N
// HBM-bound) and the per-env outputs are stored coalesced.
constexpr int kHeadWavesPerBlock = 4;

// The synthetic env's step fused behind the head (ENV: E = 1, object frames): the wave that
// sampled env n's action steps env n right away -- lanes k < D write frame element k, lane 0 the
// reward / done / episode counters -- so the rollout step needs no env launch (the env of step t
// depends only on env n's own action).
struct HeadEnv {
  uint64_t seed;
  const int64_t* step_base;
  int64_t step_offset;
  int64_t D;
  float* frame;
  float* reward;
  float* done;
  float* ep;
};

template <int CH, bool ENV = false>
__global__ __launch_bounds__(256) void policy_head_fast_kernel(
    const float* __restrict__ hidden, int64_t N, int E, const float* __restrict__ wa,
    const float* __restrict__ ba, const float* __restrict__ wc, const float* __restrict__ bc,
    NoiseSrc noise, int A, int64_t* __restrict__ action_out,
    float* __restrict__ logprob_out, float* __restrict__ entropy_out,
    float* __restrict__ value_out, float* __restrict__ logits_out, HeadEnv env = HeadEnv{}) {
  constexpr int H = 256 * CH;
  __shared__ float s_logit[kHeadWavesPerBlock][kWave][9];  // [wave][env in group][8 (+pad)]
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kHeadWavesPerBlock;
  const int64_t ngroups = (N + E - 1) / E;
  int64_t g = static_cast<int64_t>(blockIdx.x) * kHeadWavesPerBlock + wv;
  if (g >= ngroups) return;  // wave-uniform
  const int jo = lane >> 3;  // the value this lane's 8-lane group ends up owning
  const float bias = jo < A ? ba[jo] : (jo == 7 ? bc[0] : 0.f);
  float4 w[8][CH];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float* wrow = j == 7 ? wc : wa + j * H;
#pragma unroll
    for (int c = 0; c < CH; ++c)
      w[j][c] = (j < A || j == 7) ? reinterpret_cast<const float4*>(wrow)[c * kWave + lane]
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (E == 1) {  // config sizes: one environment per wave, wave-uniform tail via v_readlane
    float4 x[CH];
    head_load_row<CH>(hidden, g, lane, x);
    // the in-kernel Exp(1) draw (Philox rounds) runs while the row's loads are in flight
    float nz = lane < A ? noise.get(g * A + lane) : 1.f;
    for (; g < ngroups; g += nwaves) {
      // ENV: everything of env g's step that does not depend on its action -- the frame hashes
      // and the reward / done / episode counters -- while this row's loads are in flight
      uint64_t key = 0;
      uint32_t base = 0;
      if (ENV) {
        key = synth_env_key(env.seed, static_cast<uint64_t>(env.step_base[0] + env.step_offset), g);
        if (lane < env.D) base = synth_env_obj_base(key, lane);
        if (lane == 0) synth_env_outcome(key, g, env.reward, env.done, env.ep);
      }
      const float t = head_dots<CH>(x, w, lane) + bias;
      float l[8], nzj[7];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        l[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 8 * j));
#pragma unroll
      for (int j = 0; j < 7; ++j)
        nzj[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nz), j));
      const int best =
          head_tail(l, nzj, A, g, action_out, logprob_out, entropy_out, value_out, nullptr, lane == 0);
      const float mine = __shfl(t, 8 * (lane & 7));  // all lanes take part in the permute
      if (logits_out && lane < A) logits_out[g * A + lane] = mine;
      if (ENV) {  // best is wave-uniform (every lane ran the same tail on readlane'd values)
        if (lane < env.D) env.frame[g * env.D + lane] = synth_env_obj_act(base, lane, best);
        for (int64_t k = lane + kWave; k < env.D; k += kWave)
          env.frame[g * env.D + k] = synth_env_obj(key, k, best);
      }
      if (g + nwaves < ngroups) {
        head_load_row<CH>(hidden, g + nwaves, lane, x);
        nz = lane < A ? noise.get((g + nwaves) * A + lane) : 1.f;
      }
    }
    return;
  }
  for (; g < ngroups; g += nwaves) {
    const int64_t n0 = g * E;
    const int cnt = static_cast<int>((N - n0) < E ? (N - n0) : E);
    const int64_t nt = n0 + lane;  // this lane's environment in the tail
    float nzj[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) nzj[j] = (lane < cnt && j < A) ? noise.get(nt * A + j) : 1.f;
    float4 x[CH], xn[CH];
    head_load_row<CH>(hidden, n0, lane, x);
    for (int e = 0; e < cnt; ++e) {
      if (e + 1 < cnt) head_load_row<CH>(hidden, n0 + e + 1, lane, xn);
      const float t = head_dots<CH>(x, w, lane);
      if ((lane & 7) == 0) s_logit[wv][e][jo] = t + bias;
#pragma unroll
      for (int c = 0; c < CH; ++c) x[c] = xn[c];
    }
    // the LDS rows were written by this wave only; LDS executes one wave's ops in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < cnt) {
      float l[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) l[j] = s_logit[wv][lane][j];
      head_tail(l, nzj, A, nt, action_out, logprob_out, entropy_out, value_out, logits_out, true);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the tail's LDS reads precede the next group's writes
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

}  // namespace ocppo

using namespace ocppo;

// workspace: [tickets | per-block partials | per-group partials | adv stats (2 floats)]
static int64_t loss_blocks(int64_t M) {
  const int64_t nb = ceil_div(M, kLossThreads);
  return nb < kLossMaxBlocks ? nb : kLossMaxBlocks;
}
static int64_t loss_blocks_vec(int64_t M) {
  const int64_t nb = ceil_div(M, kLossTile);
  return nb < kHandoffMaxBlocks ? nb : kHandoffMaxBlocks;
}
#ifndef OCPPO_LOSS_VEC_MIN_M  // experiments (tools/build_variant.py) move the switch-over
#define OCPPO_LOSS_VEC_MIN_M (256 * kLossTile)
#endif
constexpr int64_t kLossVecMinM = OCPPO_LOSS_VEC_MIN_M;
static bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }
static size_t round16(size_t n) { return (n + 15) / 16 * 16; }
static size_t loss_partials_offset() { return kTicketBytes; }
static size_t loss_gpartials_offset(int64_t M) {
  const int64_t nb = loss_blocks(M) > loss_blocks_vec(M) ? loss_blocks(M) : loss_blocks_vec(M);
  return kTicketBytes + round16(static_cast<size_t>(nb) * kNumPartials * sizeof(float));
}
static size_t loss_stats_offset(int64_t M) {
  return loss_gpartials_offset(M) + round16(kHandoffMaxGroups * kNumPartials * sizeof(float));
}

extern "C" size_t ocppo_ppo_loss_workspace_bytes(int64_t M, int64_t A) {
  (void)A;
  if (M <= 0) return kTicketBytes;
  return loss_stats_offset(M) + 16;
}

extern "C" int ocppo_minibatch_adv_stats(ocppo_stream_t stream, const float* b_advantages,
                                         const int64_t* perm, int64_t M, int64_t num_mb,
                                         float* out) {
  OCPPO_REQUIRE(M > 0 && num_mb > 0 && num_mb <= INT32_MAX,
                "ocppo_minibatch_adv_stats: bad sizes M=%lld num_mb=%lld", (long long)M,
                (long long)num_mb);
  OCPPO_REQUIRE(b_advantages && out, "ocppo_minibatch_adv_stats: null pointer");
  clear_stale_error();
  launch_adv_stats(as_stream(stream), b_advantages, perm, M, num_mb, out);
  return check_launch("ocppo_minibatch_adv_stats");
}

extern "C" int ocppo_ppo_loss_fwd_bwd(ocppo_stream_t stream, const float* logits,
                                      const float* new_value, int64_t M, int64_t A,
                                      const int64_t* mb_inds, const int64_t* b_actions,
                                      const float* b_logprobs, const float* b_advantages,
                                      const float* b_returns, const float* b_values,
                                      const float* adv_stats, double clip_coef, double ent_coef,
                                      double vf_coef, int norm_adv, int clip_vloss, float* dlogits,
                                      float* dvalue, float* stats, void* workspace,
                                      size_t workspace_bytes) {
  OCPPO_REQUIRE(M > 0 && A > 0 && A <= kMaxActions && M <= (int64_t)INT32_MAX * kLossThreads,
                "ocppo_ppo_loss_fwd_bwd: bad sizes M=%lld A=%lld (A <= %d)", (long long)M,
                (long long)A, kMaxActions);
  OCPPO_REQUIRE(logits && new_value && b_actions && b_logprobs && b_advantages && b_returns &&
                    b_values && dlogits && dvalue && stats,
                "ocppo_ppo_loss_fwd_bwd: null pointer");
  if (!workspace || workspace_bytes < ocppo_ppo_loss_workspace_bytes(M, A))
    return fail(OCPPO_E_WORKSPACE, "ocppo_ppo_loss_fwd_bwd: workspace needs %zu bytes, got %zu",
                ocppo_ppo_loss_workspace_bytes(M, A), workspace_bytes);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  if (norm_adv && !adv_stats) {
    float* st = reinterpret_cast<float*>(ws + loss_stats_offset(M));
    launch_adv_stats(s, b_advantages, mb_inds, M, 1, st);
    if (int rc = check_launch("ocppo_ppo_loss_fwd_bwd/adv_stats")) return rc;
    adv_stats = st;
  }
  LossParams P;
  P.logits = logits;
  P.new_value = new_value;
  P.mb_inds = mb_inds;
  P.b_actions = b_actions;
  P.b_logprobs = b_logprobs;
  P.b_adv = b_advantages;
  P.b_ret = b_returns;
  P.b_val = b_values;
  P.adv_stats = adv_stats;
  P.dlogits = dlogits;
  P.dvalue = dvalue;
  P.stats = stats;
  P.ticket = reinterpret_cast<unsigned*>(ws);
  P.partials = reinterpret_cast<float*>(ws + loss_partials_offset());
  P.gpartials = reinterpret_cast<float*>(ws + loss_gpartials_offset(M));
  P.M = M;
  P.A = static_cast<int>(A);
  P.norm_adv = norm_adv ? 1 : 0;
  P.clip_vloss = clip_vloss ? 1 : 0;
  P.clip = static_cast<float>(clip_coef);
  P.clip_lo = static_cast<float>(1.0 - clip_coef);
  P.clip_hi = static_cast<float>(1.0 + clip_coef);
  P.ent_coef = static_cast<float>(ent_coef);
  P.vf_coef = static_cast<float>(vf_coef);
  const float fm = static_cast<float>(M);
  // autograd: mean() backward divides the upstream grad by numel; the upstream grads are
  // d loss/d pg_loss = 1, d loss/d entropy_loss = -ent_coef, d loss/d v_loss_max.mean() = vf*0.5
  P.g_pg = 1.0f / fm;
  P.g_h = (-1.0f * P.ent_coef) / fm;
  P.g_v = (P.vf_coef * 0.5f) / fm;
  P.inv_m = 1.0f / fm;
  static_assert(kLossMaxBlocks <= kHandoffMaxBlocks, "hand-off capacity");
  // streaming form: contiguous (prepared) records, 16-B aligned arrays, at least one full tile per
  // CU (below that the 256-element tiles of ppo_loss_kernel spread the latency over more CUs)
  const bool vec_ok = !mb_inds && M >= kLossVecMinM &&
                      (A == 3 || A == 4 || A == 6 || A == 9 || A == 18) &&
                      aligned16(logits) && aligned16(new_value) && aligned16(b_actions) &&
                      aligned16(b_logprobs) && aligned16(b_advantages) && aligned16(b_returns) &&
                      aligned16(b_values) && aligned16(dlogits) && aligned16(dvalue);
  if (vec_ok) {
    const dim3 g(static_cast<unsigned>(loss_blocks_vec(M))), b(kLossThreads);
    const size_t lds = sizeof(float) * kLossTile * A;
    switch (A) {
      case 3: hipLaunchKernelGGL(ppo_loss_vec_kernel<3>, g, b, lds, s, P); break;
      case 4: hipLaunchKernelGGL(ppo_loss_vec_kernel<4>, g, b, lds, s, P); break;
      case 6: hipLaunchKernelGGL(ppo_loss_vec_kernel<6>, g, b, lds, s, P); break;
      case 9: hipLaunchKernelGGL(ppo_loss_vec_kernel<9>, g, b, lds, s, P); break;
      default: hipLaunchKernelGGL(ppo_loss_vec_kernel<18>, g, b, lds, s, P); break;
    }
    return check_launch("ocppo_ppo_loss_fwd_bwd");
  }
  const int64_t nb = loss_blocks(M);
  const size_t lds = sizeof(float) * kLossThreads * A;
  const dim3 g(static_cast<unsigned>(nb)), b(kLossThreads);
  switch (A) {
    case 3: hipLaunchKernelGGL(ppo_loss_kernel_small<3>, g, b, lds, s, P); break;
    case 4: hipLaunchKernelGGL(ppo_loss_kernel_small<4>, g, b, lds, s, P); break;
    case 6: hipLaunchKernelGGL(ppo_loss_kernel_small<6>, g, b, lds, s, P); break;
    case 9: hipLaunchKernelGGL((ppo_loss_kernel<9, true>), g, b, lds, s, P); break;
    case 18: hipLaunchKernelGGL((ppo_loss_kernel<18, true>), g, b, lds, s, P); break;
    default:
      if (A <= 8)
        hipLaunchKernelGGL((ppo_loss_kernel<8, false>), g, b, lds, s, P);
      else
        hipLaunchKernelGGL((ppo_loss_kernel<kMaxActions, false>), g, b, lds, s, P);
  }
  return check_launch("ocppo_ppo_loss_fwd_bwd");
}

// The sampling entries' noise operand: `noise` read, or (philox_state set) drawn in the kernel at
// torch's (seed, offset) = philox_state[0..1] + (0, philox_offset) with grid stride philox_stride
// and written to `noise` when that is non-NULL.
static int noise_src(const char* what, float* noise, const int64_t* philox_state,
                     int64_t philox_offset, int64_t philox_stride, NoiseSrc* out) {
  OCPPO_REQUIRE(philox_state || noise, "%s: neither noise nor philox_state", what);
  OCPPO_REQUIRE(!philox_state || (philox_stride > 0 && philox_stride % 256 == 0 &&
                                  philox_offset >= 0),
                "%s: bad philox stride %lld / offset %lld", what, (long long)philox_stride,
                (long long)philox_offset);
  *out = NoiseSrc{noise, philox_state ? noise : nullptr,
                  PhiloxNoise{philox_state, philox_offset, philox_stride}};
  return OCPPO_OK;
}

extern "C" int ocppo_categorical_sample(ocppo_stream_t stream, const float* logits, float* noise,
                                        const int64_t* philox_state, int64_t philox_offset,
                                        int64_t philox_stride, int64_t N, int64_t A,
                                        int64_t* action_out, float* logprob_out,
                                        float* entropy_out, const float* value_in,
                                        float* value_out) {
  OCPPO_REQUIRE(N >= 0 && A > 0 && A <= kMaxActions, "ocppo_categorical_sample: bad sizes");
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(logits && action_out && logprob_out, "ocppo_categorical_sample: null pointer");
  NoiseSrc ns;
  if (int rc = noise_src("ocppo_categorical_sample", noise, philox_state, philox_offset,
                         philox_stride, &ns))
    return rc;
  const dim3 grid(ceil_div(N, 256));
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (A <= 8)
    hipLaunchKernelGGL(categorical_sample_kernel<8>, grid, dim3(256), 0, s, logits, ns, N,
                       (int)A, action_out, logprob_out, entropy_out, value_in, value_out);
  else
    hipLaunchKernelGGL(categorical_sample_kernel<kMaxActions>, grid, dim3(256), 0, s, logits,
                       ns, N, (int)A, action_out, logprob_out, entropy_out, value_in, value_out);
  return check_launch("ocppo_categorical_sample");
}

extern "C" int ocppo_categorical_logprob_entropy(ocppo_stream_t stream, const float* logits,
                                                 const int64_t* actions, int64_t N, int64_t A,
                                                 float* logprob_out, float* entropy_out) {
  OCPPO_REQUIRE(N >= 0 && A > 0 && A <= kMaxActions,
                "ocppo_categorical_logprob_entropy: bad sizes");
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(logits && actions, "ocppo_categorical_logprob_entropy: null pointer");
  const dim3 grid(ceil_div(N, 256));
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (A <= 8)
    hipLaunchKernelGGL(categorical_lp_ent_kernel<8>, grid, dim3(256), 0, s, logits, actions, N,
                       (int)A, logprob_out, entropy_out);
  else
    hipLaunchKernelGGL(categorical_lp_ent_kernel<kMaxActions>, grid, dim3(256), 0, s, logits,
                       actions, N, (int)A, logprob_out, entropy_out);
  return check_launch("ocppo_categorical_logprob_entropy");
}

extern "C" int ocppo_categorical_logprob_entropy_bwd(ocppo_stream_t stream, const float* logits,
                                                     const int64_t* actions,
                                                     const float* grad_logprob,
                                                     const float* grad_entropy, int64_t N,
                                                     int64_t A, float* dlogits) {
  OCPPO_REQUIRE(N >= 0 && A > 0 && A <= kMaxActions,
                "ocppo_categorical_logprob_entropy_bwd: bad sizes");
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(logits && actions && dlogits, "ocppo_categorical_logprob_entropy_bwd: null pointer");
  const dim3 grid(ceil_div(N, 256));
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (A <= 8)
    hipLaunchKernelGGL(categorical_lp_ent_bwd_kernel<8>, grid, dim3(256), 0, s, logits, actions,
                       grad_logprob, grad_entropy, N, (int)A, dlogits);
  else
    hipLaunchKernelGGL(categorical_lp_ent_bwd_kernel<kMaxActions>, grid, dim3(256), 0, s, logits,
                       actions, grad_logprob, grad_entropy, N, (int)A, dlogits);
  return check_launch("ocppo_categorical_logprob_entropy_bwd");
}

extern "C" int ocppo_policy_head_sample(ocppo_stream_t stream, const float* hidden, int64_t N,
                                        int64_t H, const float* w_actor, const float* b_actor,
                                        const float* w_critic, const float* b_critic,
                                        float* noise, const int64_t* philox_state,
                                        int64_t philox_offset, int64_t philox_stride, int64_t A,
                                        int64_t* action_out, float* logprob_out,
                                        float* entropy_out, float* value_out, float* logits_out) {
  OCPPO_REQUIRE(N >= 0 && H > 0 && H <= INT32_MAX && A > 0 && A <= kMaxActions,
                "ocppo_policy_head_sample: bad sizes N=%lld H=%lld A=%lld", (long long)N,
                (long long)H, (long long)A);
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(hidden && w_actor && b_actor && w_critic && b_critic && action_out &&
                    logprob_out && value_out,
                "ocppo_policy_head_sample: null pointer");
  NoiseSrc ns;
  if (int rc = noise_src("ocppo_policy_head_sample", noise, philox_state, philox_offset,
                         philox_stride, &ns))
    return rc;
  const dim3 grid(static_cast<unsigned>(ceil_div(N, 4))), block(256);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const bool aligned = ((reinterpret_cast<uintptr_t>(hidden) | reinterpret_cast<uintptr_t>(w_actor) |
                         reinterpret_cast<uintptr_t>(w_critic)) & 15) == 0;
  if (A <= 7 && H % 256 == 0 && H <= 256 * 4 && aligned) {
    // one wave per group of E environments; E = 1 while N fits 12 (CH > 2: 8) waves per CU,
    // doubling up to 64 environments per wave beyond that
    const int64_t cap = H <= 512 ? 256 * 12 : 256 * 8;
    int E = 1;
    while (E < 64 && ceil_div(N, static_cast<int64_t>(E)) > cap) E *= 2;
    const int64_t waves = ceil_div(N, static_cast<int64_t>(E));
    const dim3 hgrid(static_cast<unsigned>(ceil_div(waves, kHeadWavesPerBlock)));
#define OCPPO_HEAD(CH)                                                                           \
  hipLaunchKernelGGL(policy_head_fast_kernel<CH>, hgrid, dim3(kWave * kHeadWavesPerBlock), 0, s, \
                     hidden, N, E, w_actor, b_actor, w_critic, b_critic, ns, (int)A,             \
                     action_out, logprob_out, entropy_out, value_out, logits_out)
    switch (H / 256) {
      case 1: OCPPO_HEAD(1); break;
      case 2: OCPPO_HEAD(2); break;
      case 3: OCPPO_HEAD(3); break;
      default: OCPPO_HEAD(4); break;
    }
#undef OCPPO_HEAD
  } else if (A <= 8)
    hipLaunchKernelGGL(policy_head_sample_kernel<8>, grid, block, 0, s, hidden, N, (int)H, w_actor,
                       b_actor, w_critic, b_critic, ns, (int)A, action_out, logprob_out,
                       entropy_out, value_out, logits_out);
  else
    hipLaunchKernelGGL(policy_head_sample_kernel<kMaxActions>, grid, block, 0, s, hidden, N,
                       (int)H, w_actor, b_actor, w_critic, b_critic, ns, (int)A, action_out,
                       logprob_out, entropy_out, value_out, logits_out);
  return check_launch("ocppo_policy_head_sample");
}

extern "C" int ocppo_policy_head_env_step(ocppo_stream_t stream, const float* hidden, int64_t N,
                                          int64_t H, const float* w_actor, const float* b_actor,
                                          const float* w_critic, const float* b_critic,
                                          float* noise, const int64_t* philox_state,
                                          int64_t philox_offset, int64_t philox_stride,
                                          int64_t A, int64_t* action_out,
                                          float* logprob_out, float* value_out, uint64_t seed,
                                          const int64_t* step_base, int64_t step_offset,
                                          int64_t D, float* frame_out, float* reward_out,
                                          float* done_out, float* ep_state) {
  OCPPO_REQUIRE(N >= 1 && N <= 256 * 12 && H >= 256 && H % 256 == 0 && H <= 1024 && A >= 1 &&
                    A <= 7 && D >= 1 && D <= 4096 && (H <= 512 || N <= 256 * 8),
                "ocppo_policy_head_env_step: bad sizes N=%lld H=%lld A=%lld D=%lld", (long long)N,
                (long long)H, (long long)A, (long long)D);
  OCPPO_REQUIRE(hidden && w_actor && b_actor && w_critic && b_critic && action_out &&
                    logprob_out && value_out && step_base && frame_out && reward_out && done_out,
                "ocppo_policy_head_env_step: null pointer");
  NoiseSrc ns;
  if (int rc = noise_src("ocppo_policy_head_env_step", noise, philox_state, philox_offset,
                         philox_stride, &ns))
    return rc;
  OCPPO_REQUIRE(((reinterpret_cast<uintptr_t>(hidden) | reinterpret_cast<uintptr_t>(w_actor) |
                  reinterpret_cast<uintptr_t>(w_critic)) & 15) == 0,
                "ocppo_policy_head_env_step: hidden and head weights must be 16-B aligned");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  // one wave per environment (the E = 1 form of ocppo_policy_head_sample: same head results)
  const dim3 hgrid(static_cast<unsigned>(ceil_div(N, static_cast<int64_t>(kHeadWavesPerBlock))));
  const HeadEnv env{seed, step_base, step_offset, D, frame_out, reward_out, done_out, ep_state};
#define OCPPO_HEAD(CH)                                                                          \
  hipLaunchKernelGGL((policy_head_fast_kernel<CH, true>), hgrid, dim3(kWave * kHeadWavesPerBlock), \
                     0, s, hidden, N, 1, w_actor, b_actor, w_critic, b_critic, ns, (int)A,        \
                     action_out, logprob_out, nullptr, value_out, nullptr, env)
  switch (H / 256) {
    case 1: OCPPO_HEAD(1); break;
    case 2: OCPPO_HEAD(2); break;
    case 3: OCPPO_HEAD(3); break;
    default: OCPPO_HEAD(4); break;
  }
#undef OCPPO_HEAD
  return check_launch("ocppo_policy_head_env_step");
}

extern "C" int ocppo_minibatch_prepare(ocppo_stream_t stream, const int64_t* perm, int64_t M,
                                       int64_t num_mb, const int64_t* b_actions,
                                       const float* b_logprobs, const float* b_advantages,
                                       const float* b_returns, const float* b_values,
                                       int64_t* mb_actions, float* mb_logprobs,
                                       float* mb_advantages, float* mb_returns, float* mb_values,
                                       float* adv_stats) {
  OCPPO_REQUIRE(M > 0 && num_mb > 0 && num_mb <= INT32_MAX && M <= INT64_MAX / num_mb,
                "ocppo_minibatch_prepare: bad sizes M=%lld num_mb=%lld", (long long)M,
                (long long)num_mb);
  OCPPO_REQUIRE(perm && b_actions && b_logprobs && b_advantages && b_returns && b_values &&
                    mb_actions && mb_logprobs && mb_advantages && mb_returns && mb_values,
                "ocppo_minibatch_prepare: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  constexpr int VPT = 2;
  const int64_t n = M * num_mb;
  const int64_t gb = ceil_div(n, 256 * VPT);
  OCPPO_REQUIRE(gb + num_mb <= INT32_MAX, "ocppo_minibatch_prepare: too large");
  const dim3 grid(static_cast<unsigned>(gb + (adv_stats ? num_mb : 0))), block(256);
#define OCPPO_PREP(SV)                                                                           \
  hipLaunchKernelGGL((minibatch_prepare_kernel<VPT, SV>), grid, block, 0, s, perm, n, (int)gb, M, \
                     b_actions, b_logprobs, b_advantages, b_returns, b_values, mb_actions,       \
                     mb_logprobs, mb_advantages, mb_returns, mb_values, adv_stats)
  switch (adv_stats_vpt(M)) {
    case 1: OCPPO_PREP(1); break;
    case 4: OCPPO_PREP(4); break;
    case 16: OCPPO_PREP(16); break;
    case 64: OCPPO_PREP(64); break;
    default: OCPPO_PREP(0); break;
  }
#undef OCPPO_PREP
  return check_launch("ocppo_minibatch_prepare");
}

// samples (num_mb x M) from which the records' minibatch statistics are taken from the gathered
// (contiguous) advantages in a second launch instead of by the statistics blocks' own gathers
constexpr int64_t kPrepareSplitStats = int64_t(1) << 20;
#ifndef OCPPO_PREP_VPT  // records in flight per thread of the gather (experiments: tools/)
#define OCPPO_PREP_VPT 4
#endif

extern "C" int ocppo_minibatch_prepare_records(ocppo_stream_t stream, const int64_t* perm,
                                               int64_t M, int64_t num_mb, const void* records,
                                               int64_t* mb_actions, float* mb_logprobs,
                                               float* mb_advantages, float* mb_returns,
                                               float* mb_values, float* adv_stats) {
  OCPPO_REQUIRE(M > 0 && num_mb > 0 && num_mb <= INT32_MAX && M <= INT64_MAX / num_mb,
                "ocppo_minibatch_prepare_records: bad sizes M=%lld num_mb=%lld", (long long)M,
                (long long)num_mb);
  OCPPO_REQUIRE(perm && records && mb_actions && mb_logprobs && mb_advantages && mb_returns &&
                    mb_values && reinterpret_cast<uintptr_t>(records) % 16 == 0,
                "ocppo_minibatch_prepare_records: null pointer or records not 16-B aligned");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  constexpr int VPT = OCPPO_PREP_VPT;
  const int64_t n = M * num_mb;
  const int64_t gb = ceil_div(n, 256 * VPT);
  OCPPO_REQUIRE(gb + num_mb <= INT32_MAX, "ocppo_minibatch_prepare_records: too large");
  const float4* rec = static_cast<const float4*>(records);
  if (adv_stats && n >= kPrepareSplitStats) {
    // streaming sizes: the statistics blocks' own random gathers of the records (one cache line
    // fill per 4-B advantage) would double the gather's line traffic; instead the gather runs
    // alone and a second launch reads the gathered advantages contiguously -- the same values
    // in the same order, so the same figures bitwise
    hipLaunchKernelGGL((minibatch_prepare_rec_kernel<VPT, 1>), dim3(static_cast<unsigned>(gb)),
                       dim3(256), 0, s, perm, n, (int)gb, M, rec, mb_actions, mb_logprobs,
                       mb_advantages, mb_returns, mb_values, nullptr);
    if (int rc = check_launch("ocppo_minibatch_prepare_records")) return rc;
    launch_adv_stats(s, mb_advantages, nullptr, M, num_mb, adv_stats);
    return check_launch("ocppo_minibatch_prepare_records/stats");
  }
  const dim3 grid(static_cast<unsigned>(gb + (adv_stats ? num_mb : 0))), block(256);
#define OCPPO_PREP(SV)                                                                           \
  hipLaunchKernelGGL((minibatch_prepare_rec_kernel<VPT, SV>), grid, block, 0, s, perm, n, (int)gb, \
                     M, rec, mb_actions, mb_logprobs, mb_advantages, mb_returns, mb_values,      \
                     adv_stats)
  switch (adv_stats_vpt(M)) {
    case 1: OCPPO_PREP(1); break;
    case 4: OCPPO_PREP(4); break;
    case 16: OCPPO_PREP(16); break;
    case 64: OCPPO_PREP(64); break;
    default: OCPPO_PREP(0); break;
  }
#undef OCPPO_PREP
  return check_launch("ocppo_minibatch_prepare_records");
}

namespace ocppo {

// ---- policy heads forward + fused PPO loss + heads backward in ONE pass over h ---------------------
// The minibatch update's tail (ppo_atari_oc.py:566-605 from the decoder output h = relu(z) on):
// logits = h Wa^T + ba and value = h Wc^T + bc (architectures/ppo.py:81-84), the fused loss of
// loss_element (its per-row gradient needs only the prepared records, the minibatch's adv
// (mean, std) and 1/M), and the heads' whole backward with the decoder's ReLU mask:
//   c[m] = (d loss / d logits[m, 0..A), d loss / d value[m])
//   gp[m, j] = h[m, j] <= 0 ? 0 : sum_k c[m, k] W[k, j]        (W = [Wa; Wc], k order, fmaf)
//   db_h[j] = sum_m gp[m, j];  dW[k, j] = sum_m c[m, k] h[m, j];  db[k] = sum_m c[m, k]
// Row-major: one wave per row (lane = CPL = H / 64 adjacent columns), the A + 1 head dot products
// reduced by the wave's xor butterfly (bitwise the same in every lane), the loss computed by every
// lane alike, gp written once. Each workgroup sums its rows (waves, then LDS in wave order) into
// ONE partial record [H (K + 1) + K + 6]; heads_loss_finish_kernel adds the records in workgroup
// order (deterministic) and forms the loss statistics. Replaces two head GEMMs, the loss launch
// and ocppo_heads_bwd (logits / dlogits / value / dvalue never touch HBM).
struct HeadsLossParams {
  LossParams L;  // records (prepared, contiguous), adv_stats, coefficients, upstream grads
  const float* h;
  int64_t H;
  const float* wa;
  const float* ba;
  const float* wc;
  const float* bc;
  float* gp;
  float* partials;  // [gridDim.x][npw]
  int64_t npw;
  int rows_per_wg;
};

// Lane layout of a row: CPL columns per lane, interleaved so that every load of the wave is one
// contiguous run: CPL >= 4 -> float4 chunk q4 at columns 4 (q4 * 64 + lane) .. +3 (the policy
// head's layout); CPL < 4 -> column q * 64 + lane.
template <int CPL>
__device__ __forceinline__ int hl_col(int lane, int q) {
  return CPL >= 4 ? 4 * ((q >> 2) * kWave + lane) + (q & 3) : q * kWave + lane;
}

template <int CPL>
__device__ __forceinline__ void hl_load(const float* __restrict__ row, int lane, float (&x)[CPL]) {
  if (CPL >= 4) {
    const float4* r4 = reinterpret_cast<const float4*>(row);
#pragma unroll
    for (int q4 = 0; q4 < CPL / 4; ++q4) {
      const float4 v = r4[q4 * kWave + lane];
      x[4 * q4] = v.x; x[4 * q4 + 1] = v.y; x[4 * q4 + 2] = v.z; x[4 * q4 + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < CPL; ++q) x[q] = row[q * kWave + lane];
  }
}

template <int CPL>
__device__ __forceinline__ void hl_store(float* __restrict__ row, int lane, const float (&x)[CPL]) {
  if (CPL >= 4) {
    float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll
    for (int q4 = 0; q4 < CPL / 4; ++q4)
      r4[q4 * kWave + lane] = make_float4(x[4 * q4], x[4 * q4 + 1], x[4 * q4 + 2], x[4 * q4 + 3]);
  } else {
#pragma unroll
    for (int q = 0; q < CPL; ++q) row[q * kWave + lane] = x[q];
  }
}

// The 8 (A logits + value, zero-padded) dot products of one row, reduce-scattered (xor 32 / 16 / 8
// halve the values each lane carries, xor 4 / 2 / 1 finish one value per 8-lane group: 10
// cross-lane steps instead of 48) and broadcast: out[j] = lane 8j's sum, wave-uniform.
template <int CPL>
__device__ __forceinline__ void hl_dots(const float (&x)[CPL], const float (&w)[8][CPL], int lane,
                                        float (&out)[8]) {
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) s = fmaf(x[q], w[j][q], s);
    acc[j] = s;
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
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), 8 * j));
}

// ---- heads_loss rows kernel -----------------------------------------------------------------------
// A wave walks its rows U at a time. Lane layout of a row: CPL = H / 64 columns per lane
// (hl_col). Per step:
//   1. the U rows' h chunks were loaded one step ahead (ping-pong register sets); lane u < U also
//      loads row u's records (action, old log-prob, advantage, return, old value);
//   2. per lane the U x NK partial dot products (NK = AMAX actor logits + the value), then ONE
//      reduce-scatter over the wave for all of them (xor 32 .. 2: each lane keeps half of its
//      values and adds its partner's other half), so value (u, k) ends in lanes 2(8u + k) and
//      2(8u + k) + 1 (U = 4) or lane 8u + k (U = 8);
//   3. lane u gathers row u's NK sums and runs the fused loss for row u: the loss arithmetic runs
//      once per U rows, not once per row in every lane;
//   4. each row's NK gradients c are broadcast (readlane) and the heads' backward runs per row:
//      gp = (h > 0) * sum_k c_k W_k (written once), db_h += gp, dW_k += c_k h (registers).
// Lanes accumulate c (head db) and the loss partials for their own rows; the workgroup adds its
// waves through LDS in wave order and writes ONE record.
// Packed f32 pairs (v_pk_fma_f32 / v_pk_add_f32: two f32 lanes per instruction). A lane's CPL
// columns are held as CP = max(CPL / 2, 1) pairs (q = 2p, 2p + 1 of hl_col's order; CPL = 1 pads
// the second half with zeros).
typedef float hl_f2 __attribute__((ext_vector_type(2)));

template <int CPL>
__device__ __forceinline__ void hl_load2(const float* __restrict__ row, int lane,
                                         hl_f2 (&x)[CPL >= 2 ? CPL / 2 : 1]) {
  if constexpr (CPL >= 4) {
    const float4* r4 = reinterpret_cast<const float4*>(row);
#pragma unroll
    for (int q4 = 0; q4 < CPL / 4; ++q4) {
      const float4 v = r4[q4 * kWave + lane];
      x[2 * q4] = hl_f2{v.x, v.y};
      x[2 * q4 + 1] = hl_f2{v.z, v.w};
    }
  } else if constexpr (CPL == 2) {
    x[0] = hl_f2{row[lane], row[kWave + lane]};
  } else {
    x[0] = hl_f2{row[lane], 0.f};
  }
}

template <int CPL>
__device__ __forceinline__ void hl_store2(float* __restrict__ row, int lane,
                                          const hl_f2 (&x)[CPL >= 2 ? CPL / 2 : 1]) {
  if constexpr (CPL >= 4) {
    float4* r4 = reinterpret_cast<float4*>(row);
#pragma unroll
    for (int q4 = 0; q4 < CPL / 4; ++q4)
      r4[q4 * kWave + lane] = make_float4(x[2 * q4].x, x[2 * q4].y, x[2 * q4 + 1].x,
                                          x[2 * q4 + 1].y);
  } else if constexpr (CPL == 2) {
    row[lane] = x[0].x;
    row[kWave + lane] = x[0].y;
  } else {
    row[lane] = x[0].x;
  }
}

template <int CPL, int U>
struct HlRows {
  static constexpr int CP = CPL >= 2 ? CPL / 2 : 1;
  hl_f2 x[U][CP];
  int64_t a;                    // lane u < U: row u's record
  float old_lp, adv, R, v_old;
};

template <int CPL, int U>
__device__ __forceinline__ void hl_rows_load(const HeadsLossParams& P, int64_t rb, int64_t r1,
                                             int lane, HlRows<CPL, U>& s) {
  const LossParams& L = P.L;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t r = rb + u < r1 ? rb + u : rb;
    hl_load2<CPL>(P.h + r * P.H, lane, s.x[u]);
  }
  const int64_t rl = rb + (lane & (U - 1)) < r1 ? rb + (lane & (U - 1)) : rb;
  s.a = L.b_actions[rl];
  s.old_lp = L.b_logprobs[rl];
  s.adv = L.b_adv[rl];
  s.R = L.b_ret[rl];
  s.v_old = L.b_val[rl];
}

template <int CPL, int NK>
struct HlAcc {
  static constexpr int CP = CPL >= 2 ? CPL / 2 : 1;
  hl_f2 sb[CP], sw[NK][CP];
  float sc[NK], part[kNumPartials];  // per lane: the rows this lane ran the loss for
};

// One reduce-scatter step over N values: partner lane = lane ^ M; the lane with bit M set keeps
// the upper half of its values and receives the partner's upper half (the other lane the lower
// halves), so the N / 2 values left are sums over both lanes.
template <int N, int M>
__device__ __forceinline__ void hl_rs_step(float* v, int lane) {
  const bool hi = lane & M;
#pragma unroll
  for (int i = 0; i < N / 2; ++i) {
    const float send = hi ? v[i] : v[i + N / 2];
    const float keep = hi ? v[i + N / 2] : v[i];
    v[i] = keep + __shfl_xor(send, M);
  }
}

// Reduce-scatter of the 8U values over the wave (masks 32, 16, ... halving the values each step);
// returns the wave sum of value lane >> 1 (U = 4, after a last xor-1 add) or of value lane (U = 8).
template <int U>
__device__ __forceinline__ float hl_reduce_scatter(float (&v)[8 * U], int lane) {
#ifdef OCPPO_HL_NORED  // probe variant (tools/): no cross-lane reduction
  return v[lane & (8 * U - 1)];
#endif
  if constexpr (U == 8) {
    hl_rs_step<64, 32>(v, lane);
    hl_rs_step<32, 16>(v, lane);
    hl_rs_step<16, 8>(v, lane);
    hl_rs_step<8, 4>(v, lane);
    hl_rs_step<4, 2>(v, lane);
    hl_rs_step<2, 1>(v, lane);
    return v[0];
  } else {
    hl_rs_step<32, 32>(v, lane);
    hl_rs_step<16, 16>(v, lane);
    hl_rs_step<8, 8>(v, lane);
    hl_rs_step<4, 4>(v, lane);
    hl_rs_step<2, 2>(v, lane);
    return v[0] + __shfl_xor(v[0], 1);
  }
}

template <int AMAX, bool EXACT, int CPL, int U>
__device__ __forceinline__ void hl_rows_compute(const HeadsLossParams& P, int A,
                                                const hl_f2 (&w)[AMAX + 1][CPL >= 2 ? CPL / 2 : 1],
                                                const float (&bk)[AMAX + 1], float adv_mean,
                                                float adv_den, int64_t rb, int64_t r1, int lane,
                                                const HlRows<CPL, U>& s,
                                                HlAcc<CPL, AMAX + 1>& acc) {
  constexpr int NK = AMAX + 1, CP = CPL >= 2 ? CPL / 2 : 1;
  const LossParams& L = P.L;
  // 2. partial dots (even / odd columns in the two halves of a packed accumulator), slot (u, k)
  //    at u * 8 + k (k = NK..7 padding)
  float v[8 * U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    hl_f2 d[NK];  // NK independent chains interleaved (no back-to-back dependent pk_fma)
#pragma unroll
    for (int k = 0; k < NK; ++k) d[k] = hl_f2{0.f, 0.f};
#pragma unroll
    for (int p = 0; p < CP; ++p)
#pragma unroll
      for (int k = 0; k < NK; ++k) d[k] = __builtin_elementwise_fma(s.x[u][p], w[k][p], d[k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[u * 8 + k] = k < NK ? d[k].x + d[k].y : 0.f;
  }
  const float red = hl_reduce_scatter<U>(v, lane);
  // 3. the loss of row `lane` (lanes < U)
  const int lu = lane & (U - 1);
  float l[AMAX], vnew = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int src = U == 4 ? 2 * (8 * lu + k) : 8 * lu + k;
    const float t = __shfl(red, src);
    if (k < AMAX) l[k] = t + bk[k];
    else vnew = t + bk[k];
  }
  float dl[AMAX], dv;
  float pr[kNumPartials] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  loss_element<AMAX>(L, A, l, s.a, s.old_lp, s.adv, s.R, s.v_old, vnew, adv_mean, adv_den, pr,
                     dl, dv);
  const bool mine = lane < U && rb + lane < r1;
  float cl[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) cl[k] = mine ? (k < AMAX ? (k < A ? dl[k] : 0.f) : dv) : 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) acc.sc[k] += cl[k];
#pragma unroll
  for (int q = 0; q < kNumPartials; ++q) acc.part[q] += mine ? pr[q] : 0.f;
  if (L.dlogits != nullptr && mine) {
    const int64_t r = rb + lane;
#pragma unroll
    for (int k = 0; k < AMAX; ++k)
      if (k < A) L.dlogits[r * A + k] = dl[k];
    L.dvalue[r] = dv;
  }
  // 4. the heads' backward per row
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (rb + u >= r1) break;  // wave-uniform
    float c[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k)
      c[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cl[k]), u));
    hl_f2 d[CP], g[CP];  // CP independent chains interleaved
#pragma unroll
    for (int p = 0; p < CP; ++p) d[p] = hl_f2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int p = 0; p < CP; ++p)
        d[p] = __builtin_elementwise_fma(hl_f2{c[k], c[k]}, w[k][p], d[p]);
#pragma unroll
    for (int k = 0; k < NK; ++k)
#pragma unroll
      for (int p = 0; p < CP; ++p)
        acc.sw[k][p] = __builtin_elementwise_fma(hl_f2{c[k], c[k]}, s.x[u][p], acc.sw[k][p]);
#pragma unroll
    for (int p = 0; p < CP; ++p) {
      const hl_f2 xv = s.x[u][p];
      g[p] = hl_f2{xv.x <= 0.f ? 0.f : d[p].x, xv.y <= 0.f ? 0.f : d[p].y};
      acc.sb[p] += g[p];
    }
#ifndef OCPPO_HL_NOSTORE  // probe variant (tools/)
    hl_store2<CPL>(P.gp + (rb + u) * P.H, lane, g);
#else
    if (g[0].x == 12345.f) hl_store2<CPL>(P.gp + (rb + u) * P.H, lane, g);
#endif
  }
}

// Fixed grid (hl_layout): workgroup g owns rows [g * rows_per_wg, ...) and walks them in steps
// of U rows per wave (4 waves: 4U rows per step), the next step's loads issued before this step's
// arithmetic (two register sets, ping-pong). The workgroup's sums leave as ONE record
// [CPL][NV][64 lanes] (NV = AMAX + 2 slots: db_h, AMAX actor dW rows, critic dW), NK head-bias
// sums, the 6 loss partials at npw - 6: record traffic is O(grid), not O(M).
template <int AMAX, bool EXACT, int CPL, int U>
__global__ __launch_bounds__(256) void heads_loss_kernel(HeadsLossParams P) {
  static_assert(AMAX <= 7, "A logits + the value in 8 slots");
  static_assert(U == 4 || U == 8, "reduce-scatter layouts");
  constexpr int NK = AMAX + 1, NV = AMAX + 2;
  extern __shared__ __attribute__((aligned(16))) float hl_red[];  // [4][64][CPL * NV]
  __shared__ float s_misc[4][8 + kNumPartials];
  const LossParams& L = P.L;
  const int A = EXACT ? AMAX : L.A;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t H = P.H;
#ifdef OCPPO_HL_PHASES  // probe variant (tools/exp_hl_phases.py): shader-clock phase stamps
  const uint64_t t0 = __builtin_readcyclecounter();
#endif
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * P.rows_per_wg;
  const int64_t r1 = r0 + P.rows_per_wg < L.M ? r0 + P.rows_per_wg : L.M;
  int64_t rb = r0 + wv * U;
  constexpr int CP = CPL >= 2 ? CPL / 2 : 1;
  HlRows<CPL, U> sa, sbuf;
  if (rb < r1) hl_rows_load<CPL, U>(P, rb, r1, lane, sa);
  hl_f2 w[NK][CP];
  float bk[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const bool critic = k == AMAX;
    bk[k] = critic ? P.bc[0] : (k < A ? P.ba[k] : 0.f);
    const float* wr = critic ? P.wc : P.wa + static_cast<int64_t>(k < A ? k : 0) * H;
    hl_load2<CPL>(wr, lane, w[k]);
    if (!(critic || k < A)) {
#pragma unroll
      for (int p = 0; p < CP; ++p) w[k][p] = hl_f2{0.f, 0.f};
    }
  }
  HlAcc<CPL, NK> acc;
#pragma unroll
  for (int p = 0; p < CP; ++p) acc.sb[p] = hl_f2{0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    acc.sc[k] = 0.f;
#pragma unroll
    for (int p = 0; p < CP; ++p) acc.sw[k][p] = hl_f2{0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < kNumPartials; ++q) acc.part[q] = 0.f;
  const float adv_mean = L.norm_adv ? L.adv_stats[0] : 0.f;
  const float adv_den = L.norm_adv ? L.adv_stats[1] + 1e-8f : 1.f;
  constexpr int kStep = 4 * U;
  while (rb < r1) {
    if (rb + kStep < r1) hl_rows_load<CPL, U>(P, rb + kStep, r1, lane, sbuf);
    hl_rows_compute<AMAX, EXACT, CPL, U>(P, A, w, bk, adv_mean, adv_den, rb, r1, lane, sa, acc);
    rb += kStep;
    if (rb >= r1) break;
    if (rb + kStep < r1) hl_rows_load<CPL, U>(P, rb + kStep, r1, lane, sa);
    hl_rows_compute<AMAX, EXACT, CPL, U>(P, A, w, bk, adv_mean, adv_den, rb, r1, lane, sbuf,
                                         acc);
    rb += kStep;
  }
#ifdef OCPPO_HL_PHASES
  const uint64_t t1 = __builtin_readcyclecounter();
#endif
  // the lanes' head-bias and loss sums (lanes < U hold them): wave sum in lane order
  float misc[NK + kNumPartials];
#pragma unroll
  for (int k = 0; k < NK; ++k) misc[k] = acc.sc[k];
#pragma unroll
  for (int q = 0; q < kNumPartials; ++q) misc[NK + q] = acc.part[q];
#pragma unroll
  for (int i = 0; i < NK + kNumPartials; ++i) {
    float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(misc[i]), 0));
#pragma unroll
    for (int u = 1; u < U; ++u)
      t += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(misc[i]), u));
    misc[i] = t;
  }
#ifdef OCPPO_HL_NOREC  // probe variant (tools/): no workgroup combine, no record
  if (acc.sb[0].x != 12345.f) return;
#endif
  // workgroup combine: per lane CPL x NV values (+ padding to JP) through LDS as float4s,
  // waves in order. Image of a wave: [JP / 4][64 lanes][4] (consecutive lanes, consecutive
  // 16 B: conflict-free ds_write_b128 / ds_read_b128); the record keeps that layout.
  constexpr int JP = (CPL * NV + 3) / 4 * 4;
  float4* mine = reinterpret_cast<float4*>(hl_red) + static_cast<int64_t>(wv) * 16 * JP + lane;
#pragma unroll
  for (int c4 = 0; c4 < JP / 4; ++c4) {
    float e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * c4 + i, q = j / NV, slot = j - q * NV, p = q >> 1;
      e[i] = j >= CPL * NV ? 0.f
             : slot == 0   ? ((q & 1) ? acc.sb[p].y : acc.sb[p].x)
                           : ((q & 1) ? acc.sw[slot - 1][p].y : acc.sw[slot - 1][p].x);
    }
    mine[c4 * 64] = make_float4(e[0], e[1], e[2], e[3]);
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NK; ++k) s_misc[wv][k] = misc[k];
#pragma unroll
    for (int q = 0; q < kNumPartials; ++q) s_misc[wv][8 + q] = misc[NK + q];
  }
  __syncthreads();
#ifdef OCPPO_HL_PHASES
  const uint64_t t2 = __builtin_readcyclecounter();
#endif
  float* out = P.partials + static_cast<int64_t>(blockIdx.x) * P.npw;
  constexpr int nvals = 64 * JP;
  {
    const float4* img = reinterpret_cast<const float4*>(hl_red);
    float4* out4 = reinterpret_cast<float4*>(out);
    for (int c = threadIdx.x; c < nvals / 4; c += 256) {
      float4 a = img[c];
#pragma unroll
      for (int wq = 1; wq < 4; ++wq) {
        const float4 b = img[wq * (nvals / 4) + c];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      out4[c] = a;
    }
  }
  if (threadIdx.x < NK) {
    const int i = threadIdx.x;
    float sacc = s_misc[0][i];
    for (int wq = 1; wq < 4; ++wq) sacc += s_misc[wq][i];
    out[nvals + i] = sacc;
  } else if (threadIdx.x >= 64 && threadIdx.x < 64 + kNumPartials) {
    const int i = threadIdx.x - 64;
    float sacc = s_misc[0][8 + i];
    for (int wq = 1; wq < 4; ++wq) sacc += s_misc[wq][8 + i];
    out[P.npw - 8 + i] = sacc;  // at ls (npw = ls + 8)
  }
#ifdef OCPPO_HL_PHASES
  const uint64_t t3 = __builtin_readcyclecounter();
  __syncthreads();
  if (lane == 0) {  // per wave: rows done, LDS image synced, record issued (cycles after start)
    float* dbg = P.gp + (static_cast<int64_t>(blockIdx.x) * 4 + wv) * 4;
    dbg[0] = static_cast<float>(t1 - t0);
    dbg[1] = static_cast<float>(t2 - t0);
    dbg[2] = static_cast<float>(t3 - t0);
    dbg[3] = static_cast<float>(t0 & 0xFFFFFF);
  }
#endif
}

// Adds the G workgroup records with a fixed-shape tree: a block owns 32 record entries (outputs)
// x 8 record groups; group gi takes records gi, gi + 8, gi + 16, ... in batches of 32 loads in
// flight (one batch for G <= 256), each batch summed pairwise (16 / 8 / 4 / 2 / 1), batch sums
// added in batch order, then the 8 group sums pairwise through LDS. The same shape for every G:
// deterministic. The record holds the 6 loss partials at `ls` (a multiple of 32), so one block
// holds all of them and forms the loss statistics (loss_finish's formulas).
#ifndef OCPPO_HLFIN_OUT  // finish geometry (outputs x record groups per block); tools/ variants
#define OCPPO_HLFIN_OUT 32
#endif
constexpr int kHlFinOut = OCPPO_HLFIN_OUT, kHlFinGroups = 256 / kHlFinOut, kHlFinBatch = 32;

// Everything the finish needs, fixed when the rows kernel is launched (ocppo_heads_loss_rows
// hands it to the caller as an ocppo_deferred_finish_t, so the finish can ride in a later launch)
struct HlFinish {
  const float* partials;
  int G, A, amax, cpl;
  int64_t npw, ls, H;
  float *db_h, *dwa, *dwc, *dba, *dbc;
  LossParams L;
  int blocks;  // finish workgroups: ceil(npw / kHlFinOut)
};

// finish workgroup `blk` of f (256 threads)
__device__ __forceinline__ void hl_finish_block(const HlFinish& f, int blk) {
  __shared__ float red[kHlFinGroups][kHlFinOut + 1];
  __shared__ float tot[kHlFinOut];
  const int o = threadIdx.x % kHlFinOut, gi = threadIdx.x / kHlFinOut;
  const int64_t idx = static_cast<int64_t>(blk) * kHlFinOut + o;
  const float* __restrict__ partials = f.partials;
  const int G = f.G;
  float s = 0.f;
  if (idx < f.npw) {
    for (int g0 = gi; g0 < G; g0 += kHlFinGroups * kHlFinBatch) {
      float v[kHlFinBatch];
#pragma unroll
      for (int u = 0; u < kHlFinBatch; ++u) {
        const int g = g0 + u * kHlFinGroups;
        v[u] = g < G ? partials[static_cast<int64_t>(g) * f.npw + idx] : 0.f;
      }
#pragma unroll
      for (int wdt = kHlFinBatch / 2; wdt >= 1; wdt /= 2)
#pragma unroll
        for (int u = 0; u < wdt; ++u) v[u] += v[u + wdt];
      s += v[0];
    }
  }
  red[gi][o] = s;
  __syncthreads();
  for (int wdt = kHlFinGroups / 2; wdt >= 1; wdt /= 2) {
    if (gi < wdt) red[gi][o] += red[gi + wdt][o];
    __syncthreads();
  }
  const int nv = f.amax + 2;
  const int jp = (f.cpl * nv + 3) / 4 * 4;
  const int64_t nvals = 64 * jp;
  if (gi == 0) {
    const float t = red[0][o];
    tot[o] = t;
    const int ln = static_cast<int>((idx >> 2) & 63);
    const int j = static_cast<int>((idx >> 8) * 4 + (idx & 3));
    if (idx < nvals) {  // [j / 4][lane][j % 4], j = q * nv + slot (j >= cpl * nv: padding)
      const int q = j / nv, slot = j - q * nv;
      const int64_t col = f.cpl >= 4 ? 4 * ((q >> 2) * kWave + ln) + (q & 3) : q * kWave + ln;
      if (j >= f.cpl * nv) {
      } else if (slot == 0) {
        if (f.db_h) f.db_h[col] = t;
      } else if (slot == nv - 1) {
        f.dwc[col] = t;
      } else if (slot - 1 < f.A) {
        f.dwa[static_cast<int64_t>(slot - 1) * f.H + col] = t;
      }
    } else if (idx < nvals + f.amax + 1) {
      const int k = static_cast<int>(idx - nvals);
      if (k < f.A) f.dba[k] = t;
      else if (k == f.amax) f.dbc[0] = t;
    }
  }
  __syncthreads();
  if (static_cast<int64_t>(blk) * kHlFinOut == f.ls && threadIdx.x == 0) {
    const LossParams& L = f.L;
    const float pg_loss = tot[0] * L.inv_m;
    const float v_loss = 0.5f * (tot[1] * L.inv_m);
    const float ent = tot[2] * L.inv_m;
    const float loss = (pg_loss - L.ent_coef * ent) + v_loss * L.vf_coef;
    L.stats[OCPPO_STAT_LOSS] = loss;
    L.stats[OCPPO_STAT_PG_LOSS] = pg_loss;
    L.stats[OCPPO_STAT_V_LOSS] = v_loss;
    L.stats[OCPPO_STAT_ENTROPY] = ent;
    L.stats[OCPPO_STAT_OLD_APPROX_KL] = tot[3] * L.inv_m;
    L.stats[OCPPO_STAT_APPROX_KL] = tot[4] * L.inv_m;
    L.stats[OCPPO_STAT_CLIPFRAC] = tot[5] * L.inv_m;
    L.stats[OCPPO_STAT_ADV_MEAN] = L.norm_adv ? L.adv_stats[0] : 0.f;
    L.stats[OCPPO_STAT_ADV_STD] = L.norm_adv ? L.adv_stats[1] : 0.f;
  }
}

__global__ __launch_bounds__(256) void heads_loss_finish_kernel(HlFinish f) {
  hl_finish_block(f, blockIdx.x);
}

// The finish folded into the split-K combine of the decoder's weight gradient, the next
// combine the backward runs anyway (ppo_atari_oc.py:605): workgroups [0, f.blocks) are finish
// workgroups (dispatched first: their dependent load -> tree -> store chain is the launch's
// latency, the streaming combine fills the CUs beside them), the rest sum the S split blocks
// (float64, split order, one rounding: bitwise ocppo_sum_splits). One launch instead of two; the
// finish's outputs are read by no kernel before the optimizer step.
template <int S>
__global__ __launch_bounds__(256) void sum_splits_hlfin_kernel(const float4* __restrict__ part,
                                                               int64_t n4, float4* __restrict__ out,
                                                               int nsb, HlFinish f) {
  if (static_cast<int>(blockIdx.x) < f.blocks) {
    hl_finish_block(f, blockIdx.x);
    return;
  }
  const int sb = static_cast<int>(blockIdx.x) - f.blocks;
  const int64_t stride = static_cast<int64_t>(nsb) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(sb) * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    float4 v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = part[s * n4 + i];
    double ax = v[0].x, ay = v[0].y, az = v[0].z, aw = v[0].w;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      ax += v[s].x; ay += v[s].y; az += v[s].z; aw += v[s].w;
    }
    out[i] = make_float4(static_cast<float>(ax), static_cast<float>(ay), static_cast<float>(az),
                         static_cast<float>(aw));
  }
}

// the deferred-finish record behind the C-ABI's opaque ocppo_deferred_finish_t
constexpr uint64_t kDeferHeads = 0x6f63707068666e31ull;  // tag of a heads-loss finish
struct DeferredFinish {
  uint64_t tag;
  HlFinish f;
};
static_assert(sizeof(DeferredFinish) <= sizeof(ocppo_deferred_finish_t),
              "ocppo_deferred_finish_t too small");

// Grid of the rows launch: G = min(ceil(M / rows_min), grid_cap) workgroups of rows_per_wg rows
// (a multiple of the 16-row step of 4 waves x U = 4 rows). rows_min = 16 keeps a config-size
// minibatch (4096 rows) on 256 workgroups, one per CU, every wave's 4 rows loaded at once;
// grid_cap = 256 (one per CU: ~300 VGPRs, one wave per SIMD, 64 KB of h in flight per CU with the
// ping-pong) bounds the records at streaming sizes.
// Compile-time only (-DOCPPO_HL_ROWS=... / -DOCPPO_HL_GRID=..., tools/build_variant.py): the
// grid fixes the records' summation order, so the shipped library has one geometry, independent
// of the environment.
#ifndef OCPPO_HL_ROWS
#define OCPPO_HL_ROWS 16
#endif
#ifndef OCPPO_HL_GRID
#define OCPPO_HL_GRID 256
#endif
static_assert(OCPPO_HL_ROWS >= 16 && OCPPO_HL_ROWS % 16 == 0 && OCPPO_HL_GRID >= 1,
              "heads_loss geometry");

// the action count the rows kernel is instantiated with: exact for 4 (Breakout) and 6 (Pong,
// SpaceInvaders), else the 7-wide generic form
inline int hl_amax(int64_t A) { return A == 4 || A == 6 ? static_cast<int>(A) : 7; }

inline int64_t hl_layout(int64_t M, int64_t H, int64_t A, int64_t& G, int64_t& ls,
                         int64_t* rows_per_wg = nullptr) {
  constexpr int rows_min = OCPPO_HL_ROWS;
  constexpr int grid_cap = OCPPO_HL_GRID;
  G = (M + rows_min - 1) / rows_min;
  if (G > grid_cap) G = grid_cap;
  int64_t rpw = (M + G - 1) / G;
  rpw = (rpw + 15) / 16 * 16;
  G = (M + rpw - 1) / rpw;
  if (rows_per_wg) *rows_per_wg = rpw;
  const int64_t amax = hl_amax(A);
  // 64 lanes x (H / 64) columns x (amax + 2) slots (padded to a multiple of 4 per lane),
  // amax + 1 head-bias sums; the 6 loss partials at ls (npw = ls + 8 keeps records 16-B aligned)
  const int64_t jp = ((H / 64) * (amax + 2) + 3) / 4 * 4;
  ls = (64 * jp + amax + 1 + kHlFinOut - 1) / kHlFinOut * kHlFinOut;
  return ls + 8;  // npw
}

// the decoder widths the rows kernel is instantiated for: H / 64 columns per lane in {1, 2, 4, 8}
inline bool hl_width_ok(int64_t H) {
  return H == 64 || H == 128 || H == 256 || H == 512;
}

template <int AMAX, bool EXACT>
static void launch_heads_loss(hipStream_t s, const HeadsLossParams& P, int G, int cpl) {
  const size_t lds = sizeof(float) * 4 * 64 * ((cpl * (AMAX + 2) + 3) / 4 * 4);
  const dim3 g(G), b(256);
  switch (cpl) {
    case 1: hipLaunchKernelGGL((heads_loss_kernel<AMAX, EXACT, 1, 4>), g, b, lds, s, P); break;
    case 2: hipLaunchKernelGGL((heads_loss_kernel<AMAX, EXACT, 2, 4>), g, b, lds, s, P); break;
    case 4: hipLaunchKernelGGL((heads_loss_kernel<AMAX, EXACT, 4, 4>), g, b, lds, s, P); break;
    case 8: hipLaunchKernelGGL((heads_loss_kernel<AMAX, EXACT, 8, 4>), g, b, lds, s, P); break;
    default: break;  // rejected by hl_width_ok before the launch
  }
}

}  // namespace ocppo

extern "C" size_t ocppo_heads_loss_workspace_bytes(int64_t M, int64_t H, int64_t A) {
  if (M < 1 || H < 1 || A < 1) return 0;
  int64_t G, ls;
  const int64_t npw = ocppo::hl_layout(M, H, A, G, ls);
  return static_cast<size_t>(G * npw) * sizeof(float);
}

// validates, launches the rows kernel and fills the finish record
static int heads_loss_rows(ocppo_stream_t stream, const float* h, int64_t M, int64_t H,
                           const float* w_actor, const float* b_actor, const float* w_critic,
                           const float* b_critic, int64_t A, const int64_t* mb_actions,
                           const float* mb_logprobs, const float* mb_advantages,
                           const float* mb_returns, const float* mb_values,
                           const float* adv_stats, double clip_coef, double ent_coef,
                           double vf_coef, int norm_adv, int clip_vloss, float* gp, float* db_h,
                           float* dwa, float* dwc, float* dba, float* dbc, float* stats,
                           float* dlogits, float* dvalue, void* workspace,
                           size_t workspace_bytes, HlFinish& fin) {
  OCPPO_REQUIRE(M >= 1 && M <= INT32_MAX && hl_width_ok(H) && A >= 1 && A <= 7,
                "ocppo_heads_loss_fwd_bwd: bad sizes M=%lld H=%lld A=%lld (H in {64, 128, 256, "
                "512}, 1 <= A <= 7)", (long long)M, (long long)H, (long long)A);
  OCPPO_REQUIRE(h && w_actor && b_actor && w_critic && b_critic && mb_actions && mb_logprobs &&
                    mb_advantages && mb_returns && mb_values && gp && dwa && dwc && dba && dbc &&
                    stats && (!norm_adv || adv_stats) && (!dlogits == !dvalue),
                "ocppo_heads_loss_fwd_bwd: null pointer");
  OCPPO_REQUIRE(aligned16(h) && aligned16(gp) && aligned16(w_actor) && aligned16(w_critic),
                "ocppo_heads_loss_fwd_bwd: h / gp / weights must be 16-B aligned");
  if (!workspace || workspace_bytes < ocppo_heads_loss_workspace_bytes(M, H, A))
    return fail(OCPPO_E_WORKSPACE, "ocppo_heads_loss_fwd_bwd: workspace needs %zu bytes, got %zu",
                ocppo_heads_loss_workspace_bytes(M, H, A), workspace_bytes);
  int64_t G, ls, rpw;
  const int64_t npw = hl_layout(M, H, A, G, ls, &rpw);
  HeadsLossParams P;
  LossParams& L = P.L;
  L.logits = nullptr;
  L.new_value = nullptr;
  L.mb_inds = nullptr;
  L.b_actions = mb_actions;
  L.b_logprobs = mb_logprobs;
  L.b_adv = mb_advantages;
  L.b_ret = mb_returns;
  L.b_val = mb_values;
  L.adv_stats = adv_stats;
  L.dlogits = dlogits;
  L.dvalue = dvalue;
  L.stats = stats;
  L.ticket = nullptr;
  L.partials = nullptr;
  L.gpartials = nullptr;
  L.M = M;
  L.A = static_cast<int>(A);
  L.norm_adv = norm_adv ? 1 : 0;
  L.clip_vloss = clip_vloss ? 1 : 0;
  L.clip = static_cast<float>(clip_coef);
  L.clip_lo = static_cast<float>(1.0 - clip_coef);
  L.clip_hi = static_cast<float>(1.0 + clip_coef);
  L.ent_coef = static_cast<float>(ent_coef);
  L.vf_coef = static_cast<float>(vf_coef);
  const float fm = static_cast<float>(M);
  L.g_pg = 1.0f / fm;  // the upstream grads of ocppo_ppo_loss_fwd_bwd (mean() backward)
  L.g_h = (-1.0f * L.ent_coef) / fm;
  L.g_v = (L.vf_coef * 0.5f) / fm;
  L.inv_m = 1.0f / fm;
  P.h = h;
  P.H = H;
  P.wa = w_actor;
  P.ba = b_actor;
  P.wc = w_critic;
  P.bc = b_critic;
  P.gp = gp;
  P.partials = static_cast<float*>(workspace);
  P.npw = npw;
  P.rows_per_wg = static_cast<int>(rpw);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const int cpl = static_cast<int>(H / 64);
  switch (A) {
    case 4: launch_heads_loss<4, true>(s, P, (int)G, cpl); break;
    case 6: launch_heads_loss<6, true>(s, P, (int)G, cpl); break;
    default: launch_heads_loss<7, false>(s, P, (int)G, cpl); break;
  }
  if (int rc = check_launch("ocppo_heads_loss_fwd_bwd")) return rc;
  fin = HlFinish{static_cast<const float*>(workspace), (int)G, (int)A, hl_amax(A), cpl,
                 npw, ls, H, db_h, dwa, dwc, dba, dbc, L,
                 static_cast<int>((npw + kHlFinOut - 1) / kHlFinOut)};
  return OCPPO_OK;
}

extern "C" int ocppo_heads_loss_fwd_bwd(
    ocppo_stream_t stream, const float* h, int64_t M, int64_t H, const float* w_actor,
    const float* b_actor, const float* w_critic, const float* b_critic, int64_t A,
    const int64_t* mb_actions, const float* mb_logprobs, const float* mb_advantages,
    const float* mb_returns, const float* mb_values, const float* adv_stats, double clip_coef,
    double ent_coef, double vf_coef, int norm_adv, int clip_vloss, float* gp, float* db_h,
    float* dwa, float* dwc, float* dba, float* dbc, float* stats, float* dlogits, float* dvalue,
    void* workspace, size_t workspace_bytes) {
  HlFinish fin;
  if (int rc = heads_loss_rows(stream, h, M, H, w_actor, b_actor, w_critic, b_critic, A,
                               mb_actions, mb_logprobs, mb_advantages, mb_returns, mb_values,
                               adv_stats, clip_coef, ent_coef, vf_coef, norm_adv, clip_vloss, gp,
                               db_h, dwa, dwc, dba, dbc, stats, dlogits, dvalue, workspace,
                               workspace_bytes, fin))
    return rc;
  hipLaunchKernelGGL(heads_loss_finish_kernel, dim3(fin.blocks), dim3(256), 0, as_stream(stream),
                     fin);
  return check_launch("ocppo_heads_loss_fwd_bwd/finish");
}

extern "C" int ocppo_heads_loss_rows(
    ocppo_stream_t stream, const float* h, int64_t M, int64_t H, const float* w_actor,
    const float* b_actor, const float* w_critic, const float* b_critic, int64_t A,
    const int64_t* mb_actions, const float* mb_logprobs, const float* mb_advantages,
    const float* mb_returns, const float* mb_values, const float* adv_stats, double clip_coef,
    double ent_coef, double vf_coef, int norm_adv, int clip_vloss, float* gp, float* db_h,
    float* dwa, float* dwc, float* dba, float* dbc, float* stats, float* dlogits, float* dvalue,
    void* workspace, size_t workspace_bytes, ocppo_deferred_finish_t* finish) {
  OCPPO_REQUIRE(finish, "ocppo_heads_loss_rows: null finish record");
  DeferredFinish d;
  d.tag = kDeferHeads;
  if (int rc = heads_loss_rows(stream, h, M, H, w_actor, b_actor, w_critic, b_critic, A,
                               mb_actions, mb_logprobs, mb_advantages, mb_returns, mb_values,
                               adv_stats, clip_coef, ent_coef, vf_coef, norm_adv, clip_vloss, gp,
                               db_h, dwa, dwc, dba, dbc, stats, dlogits, dvalue, workspace,
                               workspace_bytes, d.f))
    return rc;
  memset(finish, 0, sizeof(*finish));
  memcpy(finish, &d, sizeof(d));
  return OCPPO_OK;
}

static int deferred_of(const ocppo_deferred_finish_t* finish, DeferredFinish& d,
                       const char* who) {
  OCPPO_REQUIRE(finish, "%s: null finish record", who);
  memcpy(&d, finish, sizeof(d));
  OCPPO_REQUIRE(d.tag == kDeferHeads, "%s: not a finish record of ocppo_heads_loss_rows", who);
  return OCPPO_OK;
}

namespace ocppo {
int wgrad_finish_run(hipStream_t s, const ocppo_deferred_finish_t* finish);  // ocppo_linear_bwd.hip
}

extern "C" int ocppo_deferred_finish_run(ocppo_stream_t stream,
                                         const ocppo_deferred_finish_t* finish) {
  OCPPO_REQUIRE(finish, "ocppo_deferred_finish_run: null finish record");
  clear_stale_error();
  if (ocppo::wgrad_finish_run(as_stream(stream), finish))
    return check_launch("ocppo_deferred_finish_run");
  DeferredFinish d;
  if (int rc = deferred_of(finish, d, "ocppo_deferred_finish_run")) return rc;
  hipLaunchKernelGGL(heads_loss_finish_kernel, dim3(d.f.blocks), dim3(256), 0, as_stream(stream),
                     d.f);
  return check_launch("ocppo_deferred_finish_run");
}

extern "C" int ocppo_sum_splits_finish(ocppo_stream_t stream, const float* part, int64_t S,
                                       int64_t n, float* out,
                                       const ocppo_deferred_finish_t* finish) {
  OCPPO_REQUIRE(n >= 4 && n % 4 == 0 && (S == 1 || S == 2 || S == 4 || S == 8 || S == 16),
                "ocppo_sum_splits_finish: bad sizes S=%lld n=%lld (S in {1,2,4,8,16}, n %% 4 == 0)",
                (long long)S, (long long)n);
  OCPPO_REQUIRE(part && out, "ocppo_sum_splits_finish: null pointer");
  OCPPO_REQUIRE(aligned16(part) && aligned16(out),
                "ocppo_sum_splits_finish: part and out must be 16-B aligned");
  DeferredFinish d;
  if (int rc = deferred_of(finish, d, "ocppo_sum_splits_finish")) return rc;
  clear_stale_error();
  const int64_t n4 = n / 4;
  const int nsb = grid_for(n4, 256);
  const dim3 grid(static_cast<unsigned>(nsb + d.f.blocks)), block(256);
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int ns = nsb;
  hipStream_t s = as_stream(stream);
  switch (S) {
    case 1: hipLaunchKernelGGL(sum_splits_hlfin_kernel<1>, grid, block, 0, s, p4, n4, o4, ns, d.f); break;
    case 2: hipLaunchKernelGGL(sum_splits_hlfin_kernel<2>, grid, block, 0, s, p4, n4, o4, ns, d.f); break;
    case 4: hipLaunchKernelGGL(sum_splits_hlfin_kernel<4>, grid, block, 0, s, p4, n4, o4, ns, d.f); break;
    case 8: hipLaunchKernelGGL(sum_splits_hlfin_kernel<8>, grid, block, 0, s, p4, n4, o4, ns, d.f); break;
    default: hipLaunchKernelGGL(sum_splits_hlfin_kernel<16>, grid, block, 0, s, p4, n4, o4, ns, d.f); break;
  }
  return check_launch("ocppo_sum_splits_finish");
}

// ---- torch's exponential_ on its own (ocppo_philox.h) ---------------------------------------------
namespace ocppo {
__global__ __launch_bounds__(256) void philox_exponential_kernel(float* __restrict__ out,
                                                                 int64_t numel, PhiloxNoise pn) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < numel;
       i += stride)
    out[i] = philox_noise(pn, i);
}
// steps draws of one shape back to back: out[t, i] = draw t (philox offset + t * increment)
__global__ __launch_bounds__(256) void philox_exponential_steps_kernel(float* __restrict__ out,
                                                                       int64_t numel,
                                                                       int64_t increment,
                                                                       PhiloxNoise pn) {
  const int64_t t = blockIdx.y;
  pn.step_offset += t * increment;
  float* o = out + t * numel;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < numel;
       i += stride)
    o[i] = philox_noise(pn, i);
}
}  // namespace ocppo

extern "C" int ocppo_philox_exponential_steps(ocppo_stream_t stream, float* out, int64_t numel,
                                              int64_t steps, const int64_t* philox_state,
                                              int64_t philox_offset, int64_t increment,
                                              int64_t philox_stride) {
  OCPPO_REQUIRE(numel >= 1 && steps >= 1 && steps <= 65535 && increment >= 0 && philox_stride >= 1,
                "ocppo_philox_exponential_steps: bad sizes numel=%lld steps=%lld", (long long)numel,
                (long long)steps);
  OCPPO_REQUIRE(out && philox_state, "ocppo_philox_exponential_steps: null pointer");
  clear_stale_error();
  int64_t gx = ceil_div(numel, 256);
  gx = gx < 1024 ? gx : 1024;
  hipLaunchKernelGGL(philox_exponential_steps_kernel,
                     dim3(static_cast<unsigned>(gx), static_cast<unsigned>(steps)), dim3(256), 0,
                     as_stream(stream), out, numel, increment,
                     PhiloxNoise{philox_state, philox_offset, philox_stride});
  return check_launch("ocppo_philox_exponential_steps");
}

extern "C" int ocppo_torch_exponential_geometry(int64_t numel, int64_t cus,
                                                int64_t max_threads_per_cu, int64_t* stride,
                                                int64_t* offset_increment) {
  OCPPO_REQUIRE(numel > 0 && cus > 0 && max_threads_per_cu >= 256 && stride && offset_increment,
                "ocppo_torch_exponential_geometry: bad arguments");
  // ATen calc_execution_policy: 256-thread blocks, grid capped at CUs * (threads per CU / 256),
  // ((numel - 1) / (256 * grid * 4) + 1) * 4 philox offsets per draw (unroll 4: float4 uniforms)
  int64_t grid = ceil_div(numel, 256);
  const int64_t cap = cus * (max_threads_per_cu / 256);
  if (grid > cap) grid = cap;
  *stride = 256 * grid;
  *offset_increment = ((numel - 1) / (*stride * 4) + 1) * 4;
  return OCPPO_OK;
}

extern "C" int ocppo_philox_exponential(ocppo_stream_t stream, float* out, int64_t numel,
                                        const int64_t* philox_state, int64_t philox_offset,
                                        int64_t philox_stride) {
  OCPPO_REQUIRE(numel >= 0, "ocppo_philox_exponential: bad size");
  if (numel == 0) return OCPPO_OK;
  OCPPO_REQUIRE(out && philox_state, "ocppo_philox_exponential: null pointer");
  OCPPO_REQUIRE(philox_stride > 0 && philox_stride % 256 == 0 && philox_offset >= 0,
                "ocppo_philox_exponential: bad philox stride %lld / offset %lld",
                (long long)philox_stride, (long long)philox_offset);
  clear_stale_error();
  const dim3 grid(static_cast<unsigned>(grid_for(numel, 256))), block(256);
  hipLaunchKernelGGL(philox_exponential_kernel, grid, block, 0, as_stream(stream), out, numel,
                     PhiloxNoise{philox_state, philox_offset, philox_stride});
  return check_launch("ocppo_philox_exponential");
}
