// Device-side bodies of the rollout store (frame stack + storage-dtype conversion + network copy)
// and of SB3 VecNormalize's reward normalisation, shared by the store launches
// (ocppo_rollout.hip) and the fused store + newest-frame encoder launch (ocppo_linear.hip).
#pragma once

#include "ocppo_common.h"

namespace ocppo {

// ---- rollout store ----------------------------------------------------------------------------
// obs_out[n, w, :] = w == W-1 ? frame[n, :] : done[n] ? R(n, w) : prev_obs[n, w+1, :]
// R(n, w) = reset_prev[n, w, :] when the caller passes the older W-1 frames of the env's own reset
// observation (host envs whose reset stack is not W copies of one frame: NoopReset/EpisodicLife
// steps), else frame[n, :] (FrameStack's fill of a fresh episode).
// Work split over `nblk` workgroups starting at workgroup `blk` (grid-stride).
template <int FDT, int ODT, int VEC>
__device__ __forceinline__ void store_groups(int64_t blk, int64_t nblk, const void* __restrict__ frame,
                                             const float* __restrict__ reward,
                                             const float* __restrict__ done, int64_t N, int W,
                                             int64_t D, const void* __restrict__ prev,
                                             void* __restrict__ out, float* __restrict__ net,
                                             float* __restrict__ reward_out,
                                             float* __restrict__ done_out, float net_scale,
                                             const void* __restrict__ reset_prev) {
  const int64_t DG = D / VEC;
  const int64_t groups = N * W * DG;
  const int64_t stride = nblk * blockDim.x;
  for (int64_t g = blk * blockDim.x + threadIdx.x; g < groups; g += stride) {
    const int64_t n = g / (W * DG);
    const int64_t rem = g - n * W * DG;
    const int w = static_cast<int>(rem / DG);
    const int64_t k = (rem - static_cast<int64_t>(w) * DG) * VEC;
    float v[VEC];
    if (w == W - 1)
      VecIO<FDT, VEC>::load(frame, n * D + k, v);
    else if (done[n] != 0.f)
      VecIO<FDT, VEC>::load(reset_prev ? reset_prev : frame,
                            reset_prev ? (n * (W - 1) + w) * D + k : n * D + k, v);
    else
      VecIO<ODT, VEC>::load(prev, (n * W + w + 1) * D + k, v);
    const int64_t o = (n * W + w) * D + k;
    VecIO<ODT, VEC>::store(out, o, v);
    if (net) {  // the network sees exactly what the rollout buffer holds
      float back[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) back[q] = Elem<ODT>::roundtrip(v[q]) * net_scale;
      VecIO<OCPPO_F32, VEC>::store(net, o, back);
    }
    if (g < N) {
      if (reward_out) reward_out[g] = reward[g];
      if (done_out) done_out[g] = done[g];
    }
  }
}

// Same store with the f32 network copy in channels-last order: net[n, p, w] (= NHWC for pixel
// stacks [N, W, 84, 84]; what MIOpen's NHWC convolutions read without a transpose). One thread per
// (env, VEC consecutive elements of the frame): it produces all W slots of those elements, so the
// W x VEC network values it writes are contiguous (W == 4: one 16-B store per element).
template <int FDT, int ODT, int VEC>
__device__ __forceinline__ void store_groups_cl(int64_t blk, int64_t nblk,
                                                const void* __restrict__ frame,
                                                const float* __restrict__ reward,
                                                const float* __restrict__ done, int64_t N, int W,
                                                int64_t D, const void* __restrict__ prev,
                                                void* __restrict__ out, float* __restrict__ net,
                                                float* __restrict__ reward_out,
                                                float* __restrict__ done_out, float net_scale,
                                                const void* __restrict__ reset_prev) {
  const int64_t DG = D / VEC;
  const int64_t groups = N * DG;
  const int64_t stride = nblk * blockDim.x;
  for (int64_t g = blk * blockDim.x + threadIdx.x; g < groups; g += stride) {
    const int64_t n = g / DG;
    const int64_t k = (g - n * DG) * VEC;
    const bool reset = done[n] != 0.f;
    float* dst = net + (n * D + k) * W;
    if (W == 4) {
      float v[4][VEC];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        if (w == 3 || (reset && !reset_prev))
          VecIO<FDT, VEC>::load(frame, n * D + k, v[w]);
        else if (reset)
          VecIO<FDT, VEC>::load(reset_prev, (n * 3 + w) * D + k, v[w]);
        else
          VecIO<ODT, VEC>::load(prev, (n * 4 + w + 1) * D + k, v[w]);
        VecIO<ODT, VEC>::store(out, (n * 4 + w) * D + k, v[w]);
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        float px[4] = {Elem<ODT>::roundtrip(v[0][q]) * net_scale,
                       Elem<ODT>::roundtrip(v[1][q]) * net_scale,
                       Elem<ODT>::roundtrip(v[2][q]) * net_scale,
                       Elem<ODT>::roundtrip(v[3][q]) * net_scale};
        VecIO<OCPPO_F32, 4>::store(dst, 4 * q, px);  // net is 16-B aligned (host check)
      }
    } else {
      for (int w = 0; w < W; ++w) {
        float v[VEC];
        if (w == W - 1 || (reset && !reset_prev))
          VecIO<FDT, VEC>::load(frame, n * D + k, v);
        else if (reset)
          VecIO<FDT, VEC>::load(reset_prev, (n * (W - 1) + w) * D + k, v);
        else
          VecIO<ODT, VEC>::load(prev, (n * W + w + 1) * D + k, v);
        VecIO<ODT, VEC>::store(out, (n * W + w) * D + k, v);
#pragma unroll
        for (int q = 0; q < VEC; ++q) dst[q * W + w] = Elem<ODT>::roundtrip(v[q]) * net_scale;
      }
    }
    if (g < N) {
      if (reward_out) reward_out[g] = reward[g];
      if (done_out) done_out[g] = done[g];
    }
  }
}

// ---- VecNormalize(norm_obs=False, norm_reward=True) -----------------------------------------------
// One workgroup (the reduction spans the env axis). f64 like SB3's numpy code. `out` may alias
// `reward` (in-place normalisation of a rollout row): each element is read and written by the same
// thread.
__device__ __forceinline__ void vecnorm_block(const float* reward, const float* __restrict__ done,
                                              int64_t N, double gamma, double eps, double clip,
                                              double* __restrict__ ret, double* __restrict__ rms,
                                              float* out) {
  __shared__ double scratch[16];
  __shared__ double s_var;
  double s = 0.0;
  for (int64_t n = threadIdx.x; n < N; n += blockDim.x) {
    const double r = ret[n] * gamma + static_cast<double>(reward[n]);
    ret[n] = r;
    s += r;
  }
  s = block_sum(s, scratch);
  const double bmean = s / static_cast<double>(N);
  double q = 0.0;
  for (int64_t n = threadIdx.x; n < N; n += blockDim.x) {
    const double d = ret[n] - bmean;
    q += d * d;
  }
  q = block_sum(q, scratch);
  if (threadIdx.x == 0) {
    const double bvar = q / static_cast<double>(N);
    const double bcount = static_cast<double>(N);
    const double mean = rms[0], var = rms[1], count = rms[2];
    // RunningMeanStd.update_from_moments (Chan et al. parallel merge)
    const double delta = bmean - mean;
    const double tot = count + bcount;
    const double new_mean = mean + delta * bcount / tot;
    const double m_a = var * count;
    const double m_b = bvar * bcount;
    const double m2 = m_a + m_b + delta * delta * count * bcount / (count + bcount);
    const double new_var = m2 / (count + bcount);
    rms[0] = new_mean;
    rms[1] = new_var;
    rms[2] = bcount + count;
    s_var = new_var;
  }
  __syncthreads();
  const double denom = sqrt(s_var + eps);
  for (int64_t n = threadIdx.x; n < N; n += blockDim.x) {
    double r = static_cast<double>(reward[n]) / denom;
    r = r < -clip ? -clip : (r > clip ? clip : r);
    out[n] = static_cast<float>(r);
    if (done[n] != 0.f) ret[n] = 0.0;
  }
}

}  // namespace ocppo
