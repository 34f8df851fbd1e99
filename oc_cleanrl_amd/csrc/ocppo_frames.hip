// Frame-deduplicated PPObj minibatch encoder (obs_mode "obj"): the update's forward/backward of
// cleanrl/ppo_atari_oc.py:566 `agent.get_action_and_value(b_obs[mb_inds], ...)` through the
// per-frame Linear encoder of architectures/ppo.py:60-84.
//
// The PPObj encoder acts on every stacked frame alone, and the W frames of a stored observation
// obs[t, n] are frames of env n's timeline: slot k holds the frame of step s = t - (W-1) + k, or,
// when the env was reset at step r in (t-(W-1), t] (dones[r, n] = 1: obs[r] is the reset stack,
// every slot the first frame), the frame of step max(s, r). A minibatch of M samples therefore
// needs the encodings of far fewer than M*W distinct frames (about 0.68 of the env-steps when a
// quarter of the batch is drawn at random and W = 4): the trainer encodes the C distinct frames
// of each minibatch once (a fixed capacity C per minibatch, planned on the host from the
// permutation), expands them to [M, W, E] for the decoder, and in the backward pass sums each
// frame's W-slot gradients back onto its single row. Same math as encoding every slot (the rows
// are the same frames); the weight-gradient sums group the uses of a frame first, so the f32
// summation order differs from autograd's.
//
// Timeline id of a frame: u = (s + W - 1) * N + n, s in [-(W-1), T-1]; frames with s < 0 are the
// older slots of obs[0] (the previous iteration's last stack), s >= 0 the newest slot of obs[s].
//
// All three kernels are HBM streams (16-B accesses, one row segment per lane); the per-row index
// work is a handful of scalar loads in the block prologue.
#include "ocppo_common.h"

namespace ocppo {

constexpr int kFramesMaxW = 16;

// Latest reset step in (t-(W-1), t] of env n, or INT_MIN when there is none.
// the latest r in (t - (W-1), t] with dones[r, n] != 0 (INT32_MIN: none). The W - 1 loads are
// independent (no early exit): issued together, one memory round trip instead of up to W - 1
// dependent ones on the scatter's and the row table's setup path.
__device__ __forceinline__ int latest_reset(const float* __restrict__ dones, int t, int64_t n,
                                            int64_t N, int W) {
  int res = INT32_MIN;
#pragma unroll
  for (int i = kFramesMaxW - 2; i >= 0; --i) {  // r = t - i, oldest first: the last hit wins
    const int r = t - i;
    if (i <= W - 2 && r >= 0 && dones[r * N + n] != 0.f) res = r;
  }
  return res;
}

// The decoder's row table (frames_expand_index_kernel's) made by workgroups [gblocks, grid) of
// the same launch, beside the gather: both only read the plan, so they need no ordering
struct ExpandIdx {
  const int32_t* pos_of;
  const int64_t* perm;
  int64_t M;
  const float* dones;
  int32_t* idx;  // NULL: no row table in this launch
  int gblocks;
};

// x_out[c, :] = f32(frame of timeline id uniq[c]) (zeros for padding ids < 0)
template <int DT>
__global__ __launch_bounds__(256) void frames_gather_kernel(const void* __restrict__ obs,
                                                            int64_t N, int W, int64_t F,
                                                            const int32_t* __restrict__ uniq,
                                                            int64_t C, float* __restrict__ x_out) {
  const int64_t total = C * F;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
       g += stride) {
    const int64_t c = g / F;
    const int64_t f = g - c * F;
    const int32_t u = uniq[c];
    float v = 0.f;
    if (u >= 0) {
      const int64_t s = u / N - (W - 1);
      const int64_t n = u - (s + W - 1) * N;
      const int64_t src = s >= 0 ? ((s * N + n) * W + (W - 1)) * F + f
                                 : ((n * W) + (W - 1 + s)) * F + f;
      v = Elem<DT>::load(static_cast<const typename Elem<DT>::T*>(obs), src);
    }
    x_out[g] = v;
  }
}

// frames_gather + the encoder's first Linear(+ReLU) (F <= 16 inputs): the update's first layer
// over the C distinct frames, x written for its backward (ocppo_relu_bias_wgrad) and
// h = act(x W^T + b) in the same pass -- one launch instead of the gather and a K = F BLAS GEMM
// whose 11.8 MB output dominates. Workgroup = 16 frames; W and b staged in LDS; thread = (frame,
// 4-column group), products summed over f in order with fmaf, then + b, then ReLU.
constexpr int kGlRows = 32;  // two rows per thread (r, r + 16) share every W read
constexpr int kGlCols = 64;  // columns per workgroup (16 float4 groups): grid.y = N1 / 64
constexpr int kGlMaxF = 16;
constexpr int kGlMaxN = 1024;

// Workgroup = 32 frames x 64 columns, thread = 2 frames x one float4 column group. LDS: the
// workgroup's W^T slice [F][64] (float4 reads by consecutive column groups: conflict-free), its
// b slice, the 32 gathered rows (the column-block-0 workgroups also write x_out).
template <int DT, bool RELU>
__global__ __launch_bounds__(256) void frames_gather_linear_kernel(
    const void* __restrict__ obs, int64_t N, int W, int F, const int32_t* __restrict__ uniq,
    int64_t C, const float* __restrict__ w, const float* __restrict__ b, int N1,
    float* __restrict__ x_out, float* __restrict__ h_out, ExpandIdx) {
  __shared__ float4 wt4[kGlMaxF * kGlCols / 4];
  __shared__ float4 bs4[kGlCols / 4];
  __shared__ float xs[kGlRows][kGlMaxF];
  float* wt = reinterpret_cast<float*>(wt4);
  float* bs = reinterpret_cast<float*>(bs4);
  const int tid = threadIdx.x;
  const int n0 = blockIdx.y * kGlCols;
  for (int i = tid; i < kGlCols * F; i += 256) {
    const int f = i / kGlCols, n = i - f * kGlCols;
    wt[i] = n0 + n < N1 ? w[(n0 + n) * F + f] : 0.f;
  }
  if (tid < kGlCols) bs[tid] = (b && n0 + tid < N1) ? b[n0 + tid] : 0.f;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * kGlRows;
  for (int i = tid; i < kGlRows * F; i += 256) {
    const int r = i / F, f = i - r * F;
    const int64_t c = c0 + r;
    float v = 0.f;
    if (c < C) {
      const int32_t u = uniq[c];
      if (u >= 0) {  // u < (T + W - 1) * N < 2^31 (checked on the host): 32-bit division
        const int32_t n32 = static_cast<int32_t>(N), q = u / n32;
        const int64_t sidx = q - (W - 1);
        const int64_t n = u - q * n32;
        const int64_t src = sidx >= 0 ? ((sidx * N + n) * W + (W - 1)) * F + f
                                      : ((n * W) + (W - 1 + sidx)) * F + f;
        v = Elem<DT>::load(static_cast<const typename Elem<DT>::T*>(obs), src);
      }
      if (blockIdx.y == 0) x_out[c * F + f] = v;
    }
    xs[r][f] = v;
  }
  __syncthreads();
  const int r = tid >> 4, q = tid & 15;
  const int64_t ca = c0 + r, cb = c0 + r + 16;
  const int col = n0 + 4 * q;
  if (ca >= C || col >= N1) return;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f), bb = a;
#pragma unroll
  for (int f = 0; f < kGlMaxF; ++f) {
    if (f < F) {
      const float xa = xs[r][f], xb = xs[r + 16][f];
      const float4 wv = wt4[f * (kGlCols / 4) + q];
      a.x = fmaf(xa, wv.x, a.x); a.y = fmaf(xa, wv.y, a.y);
      a.z = fmaf(xa, wv.z, a.z); a.w = fmaf(xa, wv.w, a.w);
      bb.x = fmaf(xb, wv.x, bb.x); bb.y = fmaf(xb, wv.y, bb.y);
      bb.z = fmaf(xb, wv.z, bb.z); bb.w = fmaf(xb, wv.w, bb.w);
    }
  }
  const float4 bv = bs4[q];
  a.x += bv.x; a.y += bv.y; a.z += bv.z; a.w += bv.w;
  bb.x += bv.x; bb.y += bv.y; bb.z += bv.z; bb.w += bv.w;
  if (RELU) {
    a = relu_f4(a);
    bb = relu_f4(bb);
  }
  *reinterpret_cast<float4*>(h_out + ca * N1 + col) = a;
  if (cb < C) *reinterpret_cast<float4*>(h_out + cb * N1 + col) = bb;
}

// h[i, k, :] = enc[pos_of[u(i, k)], :] for the M samples perm[0..M) (b = t*N + n)
template <int VEC>
__global__ __launch_bounds__(256) void frames_expand_kernel(
    const float* __restrict__ enc, int64_t E, const int32_t* __restrict__ pos_of,
    const int64_t* __restrict__ perm, int64_t M, const float* __restrict__ dones, int64_t N,
    int W, float* __restrict__ h_out) {
  __shared__ int32_t src_row[kFramesMaxW];
  const int64_t groups = W * E / VEC;
  for (int64_t i = blockIdx.x; i < M; i += gridDim.x) {
    __syncthreads();  // src_row of the previous row is no longer read
    if (threadIdx.x < W) {
      const int64_t b = perm[i];
      const int t = static_cast<int>(b / N);
      const int64_t n = b - t * N;
      const int r = latest_reset(dones, t, n, N, W);
      int s = t - (W - 1) + static_cast<int>(threadIdx.x);
      s = s > r ? s : r;
      src_row[threadIdx.x] = pos_of[(s + W - 1) * N + n];
    }
    __syncthreads();
    float* dst = h_out + i * W * E;
    for (int64_t q = threadIdx.x; q < groups; q += blockDim.x) {
      const int64_t e = q * VEC;
      const int k = static_cast<int>(e / E);
      const int64_t col = e - k * E;
      float v[VEC];
      VecIO<OCPPO_F32, VEC>::load(enc, src_row[k] * E + col, v);
      VecIO<OCPPO_F32, VEC>::store(dst, e, v);
    }
  }
}

// idx[i, k] = pos_of[u(i, k)]: frames_expand's source rows alone (the update's decoder GEMMs
// gather their operand rows through it instead of reading a materialised [M, W, E] copy)
__global__ __launch_bounds__(256) void frames_expand_index_kernel(
    const int32_t* __restrict__ pos_of, const int64_t* __restrict__ perm, int64_t M,
    const float* __restrict__ dones, int64_t N, int W, int32_t* __restrict__ idx) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= M * W) return;
  const int64_t i = j / W;
  const int k = static_cast<int>(j - i * W);
  const int64_t b = perm[i];
  const int t = static_cast<int>(b / N);
  const int64_t n = b - t * N;
  const int r = latest_reset(dones, t, n, N, W);
  int s = t - (W - 1) + k;
  s = s > r ? s : r;
  idx[j] = pos_of[(s + W - 1) * N + n];
}

// denc[c, :] = sum over the (sample row i, slot k) uses of frame uniq[c] in minibatch `mb` of
// dh[i, k, :], in the fixed order (t ascending, k ascending); zeros for padding ids.
template <int VEC>
__global__ __launch_bounds__(128) void frames_scatter_kernel(
    const float* __restrict__ dh, int64_t M, int64_t E, const int32_t* __restrict__ uniq,
    int64_t C, const int32_t* __restrict__ inv, int64_t mb, const float* __restrict__ dones,
    int64_t T, int64_t N, int W, float* __restrict__ denc) {
  // slot i * W + k: the use of this frame by sample t = s + i at stack slot k (-1: none); thread
  // i < W resolves sample t = s + i (its inv entry and latest reset) in parallel with the others
  __shared__ int64_t uses[kFramesMaxW * kFramesMaxW];
  const int64_t groups = E / VEC;
  const int WW = W * W;
  for (int64_t c = blockIdx.x; c < C; c += gridDim.x) {
    __syncthreads();  // the previous row's use slots are no longer read
    for (int q = threadIdx.x; q < WW; q += blockDim.x) uses[q] = -1;
    __syncthreads();
    const int32_t u = uniq[c];
    if (u >= 0 && static_cast<int>(threadIdx.x) < W) {
      const int i = static_cast<int>(threadIdx.x);
      const int s = static_cast<int>(u / N) - (W - 1);
      const int64_t n = u - (s + W - 1) * N;
      const int t = s + i;
      if (t >= 0 && t <= T - 1) {
        const int32_t p = inv[t * N + n];
        if (p / M == mb) {
          const int64_t row = p - mb * M;
          const int r = latest_reset(dones, t, n, N, W);
          for (int k = 0; k < W; ++k) {
            int sk = t - (W - 1) + k;
            sk = sk > r ? sk : r;
            if (sk == s) uses[i * W + k] = row * W + k;
          }
        }
      }
    }
    __syncthreads();
    float* dst = denc + c * E;
    for (int64_t q = threadIdx.x; q < groups; q += blockDim.x) {
      const int64_t e = q * VEC;
      float acc[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
      for (int j = 0; j < WW; ++j) {  // (t ascending, k ascending): the fixed summation order
        const int64_t us = uses[j];
        if (us < 0) continue;
        float x[VEC];
        VecIO<OCPPO_F32, VEC>::load(dh, us * E + e, x);
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] += x[v];
      }
      VecIO<OCPPO_F32, VEC>::store(dst, e, acc);
    }
  }
}

// The same sum with the ReLU backward of the encoder's last layer fused in (its output `out`
// [C, E] is the frames' encodings): gp[c, :] = out[c, :] <= 0 ? 0 : denc[c, :] -- what
// relu_bias_grad would do next -- and the per-workgroup column sums of gp (the layer's
// bias-gradient partials, dbp [chunks, E], summed in chunk order by ocppo_sum_splits_db).
// Workgroup = kScatterFrames frames: their uses are resolved in parallel (one thread per
// (frame, candidate sample)), compacted per frame in (t, k) order into LDS sized for this W, and
// the data pass runs thread = (frame group h of kScatterGroups, float4 column group): the first
// two uses + the mask of the group's frames loaded before any is summed (almost every frame has
// one or two uses; further ones are added in order afterwards). Few registers and little LDS per
// workgroup: the use-resolution chain (uniq -> inv -> dones) of some workgroups overlaps the data
// pass of others on the same CU. MK: 0 no mask, 1 the f32 output, 2 its row-major bitmask.
#ifndef OCPPO_SCATTER_F  // experiments (tools/build_variant.py)
#define OCPPO_SCATTER_F 16
#endif
#ifndef OCPPO_SCATTER_G
#define OCPPO_SCATTER_G 4
#endif
constexpr int kScatterFrames = OCPPO_SCATTER_F;
constexpr int kScatterGroups = OCPPO_SCATTER_G;
static_assert(kScatterFrames % kScatterGroups == 0 && 256 % kScatterGroups == 0, "scatter shape");

template <int MK>
__global__ __launch_bounds__(256) void frames_scatter_relu_kernel(
    const float* __restrict__ dh, int64_t M, int64_t E, const int32_t* __restrict__ uniq,
    int64_t C, const int32_t* __restrict__ inv, int64_t mb, const float* __restrict__ dones,
    int64_t T, int64_t N, int W, const float* __restrict__ out,
    const uint32_t* __restrict__ mbits, float* __restrict__ gp, float* __restrict__ dbp) {
  constexpr int F = kScatterFrames, G = kScatterGroups, FG = F / G, QG = 256 / G;
  extern __shared__ int32_t scatter_lds[];  // uses [F][WW], list [F][WW]
  __shared__ int cnt[F];
  __shared__ float4 red[G - 1][QG];
  const int WW = W * W;
  int32_t* uses = scatter_lds;
  int32_t* list = scatter_lds + F * WW;
  const int tid = threadIdx.x;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * F;
  for (int q = tid; q < F * WW; q += blockDim.x) uses[q] = -1;
  __syncthreads();
  if (tid < F * W) {  // (frame j, candidate sample t = s + i)
    const int j = tid / W, i = tid - j * W;
    const int64_t c = c0 + j;
    const int32_t u = c < C ? uniq[c] : -1;
    if (u >= 0) {
      const int s = static_cast<int>(u / N) - (W - 1);
      const int64_t n = u - (s + W - 1) * N;
      const int t = s + i;
      if (t >= 0 && t <= T - 1) {
        const int32_t p = inv[t * N + n];
        if (p / M == mb) {
          const int32_t row = static_cast<int32_t>(p - mb * M);
          const int r = latest_reset(dones, t, n, N, W);
          for (int k = 0; k < W; ++k) {
            int sk = t - (W - 1) + k;
            sk = sk > r ? sk : r;
            if (sk == s) uses[j * WW + i * W + k] = row * W + k;
          }
        }
      }
    }
  }
  __syncthreads();
  if (tid < F) {  // compact each frame's uses, keeping the (t ascending, k ascending) order
    int m = 0;
    for (int q = 0; q < WW; ++q)
      if (uses[tid * WW + q] >= 0) list[tid * WW + m++] = uses[tid * WW + q];
    cnt[tid] = m;
  }
  __syncthreads();
  // data pass: thread = (frame group h, float4 column group qg); frames j = G p + h
  const int h = tid / QG, qg = tid % QG;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  // block-uniform trip count (the barriers below are reached by every thread); lanes past E
  // load and store nothing
  for (int64_t e0 = 0; e0 < E; e0 += QG * 4) {
    const int64_t e = e0 + static_cast<int64_t>(qg) * 4;
    const bool live = e < E;
    float4 v0[FG], v1[FG], mk[FG];
    uint32_t mb4[FG];  // the row-major bitmask's 4 bits of (frame, e .. e + 3)
#pragma unroll
    for (int p = 0; p < FG; ++p) {  // first two uses + the mask of every frame, in flight
      const int j = G * p + h;
      const int n = live ? cnt[j] : 0;
      v0[p] = n > 0 ? *reinterpret_cast<const float4*>(dh + static_cast<int64_t>(list[j * WW]) * E + e) : z;
      v1[p] = n > 1 ? *reinterpret_cast<const float4*>(dh + static_cast<int64_t>(list[j * WW + 1]) * E + e) : z;
      const bool mrow = live && c0 + j < C;
      if constexpr (MK == 2)
        mb4[p] = mrow ? (mbits[(c0 + j) * (E >> 5) + (e >> 5)] >> (e & 31)) & 0xfu : 0xfu;
      if constexpr (MK == 1)
        mk[p] = mrow ? *reinterpret_cast<const float4*>(out + (c0 + j) * E + e)
                     : make_float4(1.f, 1.f, 1.f, 1.f);
    }
    float4 cs = z;
#pragma unroll
    for (int p = 0; p < FG; ++p) {
      const int j = G * p + h;
      const int64_t c = c0 + j;
      if (c >= C || !live) continue;
      const int n = cnt[j];
      float4 a = z;
      if (n > 0) { a.x += v0[p].x; a.y += v0[p].y; a.z += v0[p].z; a.w += v0[p].w; }
      if (n > 1) { a.x += v1[p].x; a.y += v1[p].y; a.z += v1[p].z; a.w += v1[p].w; }
      for (int m = 2; m < n; ++m) {
        const float4 x = *reinterpret_cast<const float4*>(dh + static_cast<int64_t>(list[j * WW + m]) * E + e);
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      }
      if constexpr (MK == 1) {
        a.x = mk[p].x <= 0.f ? 0.f : a.x; a.y = mk[p].y <= 0.f ? 0.f : a.y;
        a.z = mk[p].z <= 0.f ? 0.f : a.z; a.w = mk[p].w <= 0.f ? 0.f : a.w;
      }
      if constexpr (MK == 2) {
        const uint32_t m4 = mb4[p];
        a.x = (m4 & 1u) ? a.x : 0.f; a.y = (m4 & 2u) ? a.y : 0.f;
        a.z = (m4 & 4u) ? a.z : 0.f; a.w = (m4 & 8u) ? a.w : 0.f;
      }
      *reinterpret_cast<float4*>(gp + c * E + e) = a;
      cs.x += a.x; cs.y += a.y; cs.z += a.z; cs.w += a.w;
    }
    if (dbp) {  // the frame groups of this column group, added in h order
      if (h > 0) red[h - 1][qg] = cs;
      __syncthreads();
      if (h == 0 && live) {
#pragma unroll
        for (int q = 0; q < G - 1; ++q) {
          const float4 o = red[q][qg];
          cs.x += o.x; cs.y += o.y; cs.z += o.z; cs.w += o.w;
        }
        *reinterpret_cast<float4*>(dbp + static_cast<int64_t>(blockIdx.x) * E + e) = cs;
      }
      __syncthreads();
    }
  }
}

// Wide form for N1 <= 256 (PPObj's first encoder layer, 12 -> 256): a workgroup owns RW frames x
// ALL N1 columns, so every frame is gathered once (not once per 64-column block) and the W^T
// [F][N1] image is staged once per workgroup from contiguous reads of W. Thread = one float4
// column group (q = tid % 64) x RW / 4 frames (r = tid / 64 + 4 i): a wave stores whole 1-KB
// rows of h (one 256-column row per store instruction), and reads W^T as one float4 per f,
// reused for all its frames. Same products in the same order as the narrow form (fmaf over f,
// + b, ReLU): bit-identical outputs.
#ifndef OCPPO_GW_ROWS  // experiments (tools/build_variant.py)
#define OCPPO_GW_ROWS 16
#endif
constexpr int kGwRows = OCPPO_GW_ROWS;
constexpr int kGwCols = 256;
template <int DT, bool RELU>
__global__ __launch_bounds__(256) void frames_gather_linear_wide_kernel(
    const void* __restrict__ obs, int64_t N, int W, int F, const int32_t* __restrict__ uniq,
    int64_t C, const float* __restrict__ w, const float* __restrict__ b, int N1,
    float* __restrict__ x_out, float* __restrict__ h_out, ExpandIdx ei) {
  if (ei.idx != nullptr && static_cast<int>(blockIdx.x) >= ei.gblocks) {  // workgroup-uniform
    const int64_t j = static_cast<int64_t>(blockIdx.x - ei.gblocks) * blockDim.x + threadIdx.x;
    if (j >= ei.M * W) return;
    const int64_t i = j / W;
    const int k = static_cast<int>(j - i * W);
    const int64_t bb = ei.perm[i];
    const int t = static_cast<int>(bb / N);
    const int64_t n = bb - t * N;
    const int r = latest_reset(ei.dones, t, n, N, W);
    int s = t - (W - 1) + k;
    s = s > r ? s : r;
    ei.idx[j] = ei.pos_of[(s + W - 1) * N + n];
    return;
  }
  __shared__ float4 wt4[kGlMaxF * kGwCols / 4];
  __shared__ float4 bs4[kGwCols / 4];
  __shared__ float xs[kGwRows][kGlMaxF];
  float* wt = reinterpret_cast<float*>(wt4);
  float* bs = reinterpret_cast<float*>(bs4);
  const int tid = threadIdx.x;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * kGwRows;
  for (int i = tid; i < kGwRows * F; i += 256) {  // the gather first: its loads go out early
    const int r = i / F, f = i - r * F;
    const int64_t c = c0 + r;
    float v = 0.f;
    if (c < C) {
      const int32_t u = uniq[c];
      if (u >= 0) {  // u < (T + W - 1) * N < 2^31 (checked on the host): 32-bit division
        const int32_t n32 = static_cast<int32_t>(N), q = u / n32;
        const int64_t sidx = q - (W - 1);
        const int64_t n = u - q * n32;
        const int64_t src = sidx >= 0 ? ((sidx * N + n) * W + (W - 1)) * F + f
                                      : ((n * W) + (W - 1 + sidx)) * F + f;
        v = Elem<DT>::load(static_cast<const typename Elem<DT>::T*>(obs), src);
      }
      x_out[c * F + f] = v;
    }
    xs[r][f] = v;
  }
  for (int i = tid; i < N1 * F; i += 256) {  // W [N1][F] read contiguously, stored transposed
    const int n = i / F, f = i - n * F;
    wt[f * kGwCols + n] = w[i];
  }
  if (tid < kGwCols) bs[tid] = (b && tid < N1) ? b[tid] : 0.f;
  __syncthreads();
  const int q = tid & 63, r0 = tid >> 6;
  const int col = 4 * q;
  if (col >= N1) return;
  constexpr int RPT = kGwRows / 4;
  float4 acc[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int f = 0; f < kGlMaxF; ++f) {
    if (f < F) {
      const float4 wv = wt4[f * (kGwCols / 4) + q];
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const float xa = xs[r0 + 4 * i][f];
        acc[i].x = fmaf(xa, wv.x, acc[i].x); acc[i].y = fmaf(xa, wv.y, acc[i].y);
        acc[i].z = fmaf(xa, wv.z, acc[i].z); acc[i].w = fmaf(xa, wv.w, acc[i].w);
      }
    }
  }
  const float4 bv = bs4[q];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int64_t c = c0 + r0 + 4 * i;
    if (c >= C) break;
    float4 a = acc[i];
    a.x += bv.x; a.y += bv.y; a.z += bv.z; a.w += bv.w;
    if (RELU) a = relu_f4(a);
    *reinterpret_cast<float4*>(h_out + c * N1 + col) = a;
  }
}

static bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_frames_gather(ocppo_stream_t stream, const void* obs, int obs_dtype,
                                   int64_t T, int64_t N, int64_t W, int64_t F,
                                   const int32_t* uniq, int64_t C, float* x_out) {
  OCPPO_REQUIRE(T >= 1 && N >= 1 && W >= 1 && W <= kFramesMaxW && F >= 1 && C >= 0 &&
                    (T + W - 1) * N < INT32_MAX,
                "ocppo_frames_gather: bad sizes");
  if (C == 0) return OCPPO_OK;
  OCPPO_REQUIRE(obs && uniq && x_out, "ocppo_frames_gather: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const int g = grid_for(C * F, 256);
  switch (obs_dtype) {
    case OCPPO_F32:
      hipLaunchKernelGGL(frames_gather_kernel<OCPPO_F32>, dim3(g), dim3(256), 0, s, obs, N,
                         (int)W, F, uniq, C, x_out);
      break;
    case OCPPO_BF16:
      hipLaunchKernelGGL(frames_gather_kernel<OCPPO_BF16>, dim3(g), dim3(256), 0, s, obs, N,
                         (int)W, F, uniq, C, x_out);
      break;
    case OCPPO_U8:
      hipLaunchKernelGGL(frames_gather_kernel<OCPPO_U8>, dim3(g), dim3(256), 0, s, obs, N,
                         (int)W, F, uniq, C, x_out);
      break;
    default:
      return fail(OCPPO_E_INVALID, "ocppo_frames_gather: bad obs dtype %d", obs_dtype);
  }
  return check_launch("ocppo_frames_gather");
}

extern "C" int ocppo_frames_expand(ocppo_stream_t stream, const float* enc, int64_t C, int64_t E,
                                   const int32_t* pos_of, const int64_t* perm, int64_t M,
                                   const float* dones, int64_t T, int64_t N, int64_t W,
                                   float* h_out) {
  OCPPO_REQUIRE(C >= 1 && E >= 1 && M >= 0 && T >= 1 && N >= 1 && W >= 1 && W <= kFramesMaxW &&
                    (T + W - 1) * N < INT32_MAX,
                "ocppo_frames_expand: bad sizes");
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(enc && pos_of && perm && dones && h_out, "ocppo_frames_expand: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const int g = static_cast<int>(M < 8192 ? M : 8192);
  if (E % 4 == 0 && aligned16(enc) && aligned16(h_out))
    hipLaunchKernelGGL(frames_expand_kernel<4>, dim3(g), dim3(256), 0, s, enc, E, pos_of, perm, M,
                       dones, N, (int)W, h_out);
  else
    hipLaunchKernelGGL(frames_expand_kernel<1>, dim3(g), dim3(256), 0, s, enc, E, pos_of, perm, M,
                       dones, N, (int)W, h_out);
  return check_launch("ocppo_frames_expand");
}

extern "C" int ocppo_frames_expand_index(ocppo_stream_t stream, const int32_t* pos_of,
                                         const int64_t* perm, int64_t M, const float* dones,
                                         int64_t T, int64_t N, int64_t W, int32_t* idx) {
  OCPPO_REQUIRE(M >= 0 && T >= 1 && N >= 1 && W >= 1 && W <= kFramesMaxW &&
                    (T + W - 1) * N < INT32_MAX && M * W < INT32_MAX,
                "ocppo_frames_expand_index: bad sizes");
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(pos_of && perm && dones && idx, "ocppo_frames_expand_index: null pointer");
  clear_stale_error();
  hipLaunchKernelGGL(frames_expand_index_kernel, dim3(static_cast<unsigned>(ceil_div(M * W, 256))),
                     dim3(256), 0, as_stream(stream), pos_of, perm, M, dones, N, (int)W, idx);
  return check_launch("ocppo_frames_expand_index");
}

extern "C" int ocppo_frames_scatter(ocppo_stream_t stream, const float* dh, int64_t M, int64_t E,
                                    const int32_t* uniq, int64_t C, const int32_t* inv,
                                    int64_t mb, const float* dones, int64_t T, int64_t N,
                                    int64_t W, float* denc_out) {
  OCPPO_REQUIRE(M >= 1 && E >= 1 && C >= 0 && mb >= 0 && T >= 1 && N >= 1 && W >= 1 &&
                    W <= kFramesMaxW && (T + W - 1) * N < INT32_MAX && T * N < INT32_MAX,
                "ocppo_frames_scatter: bad sizes");
  if (C == 0) return OCPPO_OK;
  OCPPO_REQUIRE(dh && uniq && inv && dones && denc_out, "ocppo_frames_scatter: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const int g = static_cast<int>(C < 16384 ? C : 16384);
  if (E % 4 == 0 && aligned16(dh) && aligned16(denc_out))
    hipLaunchKernelGGL(frames_scatter_kernel<4>, dim3(g), dim3(128), 0, s, dh, M, E, uniq, C, inv,
                       mb, dones, T, N, (int)W, denc_out);
  else
    hipLaunchKernelGGL(frames_scatter_kernel<1>, dim3(g), dim3(128), 0, s, dh, M, E, uniq, C, inv,
                       mb, dones, T, N, (int)W, denc_out);
  return check_launch("ocppo_frames_scatter");
}

extern "C" int64_t ocppo_frames_scatter_chunks(int64_t C) {
  return C < 1 ? 1 : (C + ocppo::kScatterFrames - 1) / ocppo::kScatterFrames;
}

extern "C" int ocppo_frames_scatter_relu(ocppo_stream_t stream, const float* dh, int64_t M,
                                         int64_t E, const int32_t* uniq, int64_t C,
                                         const int32_t* inv, int64_t mb, const float* dones,
                                         int64_t T, int64_t N, int64_t W, const float* out,
                                         const uint32_t* mbits, float* gp_out, float* dbp) {
  OCPPO_REQUIRE(!mbits || E % 32 == 0,
                "ocppo_frames_scatter_relu: the row-major bitmask needs E %% 32 == 0");
  OCPPO_REQUIRE(M >= 1 && E >= 4 && E % 4 == 0 && C >= 0 && mb >= 0 && T >= 1 && N >= 1 &&
                    W >= 1 && W <= kFramesMaxW && (T + W - 1) * N < INT32_MAX &&
                    T * N < INT32_MAX && M * W < INT32_MAX,
                "ocppo_frames_scatter_relu: bad sizes (E %% 4 == 0, W <= %d)", kFramesMaxW);
  if (C == 0) return OCPPO_OK;
  OCPPO_REQUIRE(dh && uniq && inv && dones && gp_out, "ocppo_frames_scatter_relu: null pointer");
  OCPPO_REQUIRE(aligned16(dh) && aligned16(gp_out) && (!out || aligned16(out)) &&
                    (!dbp || aligned16(dbp)),
                "ocppo_frames_scatter_relu: dh / out / gp / dbp must be 16-B aligned");
  clear_stale_error();
  const int64_t g = ocppo_frames_scatter_chunks(C);
  OCPPO_REQUIRE(g <= INT32_MAX, "ocppo_frames_scatter_relu: too large");
  const size_t lds = 2 * sizeof(int32_t) * kScatterFrames * W * W;
  const dim3 grid(static_cast<unsigned>(g)), block(256);
  hipStream_t s = as_stream(stream);
  if (mbits)
    hipLaunchKernelGGL(frames_scatter_relu_kernel<2>, grid, block, lds, s, dh, M, E, uniq, C, inv,
                       mb, dones, T, N, (int)W, out, mbits, gp_out, dbp);
  else if (out)
    hipLaunchKernelGGL(frames_scatter_relu_kernel<1>, grid, block, lds, s, dh, M, E, uniq, C, inv,
                       mb, dones, T, N, (int)W, out, mbits, gp_out, dbp);
  else
    hipLaunchKernelGGL(frames_scatter_relu_kernel<0>, grid, block, lds, s, dh, M, E, uniq, C, inv,
                       mb, dones, T, N, (int)W, out, mbits, gp_out, dbp);
  return check_launch("ocppo_frames_scatter_relu");
}

extern "C" int ocppo_frames_gather_linear(ocppo_stream_t stream, const void* obs, int obs_dtype,
                                          int64_t T, int64_t N, int64_t W, int64_t F,
                                          const int32_t* uniq, int64_t C, const float* w,
                                          const float* b, int64_t N1, int relu, float* x_out,
                                          float* h_out, const int32_t* pos_of,
                                          const int64_t* perm, int64_t M, const float* dones,
                                          int32_t* idx_out) {
  OCPPO_REQUIRE(T >= 1 && N >= 1 && W >= 1 && W <= kFramesMaxW && F >= 1 && F <= kGlMaxF &&
                    N1 >= 4 && N1 % 4 == 0 && N1 <= kGlMaxN && C >= 0 &&
                    (T + W - 1) * N < INT32_MAX,
                "ocppo_frames_gather_linear: bad sizes (F <= %d, N1 %% 4 == 0, N1 <= %d)",
                kGlMaxF, kGlMaxN);
  OCPPO_REQUIRE(!idx_out || (pos_of && perm && dones && M >= 1 && M * W < INT32_MAX),
                "ocppo_frames_gather_linear: the row table needs pos_of, perm, dones, M >= 1");
  if (C == 0) {
    if (!idx_out) return OCPPO_OK;
    clear_stale_error();
    hipLaunchKernelGGL(frames_expand_index_kernel, dim3(static_cast<unsigned>(ceil_div(M * W, 256))),
                       dim3(256), 0, as_stream(stream), pos_of, perm, M, dones, N, (int)W, idx_out);
    return check_launch("ocppo_frames_gather_linear/index");
  }
  OCPPO_REQUIRE(obs && uniq && w && x_out && h_out, "ocppo_frames_gather_linear: null pointer");
  OCPPO_REQUIRE(aligned16(h_out), "ocppo_frames_gather_linear: h_out must be 16-B aligned");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const bool wide = N1 <= kGwCols;
  const int64_t g = (C + (wide ? kGwRows : kGlRows) - 1) / (wide ? kGwRows : kGlRows);
  OCPPO_REQUIRE(g <= INT32_MAX, "ocppo_frames_gather_linear: too large");
  // the decoder's row table in the same launch (wide form), else in its own right after
  const bool fuse_idx = idx_out != nullptr && wide;
  const int64_t ib = fuse_idx ? ceil_div(M * W, 256) : 0;
  OCPPO_REQUIRE(g + ib <= INT32_MAX, "ocppo_frames_gather_linear: too large");
  const ExpandIdx ei{pos_of, perm, M, dones, fuse_idx ? idx_out : nullptr, static_cast<int>(g)};
  const dim3 grid(static_cast<unsigned>(g + ib),
                  wide ? 1u : static_cast<unsigned>((N1 + kGlCols - 1) / kGlCols));
  const dim3 block(256);
#define OCPPO_GL_K(KERN, DT)                                                                      \
  do {                                                                                            \
    if (relu)                                                                                     \
      hipLaunchKernelGGL((KERN<DT, true>), grid, block, 0, s, obs, N, (int)W, (int)F, uniq, C, w, \
                         b, (int)N1, x_out, h_out, ei);                                           \
    else                                                                                          \
      hipLaunchKernelGGL((KERN<DT, false>), grid, block, 0, s, obs, N, (int)W, (int)F, uniq, C,   \
                         w, b, (int)N1, x_out, h_out, ei);                                        \
  } while (0)
#define OCPPO_GL(DT)                                                                              \
  do {                                                                                            \
    if (wide) OCPPO_GL_K(frames_gather_linear_wide_kernel, DT);                                   \
    else OCPPO_GL_K(frames_gather_linear_kernel, DT);                                             \
  } while (0)
  switch (obs_dtype) {
    case OCPPO_F32: OCPPO_GL(OCPPO_F32); break;
    case OCPPO_BF16: OCPPO_GL(OCPPO_BF16); break;
    case OCPPO_U8: OCPPO_GL(OCPPO_U8); break;
    default: return fail(OCPPO_E_INVALID, "ocppo_frames_gather_linear: bad obs dtype %d", obs_dtype);
  }
#undef OCPPO_GL
#undef OCPPO_GL_K
  if (int rc = check_launch("ocppo_frames_gather_linear")) return rc;
  if (idx_out && !fuse_idx) {
    hipLaunchKernelGGL(frames_expand_index_kernel, dim3(static_cast<unsigned>(ceil_div(M * W, 256))),
                       dim3(256), 0, s, pos_of, perm, M, dones, N, (int)W, idx_out);
    return check_launch("ocppo_frames_gather_linear/index");
  }
  return OCPPO_OK;
}
