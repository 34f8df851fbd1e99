// Rollout-batch Linear(+ReLU) on the f32 matrix cores: y = act(x W^T + b) for the few-hundred-row
// batches of the rollout forward (cleanrl/ppo_atari_oc.py:506 `agent.get_action_and_value(next_obs)`
// and :534 `agent.get_value(next_obs)` through the PPObj / NatureCNN-head Linear layers of
// architectures/ppo.py:60-84 and :36-46).
//
// Why not the BLAS library: at M = 128..512 rows every layer is a few hundred 16x16 output tiles;
// the library's fp32 kernels take 6-10 us per layer there (1-60 TFLOP/s, tools/exp_rollout_gemms.py)
// because their macro tiles leave most of the 256 CUs idle. Here:
//   * one workgroup per 16x16 output tile, S waves per workgroup splitting K (S chosen so the
//     launch has >= ~2048 waves, i.e. >= 2 per SIMD), partial tiles summed through LDS in wave
//     order (deterministic);
//   * v_mfma_f32_16x16x4_f32 (exact f32 products, one rounding per product, f32 accumulation);
//     a lane's fragment of a 16-wide K chunk is one float4 for both x (row-major [M, K]) and W
//     (nn.Linear's [N, K]) -- MFMA j of a chunk takes element j of every lane's float4, so the
//     4 MFMAs of a chunk together cover its 16 k values, the same permutation on A and B;
//   * K % 16 == 0: operands go through a wave-private LDS image loaded in whole 128-B lines (8
//     lines per wave instruction), fragments read back from LDS, the next 32-k group's loads in
//     flight during this group's MFMAs -- fragment-shaped global loads (16 rows x 64 B per
//     instruction) cost the address units twice the work per byte: 6.4 -> 4.7 us at
//     128 x 512 -> 1024, 11.2 -> 6.8 us at 128 x 2048 -> 512 (tools/exp_rollout_linear.py);
//   * XCD-aware tile order: workgroups b and b+8 share an XCD (round-robin dispatch), and each
//     XCD gets a contiguous range of output-column tiles, so it streams 1/8 of W through its L2;
//   * bias + ReLU fused in the epilogue (torch._addmm_activation's order: acc + b, then max(., 0)).
// Roofline: MFMA-bound in principle (2*M*N*K flops), latency-bound at these sizes.
#include "ocppo_common.h"

namespace ocppo {

typedef float floatx4 __attribute__((ext_vector_type(4)));

#ifndef OCPPO_LIN_MAX_WAVES  // K-split waves per workgroup cap (experiments: tools/build_variant.py)
#define OCPPO_LIN_MAX_WAVES 8
#endif
#ifndef OCPPO_LIN_WAVE_TARGET  // split K until the launch has this many waves
#define OCPPO_LIN_WAVE_TARGET 4096
#endif
constexpr int kLinMaxWaves = OCPPO_LIN_MAX_WAVES;

// One wave's share of a 16x16 tile: chunks [c0, c1) of 16 k values. All operand loads of a group
// of up to CH chunks are issued before its MFMAs, so the wave pays one L2 / Infinity-Cache round
// trip per group instead of one per chunk.
template <int CH, bool VEC>
__device__ __forceinline__ void linear_wave_chunks(const float* xr, const float* wr, bool rok,
                                                   bool cok, int K, int g, int c0, int c1,
                                                   floatx4& acc0, floatx4& acc1) {
  for (int cb = c0; cb < c1; cb += CH) {
    float4 a[CH], bb[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      const int k = (cb + q) * 16 + 4 * g;
      const bool live = cb + q < c1;
      if (VEC && k + 3 < K) {
        a[q] = (live && rok) ? *reinterpret_cast<const float4*>(xr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
        bb[q] = (live && cok) ? *reinterpret_cast<const float4*>(wr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        const bool lr = live && rok, lc = live && cok;
        a[q].x = (lr && k + 0 < K) ? xr[k + 0] : 0.f;
        a[q].y = (lr && k + 1 < K) ? xr[k + 1] : 0.f;
        a[q].z = (lr && k + 2 < K) ? xr[k + 2] : 0.f;
        a[q].w = (lr && k + 3 < K) ? xr[k + 3] : 0.f;
        bb[q].x = (lc && k + 0 < K) ? wr[k + 0] : 0.f;
        bb[q].y = (lc && k + 1 < K) ? wr[k + 1] : 0.f;
        bb[q].z = (lc && k + 2 < K) ? wr[k + 2] : 0.f;
        bb[q].w = (lc && k + 3 < K) ? wr[k + 3] : 0.f;
      }
    }
    // two accumulator chains (the 16x16x4 f32 MFMA's dependent latency is 40 cycles vs a
    // 32-cycle issue interval); zero operands of dead chunks add exact zeros
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      floatx4& acc = (q & 1) ? acc1 : acc0;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].x, bb[q].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].y, bb[q].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].z, bb[q].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].w, bb[q].w, acc, 0, 0, 0);
    }
  }
}

// Full-line staged form (VEC, K % 16 == 0): the fragment-shaped loads above touch 16 rows x 64 B
// per wave instruction (half of each 128-B line, twice the address-unit work per byte); here each
// wave instruction loads 8 whole 128-B lines (lane = one 16-B piece) of the wave's 16-row x
// 16*CH-column slice of x and of W into a wave-private LDS image (rows padded by 4 floats:
// conflict-free 16-B fragment reads), and the MFMA fragments come from LDS. Same products in the
// same order as the direct form.
template <int CH>
struct LinStage {
  static constexpr int kRow = 16 * CH + 4;  // floats per LDS row
  float a[16 * kRow];
  float b[16 * kRow];
};

// one group's global loads: instruction i covers lines [8i, 8i+8) of the 16 x 16CH slice
// Ring: x's K dimension is K / seg segments; logical segment s of a row is stored at physical
// segment (s + rot) mod (K / seg) (the rollout's frame-encoding ring; seg a power of two >= 32, so
// a 32-float group never straddles a segment). Only the x addresses move: products and their order
// are those of the logical layout.
struct XRing {
  int seg_shift;  // log2(seg); 0: no ring (the remap is a shift and a mask: no integer division,
  int rot, nseg;  // which cost 1.1 us per launch at 128 x 2048 -> 512)
};

template <int CH>
__device__ __forceinline__ void lin_stage_load(const float* x, int64_t ldx, const float* w, int K,
                                               int row0, int col0, int M, int N, int lane, int cb,
                                               int c1, float4 (&va)[CH], float4 (&vb)[CH],
                                               XRing ring) {
  constexpr int LPR = CH / 2;  // 128-B lines per row slice
  const int piece = lane & 7, lsub = lane >> 3;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int L = i * 8 + lsub;  // row L / LPR, line L % LPR
    const int r = L / LPR, li = L - r * LPR;
    const int kk = cb * 16 + li * 32 + piece * 4;
    const bool kok = kk < c1 * 16;
    const int ar = row0 + r, bc = col0 + r;
    int kx = kk;
    if (ring.seg_shift) {
      const int sg = kk >> ring.seg_shift;
      int ps = sg + ring.rot;
      ps = ps >= ring.nseg ? ps - ring.nseg : ps;
      kx = (ps << ring.seg_shift) | (kk & ((1 << ring.seg_shift) - 1));
    }
    va[i] = (kok && ar < M) ? *reinterpret_cast<const float4*>(x + static_cast<int64_t>(ar) * ldx + kx)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    vb[i] = (kok && bc < N) ? *reinterpret_cast<const float4*>(w + static_cast<int64_t>(bc) * K + kk)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// one group: the staged lines -> LDS, fragments back, CH x 4 MFMAs
template <int CH>
__device__ __forceinline__ void lin_stage_mfma(LinStage<CH>& st, int lane, const float4 (&va)[CH],
                                               const float4 (&vb)[CH], floatx4& acc0,
                                               floatx4& acc1) {
  constexpr int LPR = CH / 2;
  constexpr int kRow = LinStage<CH>::kRow;
  const int g = lane >> 4, c16 = lane & 15;
  const int piece = lane & 7, lsub = lane >> 3;
#pragma unroll
  for (int i = 0; i < CH; ++i) {
    const int L = i * 8 + lsub;
    const int r = L / LPR, li = L - r * LPR;
    *reinterpret_cast<float4*>(&st.a[r * kRow + li * 32 + piece * 4]) = va[i];
    *reinterpret_cast<float4*>(&st.b[r * kRow + li * 32 + piece * 4]) = vb[i];
  }
#pragma unroll
  for (int q = 0; q < CH; ++q) {
    const float4 fa = *reinterpret_cast<const float4*>(&st.a[c16 * kRow + q * 16 + 4 * g]);
    const float4 fb = *reinterpret_cast<const float4*>(&st.b[c16 * kRow + q * 16 + 4 * g]);
    floatx4& acc = (q & 1) ? acc1 : acc0;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa.x, fb.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa.y, fb.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa.z, fb.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa.w, fb.w, acc, 0, 0, 0);
  }
}

// The next group's global loads are issued before this group's LDS pass and MFMAs (two register
// sets, loop unrolled by two).
template <int CH>
__device__ __forceinline__ void linear_wave_chunks_lds(const float* x, int64_t ldx, const float* w,
                                                       int K, int row0, int col0, int M, int N,
                                                       int lane, int c0, int c1, LinStage<CH>& st,
                                                       floatx4& acc0, floatx4& acc1, XRing ring) {
  if (c0 >= c1) return;
  float4 a0[CH], b0[CH], a1[CH], b1[CH];
  lin_stage_load<CH>(x, ldx, w, K, row0, col0, M, N, lane, c0, c1, a0, b0, ring);
  for (int cb = c0; cb < c1; cb += 2 * CH) {
    const bool has1 = cb + CH < c1, has2 = cb + 2 * CH < c1;  // wave-uniform
    if (has1) lin_stage_load<CH>(x, ldx, w, K, row0, col0, M, N, lane, cb + CH, c1, a1, b1, ring);
    lin_stage_mfma<CH>(st, lane, a0, b0, acc0, acc1);
    if (has2) lin_stage_load<CH>(x, ldx, w, K, row0, col0, M, N, lane, cb + 2 * CH, c1, a0, b0, ring);
    if (has1) lin_stage_mfma<CH>(st, lane, a1, b1, acc0, acc1);
  }
}

// Frame-encoding cache epilogue (PPObj rollout, the last encoder layer): the layer's output row
// m is env m's fresh frame encoding; instead of storing it to y, shift env m's cache enc[m, W, N]
// like the frame stack (ocppo_frame_cache_shift's rule) with the fresh row in slot W-1:
//   enc[m, w] = done[m] != 0 || w == W-1 ? fresh[m] : enc[m, w+1]
// Each (row, column) of the cache is read and written by the one lane that owns that output
// element, slots in increasing w, so the shift needs no second launch.
// Ring form (slot >= 0): the cache is a ring over its W physical slots (XRing above, read by the
// decoder with rot = the oldest frame's slot); the fresh row only overwrites physical slot `slot`
// (the oldest frame's), or every slot of an env that was just reset -- no old slot is read.
struct CacheOut {
  float* enc;         // [M, W, N]
  const float* done;  // [M] or NULL
  int W;
  int slot;           // -1: shift form
};
constexpr int kCacheMaxW = 8;

// VEC: x / W rows are 16-B aligned with K % 4 == 0 (float4 operand loads); else scalar loads.
// CACHE: the output goes through the frame-cache epilogue above (y / ldy unused).
template <int S, int CH, bool RELU, bool VEC, bool CACHE = false, bool STAGE = false>
__global__ __launch_bounds__(64 * S) void linear_rows_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ y, int64_t ldy, int M, int N, int K,
    int ntm, int tiles, CacheOut cache = CacheOut{nullptr, nullptr, 0, -1},
    XRing ring = XRing{0, 0, 1}) {
  __shared__ floatx4 red[S > 1 ? S - 1 : 1][64];
  const int b = blockIdx.x;
  const int per_xcd = (tiles + 7) / 8;
  const int t = (b % 8) * per_xcd + b / 8;  // XCD-contiguous tile ranges
  if (t >= tiles) return;
  const int tm = t % ntm, tn = t / ntm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int row = tm * 16 + c16;  // A operand row of this lane
  const int col = tn * 16 + c16;  // B operand column (W row) of this lane
  const bool rok = row < M, cok = col < N;
  const float* xr = x + static_cast<int64_t>(rok ? row : 0) * ldx;
  const float* wr = w + static_cast<int64_t>(cok ? col : 0) * K;

  const int nch = (K + 15) / 16;
  const int cpw = (nch + S - 1) / S;
  const int c0 = wv * cpw;
  const int c1 = c0 + cpw < nch ? c0 + cpw : nch;
  // cache epilogue: wave 0 loads the old slots and done flags of its 4 x 1 outputs before the
  // MFMA loop, so their latency hides behind it (W <= kCacheMaxW; else loaded in the epilogue)
  float old[4][kCacheMaxW - 1];
  bool dn[4] = {false, false, false, false};
  const bool pre = CACHE && cache.slot < 0 && wv == 0 && cache.W <= kCacheMaxW &&
                   tn * 16 + c16 < N;
  if (pre) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int orow = tm * 16 + 4 * g + r;
      if (orow < M) {
        const float* e = cache.enc + static_cast<int64_t>(orow) * cache.W * N + tn * 16 + c16;
        dn[r] = cache.done != nullptr && cache.done[orow] != 0.f;
#pragma unroll
        for (int q = 0; q < kCacheMaxW - 1; ++q)
          old[r][q] = q + 1 < cache.W ? e[static_cast<int64_t>(q + 1) * N] : 0.f;
      }
    }
  }
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (STAGE) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lin_stage_raw[];
    LinStage<CH>* st = reinterpret_cast<LinStage<CH>*>(lin_stage_raw) + wv;
    linear_wave_chunks_lds<CH>(x, ldx, w, K, tm * 16, tn * 16, M, N, lane, c0, c1, *st,
                               acc0, acc1, ring);
  } else {
    linear_wave_chunks<CH, VEC>(xr, wr, rok, cok, K, g, c0, c1, acc0, acc1);
  }
  floatx4 acc = acc0 + acc1;
  if (S > 1) {
    if (wv > 0) red[wv - 1][lane] = acc;
    __syncthreads();
    if (wv > 0) return;
#pragma unroll
    for (int q = 0; q < S - 1; ++q) acc += red[q][lane];
  }
  // C/D layout of 16x16 MFMA: column lane & 15, rows 4 * (lane >> 4) + r
  const int ocol = tn * 16 + c16;
  if (ocol >= N) return;
  const float bv = bias ? bias[ocol] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int orow = tm * 16 + 4 * g + r;
    if (orow < M) {
      float v = acc[r] + bv;
      if (RELU) v = relu_f(v);
      if (CACHE) {
        const int W = cache.W;
        float* e = cache.enc + static_cast<int64_t>(orow) * W * N + ocol;
        if (cache.slot >= 0) {
          if (cache.done != nullptr && cache.done[orow] != 0.f) {
            for (int q = 0; q < W; ++q) e[static_cast<int64_t>(q) * N] = v;
          } else {
            e[static_cast<int64_t>(cache.slot) * N] = v;
          }
        } else if (pre) {
#pragma unroll
          for (int q = 0; q < kCacheMaxW - 1; ++q)
            if (q + 1 < W) e[static_cast<int64_t>(q) * N] = dn[r] ? v : old[r][q];
          e[static_cast<int64_t>(W - 1) * N] = v;
        } else if (cache.done != nullptr && cache.done[orow] != 0.f) {
          for (int q = 0; q < W; ++q) e[static_cast<int64_t>(q) * N] = v;
        } else {
          for (int q = 0; q + 1 < W; ++q) e[static_cast<int64_t>(q) * N] = e[static_cast<int64_t>(q + 1) * N];
          e[static_cast<int64_t>(W - 1) * N] = v;
        }
      } else {
        y[static_cast<int64_t>(orow) * ldy + ocol] = v;
      }
    }
  }
}

#ifndef OCPPO_LIN_STAGE_CH  // chunks of 16 k per staged group (experiments: tools/)
#define OCPPO_LIN_STAGE_CH 2
#endif
constexpr int kLinStageCH = OCPPO_LIN_STAGE_CH;

template <int S, int CH, bool RELU, bool CACHE>
static void launch_linear_sc(hipStream_t s, bool vec, const float* x, int64_t ldx, const float* w,
                             const float* b, float* y, int64_t ldy, int M, int N, int K,
                             CacheOut c, XRing ring) {
  const int ntm = (M + 15) / 16, ntn = (N + 15) / 16, tiles = ntm * ntn;
  const dim3 grid(8 * ((tiles + 7) / 8)), block(64 * S);
  if (vec && K % 16 == 0)  // full-line staged, pipelined in groups of kLinStageCH chunks
    hipLaunchKernelGGL((linear_rows_kernel<S, kLinStageCH, RELU, true, CACHE, true>), grid, block,
                       sizeof(LinStage<kLinStageCH>) * S, s, x, ldx, w, b, y, ldy, M, N, K, ntm,
                       tiles, c, ring);
  else if (vec)
    hipLaunchKernelGGL((linear_rows_kernel<S, CH, RELU, true, CACHE>), grid, block, 0, s, x, ldx,
                       w, b, y, ldy, M, N, K, ntm, tiles, c);
  else
    hipLaunchKernelGGL((linear_rows_kernel<S, CH, RELU, false, CACHE>), grid, block, 0, s, x, ldx,
                       w, b, y, ldy, M, N, K, ntm, tiles, c);
}

template <int S, bool RELU, bool CACHE>
static void launch_linear_s(hipStream_t s, int cpw, bool vec, const float* x, int64_t ldx,
                            const float* w, const float* b, float* y, int64_t ldy, int M, int N,
                            int K, CacheOut c, XRing ring) {
  if (cpw <= 2)
    launch_linear_sc<S, 2, RELU, CACHE>(s, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring);
  else if (cpw <= 4)
    launch_linear_sc<S, 4, RELU, CACHE>(s, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring);
  else
    launch_linear_sc<S, 8, RELU, CACHE>(s, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring);
}

template <bool RELU, bool CACHE = false>
static void launch_linear(hipStream_t s, bool vec, const float* x, int64_t ldx, const float* w,
                          const float* b, float* y, int64_t ldy, int M, int N, int K,
                          CacheOut c = CacheOut{nullptr, nullptr, 0, -1},
                          XRing ring = XRing{0, 0, 1}) {
  const int64_t tiles = static_cast<int64_t>((M + 15) / 16) * ((N + 15) / 16);
  const int nch = (K + 15) / 16;
  int S = 1;  // K split: >= ~4096 waves (4 per SIMD), >= 2 chunks per wave
  while (S < kLinMaxWaves && tiles * S < OCPPO_LIN_WAVE_TARGET && nch >= 2 * S * 2) S *= 2;
  const int cpw = (nch + S - 1) / S;
  switch (S) {
    case 1: launch_linear_s<1, RELU, CACHE>(s, cpw, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring); break;
    case 2: launch_linear_s<2, RELU, CACHE>(s, cpw, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring); break;
    case 4: launch_linear_s<4, RELU, CACHE>(s, cpw, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring); break;
#if OCPPO_LIN_MAX_WAVES > 8
    case 8: launch_linear_s<8, RELU, CACHE>(s, cpw, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring); break;
    default: launch_linear_s<16, RELU, CACHE>(s, cpw, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring); break;
#else
    default: launch_linear_s<8, RELU, CACHE>(s, cpw, vec, x, ldx, w, b, y, ldy, M, N, K, c, ring); break;
#endif
  }
}

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_linear_act(ocppo_stream_t stream, const float* x, int64_t ldx, const float* w,
                                const float* b, float* y, int64_t ldy, int64_t M, int64_t N,
                                int64_t K, int relu) {
  OCPPO_REQUIRE(M >= 0 && N >= 1 && K >= 1 && M <= INT32_MAX && N <= INT32_MAX && K <= INT32_MAX,
                "ocppo_linear_act: bad sizes M=%lld N=%lld K=%lld", (long long)M, (long long)N,
                (long long)K);
  OCPPO_REQUIRE(ldx >= K && ldy >= N, "ocppo_linear_act: leading dimensions ldx=%lld ldy=%lld",
                (long long)ldx, (long long)ldy);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(x && w && y, "ocppo_linear_act: null pointer");
  OCPPO_REQUIRE((M + 15) / 16 * ((N + 15) / 16) <= INT32_MAX / 8, "ocppo_linear_act: too large");
  const bool vec = K % 4 == 0 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(w) % 16 == 0;
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (relu)
    launch_linear<true>(s, vec, x, ldx, w, b, y, ldy, (int)M, (int)N, (int)K);
  else
    launch_linear<false>(s, vec, x, ldx, w, b, y, ldy, (int)M, (int)N, (int)K);
  return check_launch("ocppo_linear_act");
}

extern "C" int ocppo_linear_cache_shift(ocppo_stream_t stream, const float* x, int64_t ldx,
                                        const float* w, const float* b, float* enc,
                                        const float* done, int64_t M, int64_t N, int64_t K,
                                        int64_t W, int relu) {
  OCPPO_REQUIRE(M >= 0 && N >= 1 && K >= 1 && W >= 1 && W <= 64 && M <= INT32_MAX &&
                    N <= INT32_MAX && K <= INT32_MAX,
                "ocppo_linear_cache_shift: bad sizes M=%lld N=%lld K=%lld W=%lld", (long long)M,
                (long long)N, (long long)K, (long long)W);
  OCPPO_REQUIRE(ldx >= K, "ocppo_linear_cache_shift: ldx=%lld < K", (long long)ldx);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(x && w && enc, "ocppo_linear_cache_shift: null pointer");
  OCPPO_REQUIRE((M + 15) / 16 * ((N + 15) / 16) <= INT32_MAX / 8,
                "ocppo_linear_cache_shift: too large");
  const bool vec = K % 4 == 0 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(w) % 16 == 0;
  const CacheOut c{enc, done, static_cast<int>(W), -1};
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (relu)
    launch_linear<true, true>(s, vec, x, ldx, w, b, nullptr, 0, (int)M, (int)N, (int)K, c);
  else
    launch_linear<false, true>(s, vec, x, ldx, w, b, nullptr, 0, (int)M, (int)N, (int)K, c);
  return check_launch("ocppo_linear_cache_shift");
}

extern "C" int ocppo_linear_act_ring(ocppo_stream_t stream, const float* x, int64_t ldx,
                                     const float* w, const float* b, float* y, int64_t ldy,
                                     int64_t M, int64_t N, int64_t K, int64_t seg, int64_t rot,
                                     int relu) {
  OCPPO_REQUIRE(M >= 0 && N >= 1 && K >= 1 && M <= INT32_MAX && N <= INT32_MAX && K <= INT32_MAX,
                "ocppo_linear_act_ring: bad sizes M=%lld N=%lld K=%lld", (long long)M, (long long)N,
                (long long)K);
  OCPPO_REQUIRE(seg >= 32 && (seg & (seg - 1)) == 0 && K % seg == 0 && rot >= 0 && rot < K / seg,
                "ocppo_linear_act_ring: seg=%lld rot=%lld (seg a power of two >= 32, K %% seg == "
                "0, 0 <= rot < K / seg)", (long long)seg, (long long)rot);
  OCPPO_REQUIRE(ldx >= K && ldy >= N && ldx % 4 == 0,
                "ocppo_linear_act_ring: leading dimensions ldx=%lld ldy=%lld", (long long)ldx,
                (long long)ldy);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(x && w && y, "ocppo_linear_act_ring: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0,
                "ocppo_linear_act_ring: x and w must be 16-B aligned");
  OCPPO_REQUIRE((M + 15) / 16 * ((N + 15) / 16) <= INT32_MAX / 8, "ocppo_linear_act_ring: too large");
  const XRing ring{__builtin_ctzll(static_cast<unsigned long long>(seg)), static_cast<int>(rot),
                   static_cast<int>(K / seg)};
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (relu)
    launch_linear<true>(s, true, x, ldx, w, b, y, ldy, (int)M, (int)N, (int)K,
                        CacheOut{nullptr, nullptr, 0, -1}, ring);
  else
    launch_linear<false>(s, true, x, ldx, w, b, y, ldy, (int)M, (int)N, (int)K,
                         CacheOut{nullptr, nullptr, 0, -1}, ring);
  return check_launch("ocppo_linear_act_ring");
}

namespace ocppo {

// ---- NHWC convolution (no padding) + bias + ReLU for rollout-sized batches ----------------------
// The NatureCNN trunk of the rollout forward (architectures/ppo.py:20-31 at ppo_atari_oc.py:506,
// Conv2d 4->32 8x8/4, 32->64 4x4/2, 64->64 3x3/1 on 256 envs' channels-last frames) as an
// implicit GEMM on the f32 matrix cores: rows = output pixels (b, oy, ox), columns = output
// channels, k = (ky, kx, ci) -- the order of the channels_last weight [Cout, KH, KW, Cin], so W is
// the same k-contiguous B operand as a Linear's, and a 16-k chunk of a row is 4 float4 loads of
// the NHWC input (Cin = 4: one tap's 4 channels each; Cin >= 16: 16 channels of one tap). Tiles,
// K split and epilogue are linear_rows_kernel's (one workgroup per 16 x 16 output tile, waves
// combined through LDS in wave order, bias then ReLU as torch's conv + relu). MIOpen at this
// batch runs an implicit GEMM per layer plus a zero-fill, an NCHW->NHWC copy and our bias/ReLU
// pass (tools/exp_conv_rollout.py).
#ifndef OCPPO_CONV_WAVES  // experiments (tools/build_variant.py) move the K-split target
#define OCPPO_CONV_WAVES 4096
#endif
constexpr int64_t kConvWaves = OCPPO_CONV_WAVES;

struct ConvGeom {
  int H, W, Cin, KW, stride, OH, OW;
  int cin_shift;  // log2(Cin)
  int kw_magic;   // ceil(2^16 / KW): tap / KW = (tap * kw_magic) >> 16 for tap < 2^10
};

template <int S, int CH, bool RELU>
__global__ __launch_bounds__(64 * S) void conv_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    float* __restrict__ y, int M, int N, int K, int ntm, int tiles, ConvGeom cg) {
  __shared__ floatx4 red[S > 1 ? S - 1 : 1][64];
  const int b = blockIdx.x;
  const int per_xcd = (tiles + 7) / 8;
  const int t = (b % 8) * per_xcd + b / 8;  // XCD-contiguous tile ranges (as linear_rows)
  if (t >= tiles) return;
  const int tm = t % ntm, tn = t / ntm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int row = tm * 16 + c16, col = tn * 16 + c16;
  const bool rok = row < M, cok = col < N;
  // this lane's output pixel -> the first input element of its receptive field
  const int pix = rok ? row : 0;
  const int ohw = cg.OH * cg.OW;
  const int bi = pix / ohw, r2 = pix - bi * ohw;
  const int oy = r2 / cg.OW, ox = r2 - oy * cg.OW;
  const float* xr = x + (static_cast<int64_t>(bi * cg.H + oy * cg.stride) * cg.W +
                         ox * cg.stride) * cg.Cin;
  const float* wr = w + static_cast<int64_t>(cok ? col : 0) * K;
  const int nch = K / 16;
  const int cpw = (nch + S - 1) / S;
  const int c0 = wv * cpw;
  const int c1 = c0 + cpw < nch ? c0 + cpw : nch;
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int cb = c0; cb < c1; cb += CH) {
    float4 a[CH], bb[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      const int k = (cb + q) * 16 + 4 * g;
      const bool live = cb + q < c1;
      const int tap = k >> cg.cin_shift, ci = k & (cg.Cin - 1);
      const int ky = (tap * cg.kw_magic) >> 16, kx = tap - ky * cg.KW;
      const int off = (ky * cg.W + kx) * cg.Cin + ci;
      a[q] = (live && rok) ? *reinterpret_cast<const float4*>(xr + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      bb[q] = (live && cok) ? *reinterpret_cast<const float4*>(wr + k) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < CH; ++q) {  // same MFMA order as linear_wave_chunks
      floatx4& acc = (q & 1) ? acc1 : acc0;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].x, bb[q].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].y, bb[q].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].z, bb[q].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q].w, bb[q].w, acc, 0, 0, 0);
    }
  }
  floatx4 acc = acc0 + acc1;
  if (S > 1) {
    if (wv > 0) red[wv - 1][lane] = acc;
    __syncthreads();
    if (wv > 0) return;
#pragma unroll
    for (int q = 0; q < S - 1; ++q) acc += red[q][lane];
  }
  if (!cok) return;
  const float bv = bias ? bias[col] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int orow = tm * 16 + 4 * g + r;
    if (orow < M) {
      float v = acc[r] + bv;
      if (RELU) v = relu_f(v);
      y[static_cast<int64_t>(orow) * N + col] = v;
    }
  }
}

template <int S, bool RELU>
static void launch_conv_s(hipStream_t s, int cpw, const float* x, const float* w, const float* b,
                          float* y, int M, int N, int K, ConvGeom cg) {
  const int ntm = (M + 15) / 16, ntn = (N + 15) / 16, tiles = ntm * ntn;
  const dim3 grid(8 * ((tiles + 7) / 8)), block(64 * S);
  if (cpw <= 2)
    hipLaunchKernelGGL((conv_rows_kernel<S, 2, RELU>), grid, block, 0, s, x, w, b, y, M, N, K, ntm, tiles, cg);
  else if (cpw <= 4)
    hipLaunchKernelGGL((conv_rows_kernel<S, 4, RELU>), grid, block, 0, s, x, w, b, y, M, N, K, ntm, tiles, cg);
  else
    hipLaunchKernelGGL((conv_rows_kernel<S, 8, RELU>), grid, block, 0, s, x, w, b, y, M, N, K, ntm, tiles, cg);
}

template <bool RELU>
static void launch_conv(hipStream_t s, const float* x, const float* w, const float* b, float* y,
                        int M, int N, int K, ConvGeom cg) {
  const int64_t tiles = static_cast<int64_t>((M + 15) / 16) * ((N + 15) / 16);
  const int nch = K / 16;
  int S = 1;  // K split as launch_linear: >= ~kConvWaves waves, >= 2 chunks per wave
  while (S < 8 && tiles * S < kConvWaves && nch >= 2 * S * 2) S *= 2;
  const int cpw = (nch + S - 1) / S;
  switch (S) {
    case 1: launch_conv_s<1, RELU>(s, cpw, x, w, b, y, M, N, K, cg); break;
    case 2: launch_conv_s<2, RELU>(s, cpw, x, w, b, y, M, N, K, cg); break;
    case 4: launch_conv_s<4, RELU>(s, cpw, x, w, b, y, M, N, K, cg); break;
    default: launch_conv_s<8, RELU>(s, cpw, x, w, b, y, M, N, K, cg); break;
  }
}

}  // namespace ocppo

extern "C" int ocppo_conv2d_act(ocppo_stream_t stream, const float* x, int64_t B, int64_t H,
                                int64_t W, int64_t Cin, const float* w, const float* b,
                                int64_t Cout, int64_t KH, int64_t KW, int64_t stride, float* y,
                                int relu) {
  OCPPO_REQUIRE(B >= 0 && H >= 1 && W >= 1 && Cin >= 4 && (Cin & (Cin - 1)) == 0 &&
                    Cout >= 1 && KH >= 1 && KW >= 1 && KW <= 64 && KH <= H && KW <= W &&
                    stride >= 1 && (KH * KW * Cin) % 16 == 0 && KH * KW <= 1024,
                "ocppo_conv2d_act: bad sizes B=%lld H=%lld W=%lld Cin=%lld Cout=%lld K=%lldx%lld "
                "stride=%lld (Cin a power of two >= 4, KH*KW*Cin %% 16 == 0)", (long long)B,
                (long long)H, (long long)W, (long long)Cin, (long long)Cout, (long long)KH,
                (long long)KW, (long long)stride);
  const int64_t OH = (H - KH) / stride + 1, OW = (W - KW) / stride + 1;
  const int64_t M = B * OH * OW, K = KH * KW * Cin;
  OCPPO_REQUIRE(B * H * W * Cin <= INT32_MAX && M <= INT32_MAX && Cout * K <= INT32_MAX &&
                    (M + 15) / 16 * ((Cout + 15) / 16) <= INT32_MAX / 8,
                "ocppo_conv2d_act: too large");
  if (B == 0) return OCPPO_OK;
  OCPPO_REQUIRE(x && w && y, "ocppo_conv2d_act: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0,
                "ocppo_conv2d_act: x and w must be 16-B aligned");
  ConvGeom cg;
  cg.H = (int)H; cg.W = (int)W; cg.Cin = (int)Cin; cg.KW = (int)KW; cg.stride = (int)stride;
  cg.OH = (int)OH; cg.OW = (int)OW;
  cg.cin_shift = __builtin_ctzll(static_cast<unsigned long long>(Cin));
  cg.kw_magic = static_cast<int>((65536 + KW - 1) / KW);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (relu)
    launch_conv<true>(s, x, w, b, y, (int)M, (int)Cout, (int)K, cg);
  else
    launch_conv<false>(s, x, w, b, y, (int)M, (int)Cout, (int)K, cg);
  return check_launch("ocppo_conv2d_act");
}

extern "C" int ocppo_linear_cache_ring(ocppo_stream_t stream, const float* x, int64_t ldx,
                                       const float* w, const float* b, float* enc,
                                       const float* done, int64_t M, int64_t N, int64_t K,
                                       int64_t W, int64_t slot, int relu) {
  OCPPO_REQUIRE(M >= 0 && N >= 1 && K >= 1 && W >= 1 && W <= 64 && M <= INT32_MAX &&
                    N <= INT32_MAX && K <= INT32_MAX && slot >= 0 && slot < W,
                "ocppo_linear_cache_ring: bad sizes M=%lld N=%lld K=%lld W=%lld slot=%lld",
                (long long)M, (long long)N, (long long)K, (long long)W, (long long)slot);
  OCPPO_REQUIRE(ldx >= K, "ocppo_linear_cache_ring: ldx=%lld < K", (long long)ldx);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(x && w && enc, "ocppo_linear_cache_ring: null pointer");
  OCPPO_REQUIRE((M + 15) / 16 * ((N + 15) / 16) <= INT32_MAX / 8,
                "ocppo_linear_cache_ring: too large");
  const bool vec = K % 4 == 0 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(w) % 16 == 0;
  const CacheOut c{enc, done, static_cast<int>(W), static_cast<int>(slot)};
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (relu)
    launch_linear<true, true>(s, vec, x, ldx, w, b, nullptr, 0, (int)M, (int)N, (int)K, c);
  else
    launch_linear<false, true>(s, vec, x, ldx, w, b, nullptr, 0, (int)M, (int)N, (int)K, c);
  return check_launch("ocppo_linear_cache_ring");
}

// ---- two Linear(+ReLU) layers in one launch: y = act2(act1(x W1^T + b1) W2^T + b2) ---------------
// The first two PPObj encoder layers of the rollout's newest-frame encode (architectures/ppo.py:
// 60-84: F -> 256 -> 512 at 128 rows per step): the first layer is tiny (K1 = F <= 64), so every
// workgroup recomputes the 16 hidden rows its output tile needs (16 x N1 values, K1 MACs each) into
// LDS instead of waiting for a second launch, then runs the second layer's 16x16 tile from LDS
// (A operand, rows padded to N1 + 4 floats: conflict-free 16-B reads) and global W2 (B operand),
// K = N1 split over the S waves and combined through LDS in wave order. One launch instead of
// two on the rollout's dependent chain; same v_mfma_f32_16x16x4_f32 arithmetic as linear_rows.
namespace ocppo {

constexpr int kLin2MaxK1 = 64;
constexpr int kLin2MaxN1 = 512;

// One workgroup's output tile. XDT: x is an f32 frame seen through the rollout storage dtype
// (the network reads what the rollout buffer holds: bf16 round trip for object vectors stored in
// bf16, identity for f32).
template <int S, bool RELU1, bool RELU2, int XDT>
__device__ __forceinline__ void linear2_tile(
    int b, float* smem, const float* __restrict__ x, int64_t ldx, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ y, int64_t ldy, int M, int N1, int N2, int K1, int ntm, int tiles) {
  const int ldh = N1 + 4;
  float* h1 = smem;                                                    // [16][ldh]
  floatx4* red = reinterpret_cast<floatx4*>(smem + 16 * ldh);          // [S-1][64]
  const int per_xcd = (tiles + 7) / 8;
  const int t = (b % 8) * per_xcd + b / 8;  // XCD-contiguous tile ranges (as linear_rows)
  if (t >= tiles) return;
  const int tm = t % ntm, tn = t / ntm;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int row = tm * 16 + c16;
  const bool rok = row < M;
  const float* xr = x + static_cast<int64_t>(rok ? row : 0) * ldx;

  // every global operand of both phases is loaded up front (one round trip of latency): the x
  // chunks, this wave's W1 rows (phase-1 tiles ct = wv, wv + S, ...) and its W2 K-chunks
  const int nkc = (K1 + 15) / 16;
  const int nct = N1 / 16;
  const int col2 = tn * 16 + c16;
  const bool cok = col2 < N2;
  const float* w2r = w2 + static_cast<int64_t>(cok ? col2 : 0) * N1;
  const int cpw = (nct + S - 1) / S;
  const int c0 = wv * cpw;
  const int c1 = c0 + cpw < nct ? c0 + cpw : nct;
  constexpr int kMaxT = kLin2MaxN1 / 16 / S;  // phase-1 tiles and phase-2 chunks per wave
  float4 a1[kLin2MaxK1 / 16];
#pragma unroll
  for (int kc = 0; kc < kLin2MaxK1 / 16; ++kc) {
    const int k = kc * 16 + 4 * g;
    a1[kc].x = (kc < nkc && rok && k + 0 < K1) ? Elem<XDT>::roundtrip(xr[k + 0]) : 0.f;
    a1[kc].y = (kc < nkc && rok && k + 1 < K1) ? Elem<XDT>::roundtrip(xr[k + 1]) : 0.f;
    a1[kc].z = (kc < nkc && rok && k + 2 < K1) ? Elem<XDT>::roundtrip(xr[k + 2]) : 0.f;
    a1[kc].w = (kc < nkc && rok && k + 3 < K1) ? Elem<XDT>::roundtrip(xr[k + 3]) : 0.f;
  }
  float4 b2v[kMaxT];
#pragma unroll
  for (int q = 0; q < kMaxT; ++q) {
    const int c = c0 + q;
    b2v[q] = (c < c1 && cok) ? *reinterpret_cast<const float4*>(w2r + c * 16 + 4 * g)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // phase 1: h1[16][N1] = act1(x[16 rows] W1^T + b1)
#pragma unroll
  for (int q = 0; q < kMaxT; ++q) {
    const int ct = wv + q * S;
    if (ct < nct) {
      const int col = ct * 16 + c16;  // W1 row of this lane's B operand
      const float* wr = w1 + static_cast<int64_t>(col) * K1;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < kLin2MaxK1 / 16; ++kc) {
        if (kc < nkc) {
          const int k = kc * 16 + 4 * g;
          float4 bb;
          bb.x = k + 0 < K1 ? wr[k + 0] : 0.f;
          bb.y = k + 1 < K1 ? wr[k + 1] : 0.f;
          bb.z = k + 2 < K1 ? wr[k + 2] : 0.f;
          bb.w = k + 3 < K1 ? wr[k + 3] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[kc].x, bb.x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[kc].y, bb.y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[kc].z, bb.z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[kc].w, bb.w, acc, 0, 0, 0);
        }
      }
      const float bv = b1 ? b1[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[r] + bv;
        if (RELU1) v = relu_f(v);
        h1[(4 * g + r) * ldh + col] = v;  // C layout: column lane & 15, rows 4 * (lane >> 4) + r
      }
    }
  }
  __syncthreads();

  // phase 2: the 16x16 tile of y; K = N1 in 16-wide chunks split over the S waves
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < kMaxT; ++q) {
    const int c = c0 + q;
    if (c < c1) {
      const float4 a = *reinterpret_cast<const float4*>(h1 + c16 * ldh + c * 16 + 4 * g);
      const float4 bb = b2v[q];
      floatx4& acc = (q & 1) ? acc1 : acc0;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, bb.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, bb.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, bb.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, bb.w, acc, 0, 0, 0);
    }
  }
  floatx4 acc = acc0 + acc1;
  if (S > 1) {
    if (wv > 0) red[(wv - 1) * 64 + lane] = acc;
    __syncthreads();
    if (wv > 0) return;
#pragma unroll
    for (int q = 0; q < S - 1; ++q) acc += red[q * 64 + lane];
  }
  if (!cok) return;
  const float bv2 = b2 ? b2[col2] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int orow = tm * 16 + 4 * g + r;
    if (orow < M) {
      float v = acc[r] + bv2;
      if (RELU2) v = relu_f(v);
      y[static_cast<int64_t>(orow) * ldy + col2] = v;
    }
  }
}

template <int S, bool RELU1, bool RELU2>
__global__ __launch_bounds__(64 * S) void linear2_rows_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ y, int64_t ldy, int M, int N1, int N2, int K1, int ntm, int tiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  linear2_tile<S, RELU1, RELU2, OCPPO_F32>(blockIdx.x, smem, x, ldx, w1, b1, w2, b2, y, ldy, M,
                                           N1, N2, K1, ntm, tiles);
}

template <bool R1, bool R2>
static void launch_linear2(hipStream_t s, const float* x, int64_t ldx, const float* w1,
                           const float* b1, const float* w2, const float* b2, float* y,
                           int64_t ldy, int M, int N1, int N2, int K1) {
  constexpr int S = 4;
  const int ntm = (M + 15) / 16, ntn = (N2 + 15) / 16, tiles = ntm * ntn;
  const size_t lds = sizeof(float) * 16 * (N1 + 4) + sizeof(floatx4) * 64 * (S - 1);
  hipLaunchKernelGGL((linear2_rows_kernel<S, R1, R2>), dim3(8 * ((tiles + 7) / 8)), dim3(64 * S),
                     lds, s, x, ldx, w1, b1, w2, b2, y, ldy, M, N1, N2, K1, ntm, tiles);
}

}  // namespace ocppo

extern "C" int ocppo_linear2_act(ocppo_stream_t stream, const float* x, int64_t ldx,
                                 const float* w1, const float* b1, const float* w2,
                                 const float* b2, float* y, int64_t ldy, int64_t M, int64_t N1,
                                 int64_t N2, int64_t K1, int relu1, int relu2) {
  OCPPO_REQUIRE(M >= 0 && K1 >= 1 && K1 <= kLin2MaxK1 && N1 >= 16 && N1 % 16 == 0 &&
                    N1 <= kLin2MaxN1 && N2 >= 1 && N2 <= INT32_MAX && M <= INT32_MAX,
                "ocppo_linear2_act: bad sizes M=%lld K1=%lld N1=%lld N2=%lld (K1 <= 64, N1 %% 16 "
                "== 0, N1 <= 512)", (long long)M, (long long)K1, (long long)N1, (long long)N2);
  OCPPO_REQUIRE(ldx >= K1 && ldy >= N2, "ocppo_linear2_act: leading dimensions ldx=%lld ldy=%lld",
                (long long)ldx, (long long)ldy);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(x && w1 && w2 && y, "ocppo_linear2_act: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(w2) % 16 == 0,
                "ocppo_linear2_act: w2 must be 16-B aligned");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const int m = (int)M, n1 = (int)N1, n2 = (int)N2, k1 = (int)K1;
  if (relu1 && relu2)
    launch_linear2<true, true>(s, x, ldx, w1, b1, w2, b2, y, ldy, m, n1, n2, k1);
  else if (relu1)
    launch_linear2<true, false>(s, x, ldx, w1, b1, w2, b2, y, ldy, m, n1, n2, k1);
  else if (relu2)
    launch_linear2<false, true>(s, x, ldx, w1, b1, w2, b2, y, ldy, m, n1, n2, k1);
  else
    launch_linear2<false, false>(s, x, ldx, w1, b1, w2, b2, y, ldy, m, n1, n2, k1);
  return check_launch("ocppo_linear2_act");
}

// ---- rollout store of step t-1 + the first two encoder layers of step t in ONE launch -----------
// The PPObj rollout with the frame-encoding cache (ocppo_frame_cache_shift): each step stores the
// env's output (ocppo_rollout_store[_vecnorm]: frame stack into rollout slot t, f32 network copy,
// reward / done rows, VecNormalize) and then encodes ONLY the newest frame, whose first two
// Linear+ReLU layers are ocppo_linear2_act over those N frames. Neither half reads what the other
// writes (the encoder takes the newest frame straight from the env output, seen through the
// storage dtype exactly as the stored slot holds it), so they share a launch: workgroups
// [0, lin) run linear2 tiles, workgroup lin the VecNormalize reduction (when asked), the rest the
// store groups. Same arithmetic as the two launches it replaces (ppo_atari_oc.py:502-514 and the
// encoder half of :506).
#include "ocppo_store.h"

namespace ocppo {

struct StoreLin2Args {
  // store
  const float* frame;
  const float* reward;
  const float* done;
  int64_t N, D;
  int W;
  const void* prev;
  void* out;
  float* net;
  float* reward_out;
  float* done_out;
  double gamma, eps, clip;
  double* ret;
  double* rms;
  // linear2
  const float* w1;
  const float* b1;
  const float* w2;
  const float* b2;
  float* y;
  int64_t ldy;
  int N1, N2, ntm, tiles, lin_blocks;
};

template <int ODT, int VEC, bool VN>
__global__ __launch_bounds__(256) void store_linear2_kernel(StoreLin2Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x;
  if (b < a.lin_blocks) {
    // the newest frame of slot t+1 is frame[n] itself (slot W-1, reset fill or not)
    linear2_tile<4, true, true, ODT>(b, smem, a.frame, a.D, a.w1, a.b1, a.w2, a.b2, a.y, a.ldy,
                                     static_cast<int>(a.N), a.N1, a.N2, static_cast<int>(a.D),
                                     a.ntm, a.tiles);
    return;
  }
  if (VN && b == a.lin_blocks) {
    vecnorm_block(a.reward, a.done, a.N, a.gamma, a.eps, a.clip, a.ret, a.rms, a.reward_out);
    return;
  }
  const int s0 = a.lin_blocks + (VN ? 1 : 0);
  store_groups<OCPPO_F32, ODT, VEC>(b - s0, gridDim.x - s0, a.frame, a.reward, a.done, a.N, a.W,
                                    a.D, a.prev, a.out, a.net, VN ? nullptr : a.reward_out,
                                    a.done_out, 1.0f, nullptr);
}

template <int ODT, bool VN>
static void launch_store_linear2(hipStream_t s, const StoreLin2Args& a) {
  const size_t lds = sizeof(float) * 16 * (a.N1 + 4) + sizeof(floatx4) * 64 * 3;
  const int vec = a.D % 4 == 0 ? 4 : 1;
  const int64_t groups = a.N * a.W * (a.D / vec);
  const int sg = grid_for(groups, 256);
  const dim3 grid(a.lin_blocks + (VN ? 1 : 0) + sg);
  if (vec == 4)
    hipLaunchKernelGGL((store_linear2_kernel<ODT, 4, VN>), grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((store_linear2_kernel<ODT, 1, VN>), grid, dim3(256), lds, s, a);
}

}  // namespace ocppo

extern "C" int ocppo_store_linear2(ocppo_stream_t stream, const float* frame, const float* reward,
                                   const float* done, int64_t N, int64_t W, int64_t D,
                                   const void* prev_obs, void* obs_out, int obs_dtype,
                                   float* net_obs, float* reward_out, float* done_out,
                                   int vecnorm, double gamma, double epsilon, double clip_reward,
                                   double* ret_state, double* rms_state, const float* w1,
                                   const float* b1, const float* w2, const float* b2, float* y,
                                   int64_t ldy, int64_t N1, int64_t N2) {
  OCPPO_REQUIRE(N >= 1 && N <= INT32_MAX && W >= 1 && W <= 64 && D >= 1 && D <= kLin2MaxK1 &&
                    N1 >= 16 && N1 % 16 == 0 && N1 <= kLin2MaxN1 && N2 >= 1 && N2 <= INT32_MAX &&
                    ldy >= N2,
                "ocppo_store_linear2: bad sizes N=%lld W=%lld D=%lld N1=%lld N2=%lld (D <= 64, "
                "N1 %% 16 == 0, N1 <= 512)", (long long)N, (long long)W, (long long)D,
                (long long)N1, (long long)N2);
  OCPPO_REQUIRE(obs_dtype == OCPPO_F32 || obs_dtype == OCPPO_BF16,
                "ocppo_store_linear2: obs dtype must be OCPPO_F32 or OCPPO_BF16 (object vectors)");
  OCPPO_REQUIRE(frame && reward && done && prev_obs && obs_out && w1 && w2 && y,
                "ocppo_store_linear2: null pointer");
  OCPPO_REQUIRE(prev_obs != obs_out, "ocppo_store_linear2: prev_obs must not alias obs_out");
  OCPPO_REQUIRE(!vecnorm || (ret_state && rms_state && reward_out && reward_out != reward),
                "ocppo_store_linear2: VecNormalize needs ret/rms state and a separate reward_out");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(w2) % 16 == 0,
                "ocppo_store_linear2: w2 must be 16-B aligned");
  StoreLin2Args a;
  a.frame = frame; a.reward = reward; a.done = done; a.N = N; a.D = D; a.W = (int)W;
  a.prev = prev_obs; a.out = obs_out; a.net = net_obs; a.reward_out = reward_out;
  a.done_out = done_out; a.gamma = gamma; a.eps = epsilon; a.clip = clip_reward;
  a.ret = ret_state; a.rms = rms_state;
  a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.y = y; a.ldy = ldy;
  a.N1 = (int)N1; a.N2 = (int)N2;
  a.ntm = (int)((N + 15) / 16);
  a.tiles = a.ntm * (int)((N2 + 15) / 16);
  a.lin_blocks = 8 * ((a.tiles + 7) / 8);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (obs_dtype == OCPPO_BF16) {
    if (vecnorm) launch_store_linear2<OCPPO_BF16, true>(s, a);
    else launch_store_linear2<OCPPO_BF16, false>(s, a);
  } else {
    if (vecnorm) launch_store_linear2<OCPPO_F32, true>(s, a);
    else launch_store_linear2<OCPPO_F32, false>(s, a);
  }
  return check_launch("ocppo_store_linear2");
}
