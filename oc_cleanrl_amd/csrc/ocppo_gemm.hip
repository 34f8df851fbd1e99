// Update-phase GEMMs of the PPObj / NatureCNN-head Linear layers on the f32 matrix cores
// (cleanrl/ppo_atari_oc.py:566-606: the minibatch forward `agent.get_action_and_value(b_obs[mb])`
// through architectures/ppo.py:60-84 and its `loss.backward()`), f32 in / f32 accumulate like the
// reference's torch.float32 Linear layers.
//
//   C[m, n] = epilogue( sum_k A(m, k) B(n, k) )
//
// A(m, k) and B(n, k) are strided views (one of the two strides is 1), so one kernel covers the
// three products of a Linear layer without transposing anything in HBM:
//   forward  y  = x W^T        A = x  [M, K] (k-contiguous), B = W [N, K] (k-contiguous)
//   dX       dx = g' W         A = g' [M, N] (k-contiguous), B(n=k_in, k=n_out) = W (n-contiguous)
//   dW       dW = g'^T x       A(m=n_out, k=row) = g' (m-contiguous), B(n=k_in, k=row) = x
//                              (n-contiguous), the rows split over `splits` partial outputs.
// Epilogues: plain store; + bias; + bias then ReLU (torch._addmm_activation's order); and the
// ReLU-backward of the layer BELOW fused into a dX product: C = mask(m, n) > 0 ? acc : 0 with
// `mask` = that layer's ReLU output (this layer's input), plus the column sums of C per row tile
// (the layer below's bias-gradient partials, [M / BM, N], summed in row-tile order by
// ocppo_sum_splits_db) -- the separate ReLU-backward pass over [rows, N] disappears.
//
// Structure (gfx950, 256 CUs, 64-wide waves):
//   * workgroup = 4 waves in 2 x 2, output tile BM x BN = 32 FM x 32 FN, each wave (16 FM) x
//     (16 FN) = FM x FN accumulators of v_mfma_f32_16x16x4_f32 (exact f32 products, one
//     rounding per product);
//   * K in steps of 32: the next step's A / B tiles are loaded to registers (float4, whole 128-B
//     lines per 8 lanes) while this step's MFMAs run from LDS, then written to the other LDS
//     buffer; one barrier per step. LDS images keep the global orientation (no transpose pass):
//     a k-contiguous operand as [rows][32 + 4], an m/n-contiguous one as [32][rows + 16]; both
//     paddings make the one-float fragment reads (lane l: row l & 15, k l >> 4) bank-conflict
//     free. 2 workgroups per CU (73.7 KB LDS each at 128 x 128);
//   * XCD-aware order: each XCD gets a contiguous range of work units, consecutive units share
//     their A row tile (or, split-K, their row chunk), so each XCD's L2 holds what its CUs share.
// Roofline: MFMA-bound (2 M N K flops; f32 MFMA peak 157.3 TFLOP/s, 64 flop/clk/SIMD).
#include "ocppo_common.h"

namespace ocppo {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kGemmBK = 32;
constexpr int kGemmThreads = 256;

struct GemmArgs {
  const float* a;
  int64_t sam, sak;  // A(m, k) = a[m * sam + k * sak]
  const float* b;
  int64_t sbn, sbk;  // B(n, k) = b[n * sbn + k * sbk]
  float* c;
  int64_t ldc;       // C[m, n] = c[m * ldc + n]
  const float* bias;
  const float* mask;
  int64_t ldmask;
  float* dbp;        // [M / BM, N]
  int epi;
  int M, N, K;       // K: reduction length of ONE split
  int tiles_m, tiles_n, units;
  int64_t split_a, split_b, split_c;  // element offsets of split s: s * split_*
};

template <int FM, int FN, bool AKC, bool BKC>
struct GemmCfg {
  static constexpr int BM = 32 * FM, BN = 32 * FN, BK = kGemmBK;
  static constexpr int LDA = AKC ? BK + 4 : BM + 4;  // LDS row stride (floats)
  static constexpr int LDB = BKC ? BK + 4 : BN + 4;
  static constexpr int A_ELEMS = AKC ? BM * LDA : BK * LDA;
  static constexpr int B_ELEMS = BKC ? BN * LDB : BK * LDB;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;  // one buffer, floats
  static constexpr int LA = BM * BK / 4 / kGemmThreads;  // float4 loads per thread per step
  static constexpr int LB = BN * BK / 4 / kGemmThreads;
  static_assert(LA >= 1 && LB >= 1, "tile too small for 256 threads");
};

// global -> registers: the float4 pieces of one operand tile of one K step
template <int ROWS, bool KC, int L>
__device__ __forceinline__ void gemm_load(const float* __restrict__ p, int64_t srow, int64_t sk,
                                          int row0, int k0, int t, floatx4 (&r)[L]) {
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int f = t + kGemmThreads * j;
    if constexpr (KC) {  // [ROWS][32]: 8 float4 per row
      const int row = f >> 3, kq = f & 7;
      r[j] = *reinterpret_cast<const floatx4*>(p + static_cast<int64_t>(row0 + row) * srow + k0 + 4 * kq);
    } else {             // [32][ROWS]: ROWS / 4 float4 per k row
      const int kr = f / (ROWS / 4), q = f % (ROWS / 4);
      r[j] = *reinterpret_cast<const floatx4*>(p + static_cast<int64_t>(k0 + kr) * sk + row0 + 4 * q);
    }
  }
}

template <int ROWS, bool KC, int LD, int L>
__device__ __forceinline__ void gemm_stash(float* s, int t, const floatx4 (&r)[L]) {
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int f = t + kGemmThreads * j;
    if constexpr (KC) {
      const int row = f >> 3, kq = f & 7;
      *reinterpret_cast<floatx4*>(s + row * LD + 4 * kq) = r[j];
    } else {
      const int kr = f / (ROWS / 4), q = f % (ROWS / 4);
      *reinterpret_cast<floatx4*>(s + kr * LD + 4 * q) = r[j];
    }
  }
}

// One 16-k group h of a wave's fragments, read as 16-B (or 8-B) LDS words. The MFMA k slot of
// lane l (fk = l >> 4) holds real k = 16 h + 4 fk + j in MFMA j of the group (j = 0..3), the same
// permutation on both operands, so the 4 MFMAs of a group cover its 16 k values.
//   k-contiguous image [row][k]: v[f] = the lane's 4 k values of fragment f (row 16 f + fr);
//   m/n-contiguous image [k][row]: v[j] = fragments 0..F-1 at k slot j, fragment f's lane fr
//     holding row F fr + f (rows permuted within the wave tile: one LDS word feeds F fragments).
template <int F, bool KC, int LD>
__device__ __forceinline__ void gemm_frags(const float* s, int row0, int h, int fr, int fk,
                                           floatx4 (&v)[4]) {
  if constexpr (KC) {
#pragma unroll
    for (int f = 0; f < F; ++f)
      v[f] = *reinterpret_cast<const floatx4*>(s + (row0 + 16 * f + fr) * LD + 16 * h + 4 * fk);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* p = s + (16 * h + 4 * fk + j) * LD + row0 + F * fr;
      if constexpr (F == 4) {
        v[j] = *reinterpret_cast<const floatx4*>(p);
      } else {
        const float2 t = *reinterpret_cast<const float2*>(p);
        v[j] = floatx4{t.x, t.y, 0.f, 0.f};
      }
    }
  }
}

template <bool KC>
__device__ __forceinline__ float gemm_fval(const floatx4 (&v)[4], int f, int j) {
  return KC ? v[f][j] : v[j][f];
}

template <int FM, int FN, bool AKC, bool BKC>
__global__ __launch_bounds__(kGemmThreads) void gemm_kernel(GemmArgs g) {
  using C = GemmCfg<FM, FN, AKC, BKC>;
  extern __shared__ __attribute__((aligned(16))) float gsm[];
  // XCD-aware bijective remap: workgroups b, b + 8, ... share an XCD; XCD x gets units
  // [start(x), start(x) + count(x)) in order
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nb >> 3, rr = nb & 7;
  const int u = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  if (u >= g.units) return;
  const int per_split = g.tiles_m * g.tiles_n;
  const int s = u / per_split, rem = u - s * per_split;
  const int tm = rem / g.tiles_n, tn = rem - tm * g.tiles_n;
  const int m0 = tm * C::BM, n0 = tn * C::BN;
  const float* __restrict__ A = g.a + s * g.split_a;
  const float* __restrict__ B = g.b + s * g.split_b;

  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int fr = lane & 15, fk = lane >> 4;

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  floatx4 ra[C::LA], rb[C::LB];
  const int nk = g.K / C::BK;
  gemm_load<C::BM, AKC, C::LA>(A, g.sam, g.sak, m0, 0, t, ra);
  gemm_load<C::BN, BKC, C::LB>(B, g.sbn, g.sbk, n0, 0, t, rb);
  gemm_stash<C::BM, AKC, C::LDA, C::LA>(gsm, t, ra);
  gemm_stash<C::BN, BKC, C::LDB, C::LB>(gsm + C::A_ELEMS, t, rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    // the next step's tiles (the last step re-loads its own: unconditional code keeps the
    // staging registers out of scratch)
    const int kn = (kt + 1 < nk ? kt + 1 : kt) * C::BK;
    gemm_load<C::BM, AKC, C::LA>(A, g.sam, g.sak, m0, kn, t, ra);
    gemm_load<C::BN, BKC, C::LB>(B, g.sbn, g.sbk, n0, kn, t, rb);
    // keep the loads at the top: left to itself the scheduler sinks them behind the MFMAs, next
    // to the LDS writes that consume them, and every step then waits out a full L2 / HBM trip
    __builtin_amdgcn_sched_barrier(0);
    const float* sa = gsm + (kt & 1) * C::STAGE;
    const float* sb = sa + C::A_ELEMS;
#pragma unroll
    for (int h = 0; h < C::BK / 16; ++h) {
      floatx4 av[4], bv[4];
      gemm_frags<FM, AKC, C::LDA>(sa, wm * (16 * FM), h, fr, fk, av);
      gemm_frags<FN, BKC, C::LDB>(sb, wn * (16 * FN), h, fr, fk, bv);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int jj = 0; jj < FN; ++jj)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                gemm_fval<AKC>(av, i, j), gemm_fval<BKC>(bv, jj, j), acc[i][jj], 0, 0, 0);
    }
    float* da = gsm + ((kt + 1) & 1) * C::STAGE;
    gemm_stash<C::BM, AKC, C::LDA, C::LA>(da, t, ra);
    gemm_stash<C::BN, BKC, C::LDB, C::LB>(da + C::A_ELEMS, t, rb);
    __syncthreads();
  }

  // epilogue: MFMA result C[4 fk + r][fr] of fragment (i, jj), mapped back through the row /
  // column permutations of the m/n-contiguous operand images
  float* __restrict__ Cp = g.c + s * g.split_c;
  const int wr0 = m0 + wm * (16 * FM), wc0 = n0 + wn * (16 * FN);
  auto row_of = [&](int i, int r) { return AKC ? wr0 + 16 * i + 4 * fk + r : wr0 + FM * (4 * fk + r) + i; };
  auto col_of = [&](int jj) { return BKC ? wc0 + 16 * jj + fr : wc0 + FN * fr + jj; };
  if (g.epi == OCPPO_GEMM_MASK_DB) {
    float colsum[FN];
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) colsum[jj] = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row_of(i, r);
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) {
          const int col = col_of(jj);
          const float mk = g.mask[row * g.ldmask + col];
          const float v = mk > 0.f ? acc[i][jj][r] : 0.f;
          Cp[row * g.ldc + col] = v;
          colsum[jj] += v;
        }
      }
    }
    // the 4 row groups of the wave (lanes fr, fr + 16, fr + 32, fr + 48), fixed order
#pragma unroll
    for (int jj = 0; jj < FN; ++jj) {
      colsum[jj] += __shfl_xor(colsum[jj], 16, kWave);
      colsum[jj] += __shfl_xor(colsum[jj], 32, kWave);
    }
    // the two row halves of the tile (wm = 0, 1) through LDS, in wm order
    float* red = gsm;  // the K loop ended with a barrier: the staging buffers are free
    if (wm == 1 && fk == 0) {
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) red[col_of(jj) - n0] = colsum[jj];
    }
    __syncthreads();
    if (wm == 0 && fk == 0) {
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        const int lc = col_of(jj) - n0;
        g.dbp[static_cast<int64_t>(tm) * g.N + n0 + lc] = colsum[jj] + red[lc];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = row_of(i, r);
      float v[FN];
#pragma unroll
      for (int jj = 0; jj < FN; ++jj) {
        v[jj] = acc[i][jj][r];
        if (g.epi != OCPPO_GEMM_STORE) v[jj] = v[jj] + g.bias[col_of(jj)];
        if (g.epi == OCPPO_GEMM_BIAS_RELU) v[jj] = fmaxf(v[jj], 0.f);
      }
      if constexpr (!BKC && FN == 4) {  // 4 consecutive columns per lane
        *reinterpret_cast<float4*>(Cp + row * g.ldc + col_of(0)) = make_float4(v[0], v[1], v[2], v[3]);
      } else if constexpr (!BKC && FN == 2) {
        *reinterpret_cast<float2*>(Cp + row * g.ldc + col_of(0)) = make_float2(v[0], v[1]);
      } else {
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) Cp[row * g.ldc + col_of(jj)] = v[jj];
      }
    }
  }
}

template <int FM, int FN, bool AKC, bool BKC>
static void launch_gemm_t(hipStream_t st, const GemmArgs& g) {
  using C = GemmCfg<FM, FN, AKC, BKC>;
  const size_t lds = sizeof(float) * 2 * C::STAGE;
  hipLaunchKernelGGL((gemm_kernel<FM, FN, AKC, BKC>), dim3(g.units), dim3(kGemmThreads), lds, st, g);
}

template <int FM, int FN>
static void launch_gemm_f(hipStream_t st, bool akc, bool bkc, const GemmArgs& g) {
  if (akc && bkc) launch_gemm_t<FM, FN, true, true>(st, g);
  else if (akc) launch_gemm_t<FM, FN, true, false>(st, g);
  else if (bkc) launch_gemm_t<FM, FN, false, true>(st, g);
  else launch_gemm_t<FM, FN, false, false>(st, g);
}

// tile choice: the configuration whose busiest CU (2 workgroups per CU) has the least work,
// larger tiles on ties (less L2 traffic per flop)
static int gemm_auto_tile(int64_t M, int64_t N, int64_t splits) {
  static const int cand[4] = {44, 42, 24, 22};
  int best = 0;
  double best_t = 1e30;
  for (int c : cand) {
    const int bm = 32 * (c / 10), bn = 32 * (c % 10);
    if (M % bm || N % bn) continue;
    const int64_t units = (M / bm) * (N / bn) * splits;
    const int64_t per_cu = (units + 255) / 256;                // tiles on the busiest CU
    const double t = static_cast<double>(per_cu) * bm * bn * (1.0 + 0.15 * (64.0 / bm + 64.0 / bn));
    if (t < best_t - 1e-9) { best_t = t; best = c; }
  }
  return best;
}

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_gemm_tile(int64_t M, int64_t N, int64_t splits) {
  if (M <= 0 || N <= 0 || splits <= 0) return 0;
  return gemm_auto_tile(M, N, splits);
}

extern "C" int ocppo_gemm(ocppo_stream_t stream, int64_t M, int64_t N, int64_t K,
                          const float* a, int64_t sam, int64_t sak, const float* b, int64_t sbn,
                          int64_t sbk, float* c, int64_t ldc, int64_t splits,
                          int64_t split_stride_c, int epilogue, const float* bias,
                          const float* mask, int64_t ldmask, float* dbp, int tile) {
  OCPPO_REQUIRE(M >= 1 && N >= 1 && K >= 1 && splits >= 1 && M <= INT32_MAX && N <= INT32_MAX &&
                    K <= INT32_MAX,
                "ocppo_gemm: bad sizes M=%lld N=%lld K=%lld splits=%lld", (long long)M,
                (long long)N, (long long)K, (long long)splits);
  OCPPO_REQUIRE(a && b && c, "ocppo_gemm: null operand");
  OCPPO_REQUIRE((sak == 1 && sam >= K && sam % 4 == 0) || (sam == 1 && sak >= M && sak % 4 == 0),
                "ocppo_gemm: A strides (sam=%lld, sak=%lld): one must be 1, the other a multiple "
                "of 4 covering the row", (long long)sam, (long long)sak);
  OCPPO_REQUIRE((sbk == 1 && sbn >= K && sbn % 4 == 0) || (sbn == 1 && sbk >= N && sbk % 4 == 0),
                "ocppo_gemm: B strides (sbn=%lld, sbk=%lld): one must be 1, the other a multiple "
                "of 4 covering the row", (long long)sbn, (long long)sbk);
  OCPPO_REQUIRE(ldc >= N && ldc % 4 == 0 && reinterpret_cast<uintptr_t>(c) % 16 == 0,
                "ocppo_gemm: C must be 16-B aligned with ldc (%lld) >= N and a multiple of 4",
                (long long)ldc);
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(a) % 16 == 0 && reinterpret_cast<uintptr_t>(b) % 16 == 0,
                "ocppo_gemm: A and B must be 16-B aligned");
  OCPPO_REQUIRE(epilogue >= OCPPO_GEMM_STORE && epilogue <= OCPPO_GEMM_MASK_DB,
                "ocppo_gemm: unknown epilogue %d", epilogue);
  OCPPO_REQUIRE(epilogue == OCPPO_GEMM_STORE || splits == 1,
                "ocppo_gemm: split-K partial outputs take the plain-store epilogue only");
  OCPPO_REQUIRE(epilogue != OCPPO_GEMM_BIAS && epilogue != OCPPO_GEMM_BIAS_RELU || bias,
                "ocppo_gemm: bias epilogue without a bias");
  OCPPO_REQUIRE(epilogue != OCPPO_GEMM_MASK_DB || (mask && dbp && ldmask >= N),
                "ocppo_gemm: mask epilogue needs mask (ldmask >= N) and dbp");
  OCPPO_REQUIRE(splits == 1 || split_stride_c >= (M - 1) * ldc + N,
                "ocppo_gemm: split_stride_c=%lld overlaps the partial outputs",
                (long long)split_stride_c);
  if (tile == 0) tile = gemm_auto_tile(M, N, splits);
  OCPPO_REQUIRE(tile == 44 || tile == 42 || tile == 24 || tile == 22,
                "ocppo_gemm: no tile fits M=%lld N=%lld (tile %d; M, N multiples of 64 needed)",
                (long long)M, (long long)N, tile);
  const int bm = 32 * (tile / 10), bn = 32 * (tile % 10);
  OCPPO_REQUIRE(M % bm == 0 && N % bn == 0 && K % (splits * kGemmBK) == 0,
                "ocppo_gemm: M=%lld %% %d, N=%lld %% %d, K=%lld %% (32 x splits=%lld) must be 0",
                (long long)M, bm, (long long)N, bn, (long long)K, (long long)splits);
  const int64_t units = (M / bm) * (N / bn) * splits;
  OCPPO_REQUIRE(units <= INT32_MAX, "ocppo_gemm: too many tiles");
  GemmArgs g;
  const int64_t ks = K / splits;
  g.a = a; g.sam = sam; g.sak = sak;
  g.b = b; g.sbn = sbn; g.sbk = sbk;
  g.c = c; g.ldc = ldc;
  g.bias = bias; g.mask = mask; g.ldmask = ldmask; g.dbp = dbp; g.epi = epilogue;
  g.M = (int)M; g.N = (int)N; g.K = (int)ks;
  g.tiles_m = (int)(M / bm); g.tiles_n = (int)(N / bn); g.units = (int)units;
  g.split_a = ks * sak; g.split_b = ks * sbk; g.split_c = split_stride_c;
  const bool akc = sak == 1, bkc = sbk == 1;
  clear_stale_error();
  hipStream_t st = as_stream(stream);
  switch (tile) {
    case 44: launch_gemm_f<4, 4>(st, akc, bkc, g); break;
    case 42: launch_gemm_f<4, 2>(st, akc, bkc, g); break;
    case 24: launch_gemm_f<2, 4>(st, akc, bkc, g); break;
    default: launch_gemm_f<2, 2>(st, akc, bkc, g); break;
  }
  return check_launch("ocppo_gemm");
}
