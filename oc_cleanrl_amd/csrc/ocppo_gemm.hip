// Update-phase f32 GEMMs of the PPObj / NatureCNN-head Linear layers on the bf16 matrix cores
// (cleanrl/ppo_atari_oc.py:566-606: the minibatch forward `agent.get_action_and_value(b_obs[mb])`
// through architectures/ppo.py:60-84 and its `loss.backward()`; the reference's Linear layers are
// torch.float32 with TF32 off, i.e. f32 products).
//
//   C[m, n] = epilogue( sum_k A(m, k) B(n, k) )
//
// gfx950 has no TF32/xf32 matrix path; its f32 MFMA runs at 1/16 of the bf16 MFMA rate
// (157 vs 2,500 TFLOP/s dense, MI355X_MICROARCH.md). Every f32 operand is therefore split EXACTLY
// into three bf16 pieces, x = x0 + x1 + x2 (x0 = rn_bf16(x), x1 = rn_bf16(x - x0), x2 = x - x0 - x1:
// 3 x 8 significand bits hold f32's 24, each subtraction is exact), and the product is formed from
// the six piece products down to the f32 rounding level:
//   a*b = a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0) + [a1 b2 + a2 b1 + a2 b2]
// The bracketed terms are dropped: |a1 b2| <= 2^-8 * 2^-16 |a b| = 2^-24 |a b| (half an f32 ulp of
// the product at most, ~2^-28 typically, randomly signed), below the per-product rounding a plain
// f32 FMA chain already makes. Every piece product is exact in f32 (8 x 8 bits) and is accumulated
// by the MFMA in f32. The shipped variants (tile bit 4, and the mixed tiles) accumulate all six
// products into ONE f32 accumulator per output (small terms issued before the lead one in each K
// step): the accumulation then rounds like an f32 FMA chain over 6 K terms per k, measured at or
// below hipBLASLt's f32 GEMM error vs f64 up to K = 4096 (tests/test_gemm_gpu.py). The two-
// accumulator variants (bit 4 clear) keep the five small products in a second accumulator
// (x 2^-8 in magnitude), added once at the end: 3x more accurate, 0-5 % slower. Six bf16 MFMAs = 6/16 of one f32 MFMA's time for the same
// output: the f32-equivalent ceiling is 2,500 / 6 = 417 TFLOP/s against 157 for the f32 MFMA.
// tests/test_gemm_gpu.py measures the error against an f64 product next to hipBLASLt's f32 GEMM.
//
// A(m, k) and B(n, k) are strided views (one of the two strides is 1), so one kernel covers the
// three products of a Linear layer without transposing anything in HBM:
//   forward  y  = x W^T        A = x  [M, K] (k-contiguous), B = W [N, K] (k-contiguous)
//   dX       dx = g' W         A = g' [M, N] (k-contiguous), B(n=k_in, k=n_out) = W (n-contiguous)
//   dW       dW = g'^T x       A(m=n_out, k=row) = g' (m-contiguous), B(n=k_in, k=row) = x
//                              (n-contiguous), the rows (K steps of 32) split evenly over
//                              `splits` partial outputs that ocppo_sum_splits[_db] combines in
//                              split order.
//
// Structure (gfx950, 256 CUs, 64-wide waves):
//   * workgroup = 4 waves in 2 x 2, output tile BM x BN = 32 FM x 32 FN, wave tile 16 FM x 16 FN
//     = FM x FN blocks of v_mfma_f32_16x16x32_bf16, each with a lead and a small-term accumulator;
//   * K in steps of 32 (one MFMA depth): the next step's f32 tiles are loaded into registers while
//     this step's MFMAs run from LDS; then (between two barriers) they are split and written as
//     three bf16 planes [rows][32] per operand. A thread stages 4 x 4 (row, k) pieces: four 16-B
//     loads along the contiguous dimension (whole 128-B lines per 8 lanes for a k-contiguous
//     operand, 512-B runs per 32 lanes for an m/n-contiguous one, transposed in registers), then
//     one 8-B LDS write per row and plane. The plane rows are stored in 128-B pairs with a
//     3-bit XOR swizzle of their 16-B chunks (x6_chunk_off), so the fragment reads (lane l:
//     row l % 16, chunk l / 16, one ds_read_b128) and the stash writes are bank-conflict free;
//   * XCD-aware order: each XCD gets a contiguous range of work units, consecutive units share
//     their A row tile, so each XCD's L2 holds what its CUs share.
// Roofline: MFMA-bound (6 bf16 MFMA passes per f32 multiply-add: 12 M N K bf16 flops against
// the 2.5 PFLOP/s dense bf16 peak).
#include <algorithm>

#include "ocppo_common.h"
#include "ocppo_x6split.h"

namespace ocppo {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kX6BK = 32;       // K step = one MFMA depth

struct X6Args {
  const float* a;
  int64_t sam, sak;  // A(m, k) = a[m * sam + k * sak]
  const float* b;
  int64_t sbn, sbk;  // B(n, k) = b[n * sbn + k * sbk]
  float* c;
  int64_t ldc;       // C[m, n] = c[m * ldc + n]
  const float* bias;
  int relu;
  int M, N, K;       // K: the whole reduction length (K / 32 steps, split evenly over splits)
  int tiles_m, tiles_n, units, splits;
  int64_t split_c;   // element offset of split s's output: s * split_c
  // mask epilogue (dX of the layer above a Linear+ReLU): C = mask > 0 ? acc : 0 and the column
  // sums of C over each row tile into dbp[tile_m, N] (that layer's bias-gradient partials)
  const float* mask;
  int64_t ldm;
  float* dbp;
  // ReLU bitmasks in the MFMA fragment layout: bit (i FN + j) 4 + r of word [tile][thread] is
  // element (block i, j; register r) of that thread's accumulators, > 0. A forward with a ReLU
  // epilogue writes them (mbits_out); the next layer's dX, the same tile shape over the same
  // [M, N], reads them (mbits_in) instead of the f32 mask: 1 bit instead of 4 B per element.
  uint64_t* mbits_out;
  const uint64_t* mbits_in;
  // mixed tiles (variant bit 5): rows [0, mbig) in 128 x 128 tiles, dispatched first, the rest
  // in 64 x 128 tiles; dbp rows and mask words are then counted in 64-row tiles
  int mbig;
  // B pre-split (ocppo_split_planes): piece p of B(n, k) at bpl[p * bpl_ps + n * bpl_ld + k]
  const uint16_t* bpl;
  int64_t bpl_ld, bpl_ps;
  // gathered operand rows (ocppo_gemm_x6_gather): the operand's K (mode 1, A) or N (mode 2, B)
  // dimension is gw segments of gseg, segment s of row r read from source row gidx[r * gw + s]
  const int32_t* gidx;
  int64_t gw, gseg;
  // wgrad epilogue (ocppo_gemm_x6_wgrad): the product is the dX of a layer above a Linear+ReLU
  // whose input rows wx [M, wk] need no gradient; instead of writing dX, each tile writes that
  // layer's weight / bias-gradient partials (the relu_bias_wgrad record layout, record = row tile)
  const float* wx;
  int64_t ldwx;
  int wk;
  float* wrec;
  int64_t wnpw;
  // probe builds only (-DOCPPO_X6_STAMPS, tools/exp_x6_stamps.py): per workgroup clock stamps
  int64_t* stamps;
  // stream-K (x6p persistent launches, sk != 0): partial-accumulator slots and their flags (one
  // per workgroup, zero between launches)
  int sk;
  float* skws;
  int* skflag;
  // mbits_out in the row-major layout instead (ocppo_gemm_x6's relu & OCPPO_X6_MBITS_ROWS): bit
  // n % 32 of 32-bit word [m][n / 32] is !(C[m, n] <= 0), for a consumer that walks the output
  // by rows (the frame scatter of the encoder's last ReLU backward, ocppo_frames_scatter_relu)
  int mbits_rows;
  // implicit-GEMM convolution (ocppo_conv_x6): operand rows r = (b, qy, qx) over [B, cv_qh, cv_qw]
  // of an NHWC tensor; element k of row r sits at cv_row(r) + cv_seg(k), with
  //   cv_row(r) = b cv_sb + qy cv_ys + qx cv_xs,  cv_seg(k) = (k / cv_gseg) cv_segs + k % cv_gseg
  // (a segment = one kernel row's KW x C taps, contiguous in NHWC). GATH 3: A's rows (forward /
  // data gradient, k-contiguous within a segment); GATH 4: B's K index (weight gradient, B(n, k) =
  // x[cv_row(k) + cv_seg(n)]). cv_out: C row r written at b co_sb + qy co_ys + qx co_xs + co_off
  // (GATH 3: one stride class of a strided convolution's data gradient) instead of r ldc.
  // Output columns (cv_out): column n = (class c, channel n % co_cw) of a strided convolution's
  // data gradient, c = (py, px) with py = c / co_cs, px = c % co_cs, at offset py co_cy + px co_cx
  // + n % co_cw from the row's (all stride classes read the same gradient rows: one product)
  int cv_qh, cv_qw;
  int64_t cv_sb, cv_ys, cv_xs, cv_segs;
  int cv_gseg, cv_out;
  int64_t co_sb, co_ys, co_xs, co_off;
  int co_cw, co_cs;
  int64_t co_cy, co_cx;
  // the first convolution straight from the rollout's u8 frame stacks (GATH 5: A's rows; GATH 6:
  // B's K rows): sample b's stack is row u8_idx[b] of u8 [rows, C, H, W] (NCHW bytes, u8_img per
  // row); k (or n) = (c, ky, kx) in nn.Conv2d's weight order, at c u8_hw + ky u8_w + kx from the
  // window's corner (cv_row with cv_sb = 0: qy cv_ys + qx cv_xs bytes). The bytes are exact in
  // bf16; the products are divided by cdiv (255: NormalizeImg) in the epilogue (GATH 5) or in the
  // split sum (GATH 6).
  // GATH 7 (the data gradient without a padded copy): the source is the unpadded output gradient
  // [B, cv_ih, cv_iw, C]; tap (ty, tx) of row (b, qy, qx) reads pixel (qy + ty - cv_ph, qx + tx -
  // cv_pw), zero outside (cv_row's offsets are taken from the padded corner)
  int cv_ph, cv_pw, cv_ih, cv_iw, cv_c;
  const uint8_t* u8;
  const int64_t* u8_idx;
  int64_t u8_img, u8_hw, u8_w;
  int u8_khw, u8_kw, u8_nimg;  // u8_nimg: entries of u8_idx (images)
  float cdiv;
  // bounds-check builds only (-DOCPPO_X6_BOUNDS, ocppo_x6_probe_set_bounds): the extents of the
  // convolution gathers' sources from the pointers passed (elements of the f32 operand the
  // gathers read, bytes and rows of the u8 stacks), and a violation record [count, first kind,
  // first index lo, hi, first limit lo, hi]
  uint32_t* bnd;
  int64_t bnd_x, bnd_u8, bnd_u8rows;
};

// Bounds-check builds: every index a convolution gather computes (image index, u8 stack row,
// element / byte offset of a load) is checked against its extent before the load; a violation
// is counted and recorded (the first one) and the load reads offset 0 instead, so a bad index
// shows as a record, not as a fault. Compiled out otherwise (the identity).
enum X6BoundKind { kBndX = 1, kBndImg = 2, kBndU8Row = 3, kBndU8 = 4 };
__device__ __forceinline__ int64_t bnd_check(uint32_t* bnd, int kind, int64_t v, int64_t need,
                                             int64_t lim) {
#ifdef OCPPO_X6_BOUNDS
  if (bnd != nullptr && (v < 0 || v + need > lim)) {
    if (__hip_atomic_fetch_add(bnd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      bnd[1] = static_cast<uint32_t>(kind);
      bnd[2] = static_cast<uint32_t>(static_cast<uint64_t>(v));
      bnd[3] = static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32);
      bnd[4] = static_cast<uint32_t>(static_cast<uint64_t>(lim));
      bnd[5] = static_cast<uint32_t>(static_cast<uint64_t>(lim) >> 32);
    }
    return 0;
  }
#else
  (void)bnd, (void)kind, (void)need, (void)lim;
#endif
  return v;
}
__device__ __forceinline__ int64_t x6_bnd(const X6Args& g, int kind, int64_t v, int64_t need,
                                          int64_t lim) {
  return bnd_check(g.bnd, kind, v, need, lim);
}

// q = x / d for 0 <= x < 2^24, d >= 1 (f32 reciprocal estimate, corrected to the exact quotient)
__device__ __forceinline__ int x6_udiv(int x, int d) {
  int q = static_cast<int>(static_cast<float>(x) * __builtin_amdgcn_rcpf(static_cast<float>(d)));
  int r = x - q * d;
  while (r < 0) {
    --q;
    r += d;
  }
  while (r >= d) {
    ++q;
    r -= d;
  }
  return q;
}
// (b, qy, qx) of convolution row r
__device__ __forceinline__ void x6_cv_split(const X6Args& g, int r, int& b, int& qy, int& qx) {
  const int qhw = g.cv_qh * g.cv_qw;
  b = x6_udiv(r, qhw);
  const int p = r - b * qhw;
  qy = x6_udiv(p, g.cv_qw);
  qx = p - qy * g.cv_qw;
}
__device__ __forceinline__ int64_t x6_cv_row(const X6Args& g, int r) {
  int b, qy, qx;
  x6_cv_split(g, r, b, qy, qx);
  return b * g.cv_sb + qy * g.cv_ys + qx * g.cv_xs;
}
__device__ __forceinline__ int64_t x6_cv_seg(const X6Args& g, int k) {
  const int s = k / g.cv_gseg;
  return s * g.cv_segs + (k - s * g.cv_gseg);
}

// Stream-K geometry of an x6p persistent launch: the tiles (row-major) are dealt to the 8 XCDs in
// contiguous ranges; XCD x's P = grid / 8 workgroups (blockIdx b: XCD b % 8, rank b / 8) share
// its tiles' K steps evenly, each a contiguous range [r I / P, (r + 1) I / P) of I = tiles x nk
struct X6pGeom {
  int xcd, rank, P, t0, t1, nk;
  int64_t I;
};
__device__ __forceinline__ X6pGeom x6p_geom(const X6Args& g, int b, int grid) {
  X6pGeom q;
  q.xcd = b & 7;
  q.rank = b >> 3;
  q.P = grid >> 3;
  const int T = g.tiles_m * g.tiles_n;
  q.t0 = q.xcd * T / 8;
  q.t1 = (q.xcd + 1) * T / 8;
  q.nk = g.K / kX6BK;
  q.I = static_cast<int64_t>(q.t1 - q.t0) * q.nk;
  return q;
}


#ifdef OCPPO_X6_STAMPS
// stamp s of the workgroup (thread 0): [0] start, [1] prologue done, [2] K loop done, [3] stores
// done (shader clock), [4] / [5] start / end on the 100 MHz real-time clock
#define X6_STAMP(g, s, v)                                                            \
  do {                                                                               \
    if ((g).stamps && threadIdx.x == 0) (g).stamps[blockIdx.x * 8 + (s)] = (v);      \
  } while (0)
#else
#define X6_STAMP(g, s, v) \
  do {                    \
  } while (0)
#endif

// Where one tile's outputs go: its row tiles start at row0_base, its dbp partial row is
// db_base + db_mult tm (db_mult 2: the second of the two 64-row partials is written as zeros),
// its mask words at (id_base + tile id) x threads
struct X6Place {
  int tiles_m, row0_base, db_base, db_mult;
  int64_t id_base;
  // stream-K segment (x6p persistent launches): mode -1 = the unit u as usual; else tile seg_tile,
  // K steps [seg_kb, seg_kb + seg_nk), and mode 0 = the whole tile (epilogue), 1 = a later part
  // of a split tile (partial accumulators to workspace slot seg_slot, then its flag), 2 = the
  // tile's first part (adds the later parts' partials, then the epilogue)
  int seg_mode = -1, seg_tile = 0, seg_kb = 0, seg_nk = 0, seg_slot = 0;
};

// x6f2 / x6_pk / x6_unpk / x6_split2: the exact three-way bf16 split (ocppo_x6split.h, shared
// with the optimizer's plane writes)

// LDS plane layout: rows in pairs of 128 B (row r's 64 B = 16-B chunks 4 (r & 1) .. + 3 of pair
// r / 2), chunk index XOR-swizzled by H(r) = bitrev3((r / 4) % 8). Found by exhaustive search
// over the 8! chunk maps (tools/x6_swizzle.py) so that, with the piece mappings of X6Stage, every
// ds_read_b128 fragment read (its four 16-lane groups) and every ds_write_b64 stash write (four
// 16 x 8-B groups, k- or row-contiguous operand) touches each bank once: no conflicts.
__device__ __forceinline__ int x6_h(int row) {
  const int x = (row >> 2) & 7;
  return ((x & 1) << 2) | (x & 2) | (x >> 2);
}
// byte offset of 16-B chunk `chunk` (k = 8 chunk .. + 7) of plane row `row`
__device__ __forceinline__ int x6_chunk_off(int row, int chunk) {
  return (row >> 1) * 128 + 16 * ((((row & 1) << 2) | chunk) ^ x6_h(row));
}
// byte offset of (row, k..k+3), k % 4 == 0
__device__ __forceinline__ int x6_off(int row, int k) {
  return x6_chunk_off(row, k >> 3) + (k & 4) * 2;
}

// One operand tile [ROWS][32 k] of one K step: PR x 4 (row, k) pieces per thread (PR = 4; a
// k-contiguous operand may use PR = 1, one 16-B row quad per piece, so that every thread of an
// 8-wave workgroup stages the same share of a 128- or 256-row tile).
template <int ROWS, bool KC, int NT, int PR = 4>
struct X6Stage {
  static_assert(ROWS % 32 == 0, "tile rows must be a multiple of 32");
  static_assert(PR == 4 || (PR == 1 && KC), "row-quad pieces are for a k-contiguous operand");
  static constexpr int kPR = PR;
  static constexpr int kPieces = ROWS / PR * 8;
  static constexpr int kPer = (kPieces + NT - 1) / NT;
  static constexpr int kPlane = ROWS * 64;  // bytes per bf16 plane

  __device__ static void piece_of(int p, int& rq, int& kq) {
    if constexpr (KC) {  // k quads fastest: 8 lanes read one row's 128 B
      kq = p & 7;
      rq = p >> 3;  // rows PR rq .. PR rq + PR - 1
    } else {  // 8 row quads x 2 k quads per 16 lanes: 8 lanes read 128 contiguous bytes of a
              // k row (the mapping the swizzle's conflict-free stash writes assume)
      constexpr int kRqBlocks = ROWS / 32;  // blocks of 8 row quads
      rq = (p & 7) + 8 * ((p >> 4) % kRqBlocks);
      kq = ((p >> 3) & 1) + 2 * ((p >> 4) / kRqBlocks);
    }
  }

  // every wave issues the same number of loads (a counted vmcnt is per wave)
  static constexpr bool kUniform = kPieces % NT == 0;

  template <bool ASM = false>
  __device__ static void load(const float* __restrict__ src, int64_t srow, int64_t sk, int row0,
                              int k0, int t, floatx4 (&r)[kPer][4]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
      int rq, kq;
      piece_of(p, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= PR) break;
        const float* q = KC ? src + static_cast<int64_t>(row0 + PR * rq + j) * srow + (k0 + 4 * kq)
                            : src + static_cast<int64_t>(k0 + 4 * kq + j) * sk + (row0 + 4 * rq);
        if constexpr (ASM)  // invisible to the compiler's wait insertion: waited by x6_vmwait
          asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r[i][j]) : "v"(q) : "memory");
        else
          r[i][j] = *reinterpret_cast<const floatx4*>(q);
      }
    }
  }

  // Buffer-resource form of load: the piece offsets are fixed per unit (VGPRs, set once) and the
  // K advance is the scalar offset, so a step's loads need no 64-bit address VALU (41 fewer
  // v_lshl_add_u64 in the forward kernel). Base = the unit's first (row, k) element; the host
  // checks that a unit's window fits the 32-bit offsets (x6_windows_ok).
  struct Buf {
    __amdgpu_buffer_rsrc_t rs;
    int32_t vo[kPer][4];
  };
  __device__ static void buf_setup(const float* __restrict__ src, int64_t srow, int64_t sk,
                                   int row0, int kbase, int t, Buf& b) {
    const float* base = KC ? src + static_cast<int64_t>(row0) * srow + kbase
                           : src + static_cast<int64_t>(kbase) * sk + row0;
    b.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b.vo[i][j] = static_cast<int32_t>(4 * (KC ? (PR * rq + (j < PR ? j : 0)) * srow + 4 * kq
                                                  : (4 * kq + j) * sk + 4 * rq));
    }
  }
  __device__ static void load_buf(const Buf& b, int t, int32_t soff, floatx4 (&r)[kPer][4]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
#pragma unroll
      for (int j = 0; j < PR; ++j)
        r[i][j] = __builtin_bit_cast(
            floatx4, __builtin_amdgcn_raw_buffer_load_b128(b.rs, b.vo[i][j], soff, 0));
    }
  }

  // k-contiguous operand with gathered rows: roff[i][j] = element offset of piece row (i, j)
  // (its source row times the row stride, minus the segment start), fixed for a unit whose K
  // range lies in one segment
  __device__ static void gather_rows(const int32_t* __restrict__ gidx, int64_t gw, int seg,
                                     int64_t gseg, int64_t srow, int row0, int t,
                                     int64_t (&roff)[kPer][4]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        roff[i][j] = static_cast<int64_t>(gidx[static_cast<int64_t>(row0 + 4 * rq + j) * gw + seg]) *
                         srow - static_cast<int64_t>(seg) * gseg;
    }
  }
  __device__ static void load_rows(const float* __restrict__ src, const int64_t (&roff)[kPer][4],
                                   int k0, int t, floatx4 (&r)[kPer][4],
                                   const X6Args* bg = nullptr) {
    static_assert(KC, "row-gathered loads are for a k-contiguous operand");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
      int rq, kq;
      piece_of(p, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int64_t off = roff[i][j] + (k0 + 4 * kq);
        if (bg != nullptr) off = x6_bnd(*bg, kBndX, off, 4, bg->bnd_x);  // GATH 3 (bounds builds)
        r[i][j] = *reinterpret_cast<const floatx4*>(src + off);
      }
    }
  }
  // convolution rows of a k-contiguous operand (GATH 3): roff[i][j] = cv_row of piece row (i, j);
  // load_rows then takes cv_seg(k0) for k0 (a K step never straddles a segment)
  __device__ static void conv_rows(const X6Args& g, int row0, int t, int64_t (&roff)[kPer][4]) {
    static_assert(KC, "convolution rows are for a k-contiguous operand");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) roff[i][j] = x6_cv_row(g, row0 + 4 * rq + j);
    }
  }
  // GATH 7: conv_rows plus each piece row's (qy, qx) for the bounds; load_rows_bounded zero-fills
  // the taps outside the unpadded gradient
  __device__ static void conv_rows_b(const X6Args& g, int row0, int t, int64_t (&roff)[kPer][4],
                                     int (&qy)[kPer][4], int (&qx)[kPer][4]) {
    static_assert(KC, "convolution rows are for a k-contiguous operand");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int b;
        x6_cv_split(g, row0 + 4 * rq + j, b, qy[i][j], qx[i][j]);
        roff[i][j] = b * g.cv_sb + (qy[i][j] - g.cv_ph) * g.cv_ys + (qx[i][j] - g.cv_pw) * g.cv_xs;
      }
    }
  }
  __device__ static void load_rows_bounded(const float* __restrict__ src, const X6Args& g,
                                           const int64_t (&roff)[kPer][4], const int (&qy)[kPer][4],
                                           const int (&qx)[kPer][4], int k0, int t,
                                           floatx4 (&r)[kPer][4]) {
    const int ty = k0 / g.cv_gseg, w0 = k0 - ty * g.cv_gseg;
    const int64_t so = static_cast<int64_t>(ty) * g.cv_segs + w0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
      int rq, kq;
      piece_of(p, rq, kq);
      const int tx = (w0 + 4 * kq) / g.cv_c;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int iy = qy[i][j] + ty - g.cv_ph, ix = qx[i][j] + tx - g.cv_pw;
        const bool in = iy >= 0 && iy < g.cv_ih && ix >= 0 && ix < g.cv_iw;
        r[i][j] = in ? *reinterpret_cast<const floatx4*>(
                           src + x6_bnd(g, kBndX, roff[i][j] + so + 4 * kq, 4, g.bnd_x))
                     : floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  // row-contiguous operand whose K index is a convolution row (GATH 4): B(n, k) =
  // src[cv_row(k) + cv_seg(n)]; nseg[i] = cv_seg of piece i's 4 columns (one segment: cv_gseg %
  // 4 == 0), ptab[p] = qy cv_ys + qx cv_xs of the p-th pixel of an image (LDS)
  __device__ static void conv_cols(const X6Args& g, int row0, int t, int64_t (&nseg)[kPer]) {
    static_assert(!KC, "convolution K rows are for a row-contiguous operand");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
      nseg[i] = x6_cv_seg(g, row0 + 4 * rq);
    }
  }
  // the (image, pixel) of each of this thread's K rows at step k0 (load_conv_k then walks them
  // one K step of 32 rows per call: the loads of a unit are issued for consecutive steps)
  __device__ static void conv_k_state(const X6Args& g, int k0, int t, int (&cb)[kPer][4],
                                      int (&cp)[kPer][4]) {
    const int qhw = g.cv_qh * g.cv_qw;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kk = k0 + 4 * kq + j;
        cb[i][j] = x6_udiv(kk, qhw);
        cp[i][j] = kk - cb[i][j] * qhw;
      }
    }
  }
  __device__ static void load_conv_k(const float* __restrict__ src, const X6Args& g,
                                     const int64_t (&nseg)[kPer], const int32_t* ptab,
                                     int (&cb)[kPer][4], int (&cp)[kPer][4], int t,
                                     floatx4 (&r)[kPer][4]) {
    const int qhw = g.cv_qh * g.cv_qw;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t off = cb[i][j] * g.cv_sb + ptab[cp[i][j]];
        x6_bnd(g, kBndImg, cb[i][j], 1, g.K / (g.cv_qh * g.cv_qw));  // GATH 4: K rows = images
        r[i][j] = *reinterpret_cast<const floatx4*>(src + x6_bnd(g, kBndX, off + nseg[i], 4, g.bnd_x));
        cp[i][j] += kX6BK;  // the next step's row
        while (cp[i][j] >= qhw) {
          cp[i][j] -= qhw;
          ++cb[i][j];
        }
      }
    }
  }
  // u8 frame stacks, k-contiguous (GATH 5): roff[i][j] = byte offset of piece row (i, j)'s window
  // corner; segtab[q] = byte offset of taps 4q .. 4q + 3 (one kernel row: u8_kw % 4 == 0)
  __device__ static void u8_rows(const X6Args& g, int row0, int t, int64_t (&roff)[kPer][4]) {
    static_assert(KC, "u8 rows are for a k-contiguous operand");
    const int qhw = g.cv_qh * g.cv_qw;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = row0 + 4 * rq + j, b = x6_udiv(r, qhw), pix = r - b * qhw;
        const int qy = x6_udiv(pix, g.cv_qw);
        const int64_t img = g.u8_idx[x6_bnd(g, kBndImg, b, 1, g.u8_nimg)];
        roff[i][j] = x6_bnd(g, kBndU8Row, img, 1, g.bnd_u8rows) * g.u8_img + qy * g.cv_ys +
                     (pix - qy * g.cv_qw) * g.cv_xs;
      }
    }
  }
  __device__ static floatx4 u8x4(uint32_t v) {
    return floatx4{static_cast<float>(v & 0xffu), static_cast<float>((v >> 8) & 0xffu),
                   static_cast<float>((v >> 16) & 0xffu), static_cast<float>(v >> 24)};
  }
  __device__ static void load_u8_rows(const uint8_t* __restrict__ src,
                                      const int64_t (&roff)[kPer][4], const int32_t* segtab,
                                      int k0, int t, floatx4 (&r)[kPer][4], const X6Args& g) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
      int rq, kq;
      piece_of(p, rq, kq);
      const int so = segtab[(k0 >> 2) + kq];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        r[i][j] = u8x4(*reinterpret_cast<const uint32_t*>(
            src + x6_bnd(g, kBndU8, roff[i][j] + so, 4, g.bnd_u8)));
    }
  }
  // u8 frame stacks as a row-contiguous operand whose K index is a convolution row (GATH 6):
  // nseg[i] = byte offset of piece i's 4 taps; (cb, cp) walk the K rows as conv_k_state's,
  // cbase = u8_idx[cb] u8_img
  __device__ static void u8_cols(const X6Args& g, int row0, int t, int64_t (&nseg)[kPer]) {
    static_assert(!KC, "u8 K rows are for a row-contiguous operand");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      int rq, kq;
      piece_of(p < kPieces ? p : 0, rq, kq);
      const int n = row0 + 4 * rq, c = n / g.u8_khw, rem = n - c * g.u8_khw, ky = rem / g.u8_kw;
      nseg[i] = c * g.u8_hw + ky * g.u8_w + (rem - ky * g.u8_kw);
    }
  }
  __device__ static void load_u8_k(const uint8_t* __restrict__ src, const X6Args& g,
                                   const int64_t (&nseg)[kPer], const int32_t* ptab,
                                   int (&cb)[kPer][4], int (&cp)[kPer][4],
                                   int64_t (&cbase)[kPer][4], int t, floatx4 (&r)[kPer][4]) {
    const int qhw = g.cv_qh * g.cv_qw;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x6_bnd(g, kBndImg, cb[i][j], 1, g.u8_nimg);
        r[i][j] = u8x4(*reinterpret_cast<const uint32_t*>(
            src + x6_bnd(g, kBndU8, cbase[i][j] + ptab[cp[i][j]] + nseg[i], 4, g.bnd_u8)));
        cp[i][j] += kX6BK;
        if (cp[i][j] >= qhw) {
          while (cp[i][j] >= qhw) {
            cp[i][j] -= qhw;
            ++cb[i][j];
          }
          // past the last image after the unit's last step: nothing reads it, and the index
          // array ends there (no read one past its end)
          cbase[i][j] = cb[i][j] < g.u8_nimg
                            ? x6_bnd(g, kBndU8Row, g.u8_idx[cb[i][j]], 1, g.bnd_u8rows) * g.u8_img
                            : 0;
        }
      }
    }
  }
  // row-contiguous operand whose K index (a sample row) picks a gathered source row:
  // B(n, k) = src[tbl[k - kbase] * sk + coff + n] (tbl = the unit's rows of gidx, in LDS)
  __device__ static void load_ktbl(const float* __restrict__ src, int64_t sk,
                                   const int32_t* tbl, int kbase, int64_t coff, int row0, int k0,
                                   int t, floatx4 (&r)[kPer][4]) {
    static_assert(!KC, "K-gathered loads are for a row-contiguous operand");
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = t + NT * i;
      if (kPieces % NT != 0 && p >= kPieces) continue;
      int rq, kq;
      piece_of(p, rq, kq);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t sr = tbl[k0 + 4 * kq + j - kbase];
        r[i][j] = *reinterpret_cast<const floatx4*>(src + sr * sk + coff + (row0 + 4 * rq));
      }
    }
  }

  // split row j (4 elements) of staged piece i and write it into the three planes; EXACT:
  // bf16-exact values (u8 bytes), the value itself is the lead piece and only plane 0 is written
  // (the products never read the others)
  template <bool PROBE = false, bool EXACT = false>
  __device__ static void stash_row(unsigned char* lds, int t, const floatx4 (&r)[kPer][4], int i,
                                   int j) {
    const int p = t + NT * i;
    if (kPieces % NT != 0 && p >= kPieces) return;
    int rq, kq;
    piece_of(p, rq, kq);
    const x6f2 v01 = KC ? x6f2{r[i][j][0], r[i][j][1]} : x6f2{r[i][0][j], r[i][1][j]};
    const x6f2 v23 = KC ? x6f2{r[i][j][2], r[i][j][3]} : x6f2{r[i][2][j], r[i][3][j]};
    if constexpr (EXACT) {
      const uint32_t e0 = __builtin_amdgcn_perm(__float_as_uint(v01.y), __float_as_uint(v01.x),
                                                0x07060302u);
      const uint32_t e1 = __builtin_amdgcn_perm(__float_as_uint(v23.y), __float_as_uint(v23.x),
                                                0x07060302u);
      *reinterpret_cast<uint2*>(lds + x6_off((KC ? PR : 4) * rq + j, 4 * kq)) = uint2{e0, e1};
      return;
    }
    uint32_t a0, a1, a2, b0, b1, b2;
    x6_split2<PROBE>(v01, a0, a1, a2);
    x6_split2<PROBE>(v23, b0, b1, b2);
    const int off = x6_off((KC ? PR : 4) * rq + j, 4 * kq);
    *reinterpret_cast<uint2*>(lds + off) = uint2{a0, b0};
    *reinterpret_cast<uint2*>(lds + kPlane + off) = uint2{a1, b1};
    *reinterpret_cast<uint2*>(lds + 2 * kPlane + off) = uint2{a2, b2};
  }

  // split the staged pieces and write the three planes (plane p at lds + p * kPlane)
  template <bool PROBE = false, bool EXACT = false>
  __device__ static void stash(unsigned char* lds, int t, const floatx4 (&r)[kPer][4]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i)
#pragma unroll
      for (int j = 0; j < PR; ++j) stash_row<PROBE, EXACT>(lds, t, r, i, j);  // row PR rq + j
  }
};

// The B operand as three bf16 planes already split (k-contiguous, ocppo_split_planes: the layer's
// weight, split once per minibatch instead of once per row tile and K step): staging is a copy of
// 16-B chunks (8 k of one row and plane) into the swizzled plane rows -- no split VALU, and one
// ds_write_b128 per chunk (8 lanes = one 128-B row pair: conflict-free).
template <int ROWS, int NT>
struct X6StagePl {
  static constexpr int kChunks = ROWS * 4 * 3;
  static constexpr int kPer = (kChunks + NT - 1) / NT;
  static constexpr int kPlane = ROWS * 64;

  __device__ static void at(int c, int& plane, int& row, int& ch) {
    plane = c / (ROWS * 4);
    const int rc = c - plane * (ROWS * 4);
    row = rc >> 2;
    ch = rc & 3;
  }
  __device__ static void load(const uint16_t* __restrict__ pl, int64_t ld, int64_t ps, int row0,
                              int k0, int t, u32x4 (&r)[kPer]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int c = t + NT * i;
      if (kChunks % NT != 0 && c >= kChunks) continue;
      int plane, row, ch;
      at(c, plane, row, ch);
      r[i] = *reinterpret_cast<const u32x4*>(pl + plane * ps + static_cast<int64_t>(row0 + row) * ld +
                                             k0 + 8 * ch);
    }
  }
  __device__ static void stash_chunk(unsigned char* lds, int t, const u32x4 (&r)[kPer], int i) {
    const int c = t + NT * i;
    if (kChunks % NT != 0 && c >= kChunks) return;
    int plane, row, ch;
    at(c, plane, row, ch);
    *reinterpret_cast<u32x4*>(lds + plane * kPlane + x6_chunk_off(row, ch)) = r[i];
  }
  __device__ static void stash(unsigned char* lds, int t, const u32x4 (&r)[kPer]) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) stash_chunk(lds, t, r, i);
  }
};

// Counted wait for inline-asm loads: vmcnt(N) (N newer loads may stay in flight), then every
// register of the consumed set is passed through an empty asm so no use of it can be scheduled
// before the wait.
template <int N, int P>
__device__ __forceinline__ void x6_vmwait(floatx4 (&r)[P][4]) {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0 || N == 4 || N == 8, "unsupported count");
#pragma unroll
  for (int i = 0; i < P; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(r[i][j]));
}

#if defined(OCPPO_X6_PROBE_NOSPLIT)
constexpr bool kProbeA = true, kProbeB = true;
#elif defined(OCPPO_X6_PROBE_NOSPLIT_B)
constexpr bool kProbeA = false, kProbeB = true;
#else
constexpr bool kProbeA = false, kProbeB = false;
#endif

__device__ __forceinline__ bf16x8 x6_frag(const unsigned char* plane, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(plane + x6_chunk_off(row, chunk));
}

// The six piece products of one (A block i, B block j) pair into acc (lead) / acs (small terms)
template <bool LO>
__device__ __forceinline__ void x6_mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4& acc,
                                         floatx4& acs) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  floatx4& s = LO ? acs : acc;
  s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], s, 0, 0, 0);
  s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], s, 0, 0, 0);
  s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], s, 0, 0, 0);
  s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], s, 0, 0, 0);
  s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], s, 0, 0, 0);
}

// One operand bf16-exact (its pieces 1 and 2 are zero: the u8 frame stacks of ocppo_conv_x6_u8):
// the three products with its lead piece, in x6_mfma6's order
template <bool AEX>
__device__ __forceinline__ void x6_mfma3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], floatx4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  if constexpr (AEX) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  }
}

// WGM x WGN waves per workgroup, each FM x FN blocks of 16 x 16 (tile BM x BN = 16 FM WGM x
// 16 FN WGN); LO: separate small-term accumulators (else all six products go into one); PF2: two
// register sets, loads issued two K steps ahead (else one).
#ifndef OCPPO_X6_OCC  // waves per SIMD the kernel is register-budgeted for (experiments)
#define OCPPO_X6_OCC 2
#endif
template <int FM, int FN, int WGM, int WGN, bool AKC, bool BKC>
constexpr int x6_lds_bytes() {
  return 3 * X6Stage<16 * FM * WGM, AKC, 64 * WGM * WGN>::kPlane +
         3 * X6Stage<16 * FN * WGN, BKC, 64 * WGM * WGN>::kPlane;
}

// XCD-aware bijective remap of workgroups [0, nb): workgroups b, b + 8, ... share an XCD; XCD x
// gets units [start(x), start(x) + count(x)) in order
__device__ __forceinline__ int x6_remap(int b, int nb) {
  const int xcd = b & 7, q = nb >> 3, rr = nb & 7;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
}

// rows of the gathered-B table per unit (mode 2: the unit's K range, K / splits)
constexpr int kX6GTbl = 1024;

// One output tile (unit u: split u / (tiles_m tiles_n), then row-major tiles) of the product
// GATH: 0 plain operands; 1 A's rows gathered (k-contiguous A, the unit's K range in one
// segment); 2 B's K index gathered (row-contiguous B, the tile's N range in one segment; gtbl =
// kX6GTbl ints of LDS)
// piece rows of the staged operands (4; 1 = row quads, k-contiguous operands only: experiments)
#ifndef OCPPO_X6P_PR_A
#define OCPPO_X6P_PR_A 4
#endif
#ifndef OCPPO_X6P_PR_B
#define OCPPO_X6P_PR_B 4
#endif
// PIPE: the double-buffered loop (x6p kernels: lds holds two stages)
template <int FM, int FN, int WGM, int WGN, bool AKC, bool BKC, bool LO, bool PF2, bool BPL = false,
          int GATH = 0, int WGE = 0, bool PIPE = false>
__device__ __forceinline__ void x6_unit(const X6Args& g, unsigned char* lds, int u, X6Place pl_,
                                        int32_t* gtbl = nullptr) {
  constexpr int NT = 64 * WGM * WGN;
  constexpr int BM = 16 * FM * WGM, BN = 16 * FN * WGN;
  // (row-quad pieces for the pipelined loop's k-contiguous operands, every thread the same
  // share, measured slower: 58's dX [4096 x 2048] 47.4 vs 44.7 us, profiles/r05/exp_x6_pipe.txt)
  using SA = X6Stage<BM, AKC, NT, (PIPE && AKC) ? OCPPO_X6P_PR_A : 4>;
  using SB = X6Stage<BN, BKC, NT, (PIPE && BKC) ? OCPPO_X6P_PR_B : 4>;
  unsigned char* la = lds;
  unsigned char* lb = lds + 3 * SA::kPlane;
  const int per_split = pl_.tiles_m * g.tiles_n;
  const bool seg = PIPE && pl_.seg_mode >= 0;
  const int s = seg ? 0 : u / per_split, rem = seg ? pl_.seg_tile : u - s * per_split;
  const int tm = rem / g.tiles_n, tn = rem - tm * g.tiles_n;
  const int m0 = pl_.row0_base + tm * BM, n0 = tn * BN;
  const float* __restrict__ A = g.a;
  const float* __restrict__ B = g.b;
  // split s reduces K steps [kb, kb + nk): an even partition of the K / 32 steps
  const int nall = g.K / kX6BK;
  const int kb = seg ? pl_.seg_kb : static_cast<int>(static_cast<int64_t>(s) * nall / g.splits);
  const int nk = seg ? pl_.seg_nk
                     : static_cast<int>(static_cast<int64_t>(s + 1) * nall / g.splits) - kb;

  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wm = wv / WGN, wn = wv % WGN;
  const int fr = lane & 15, fc = lane >> 4;
  const int64_t tile_id = pl_.id_base + static_cast<int64_t>(tm) * g.tiles_n + tn;
  // the mask epilogue's bitmask word, fetched before the K loop (off the epilogue's critical path)
  const uint64_t bits_in = g.mbits_in ? g.mbits_in[tile_id * NT + t] : 0;

  // operand loads of K step k0 into a register set (GATH: through the gathered row offsets)
  static_assert(GATH == 0 || (GATH == 1 && AKC) || (GATH == 2 && !BKC && !BPL) ||
                    (GATH == 3 && AKC) || (GATH == 4 && !BKC && !BPL) ||
                    (GATH == 5 && AKC && !BPL) || (GATH == 6 && !BKC && !BPL) ||
                    (GATH == 7 && AKC),
                "gather modes");
  constexpr bool kKRows = GATH == 4 || GATH == 6;  // B's K index walks convolution rows
  int64_t roffA[(GATH == 1 || GATH == 3 || GATH == 5 || GATH == 7) ? SA::kPer : 1][4];
  int qyA[GATH == 7 ? SA::kPer : 1][4], qxA[GATH == 7 ? SA::kPer : 1][4];
  int64_t nsegB[kKRows ? SB::kPer : 1];
  int cbB[kKRows ? SB::kPer : 1][4], cpB[kKRows ? SB::kPer : 1][4];
  int64_t cbaseB[GATH == 6 ? SB::kPer : 1][4];
  int64_t coffB = 0;
  if constexpr (GATH == 1) {
    const int seg = static_cast<int>((static_cast<int64_t>(kb) * kX6BK) / g.gseg);
    SA::gather_rows(g.gidx, g.gw, seg, g.gseg, g.sam, m0, t, roffA);
  } else if constexpr (GATH == 3) {
    SA::conv_rows(g, m0, t, roffA);
  } else if constexpr (GATH == 7) {
    SA::conv_rows_b(g, m0, t, roffA, qyA, qxA);
  } else if constexpr (GATH == 5) {
    SA::u8_rows(g, m0, t, roffA);
    for (int q = t; q < g.K / 4; q += NT) {
      const int k = 4 * q, c = k / g.u8_khw, rem = k - c * g.u8_khw, ky = rem / g.u8_kw;
      gtbl[q] = static_cast<int32_t>(c * g.u8_hw + ky * g.u8_w + (rem - ky * g.u8_kw));
    }
    __syncthreads();
  } else if constexpr (kKRows) {
    if constexpr (GATH == 4) SB::conv_cols(g, n0, t, nsegB);
    else SB::u8_cols(g, n0, t, nsegB);
    SB::conv_k_state(g, kb * kX6BK, t, cbB, cpB);
    if constexpr (GATH == 6) {
#pragma unroll
      for (int i = 0; i < SB::kPer; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          cbaseB[i][j] = x6_bnd(g, kBndU8Row,
                                g.u8_idx[x6_bnd(g, kBndImg, cbB[i][j], 1, g.u8_nimg)], 1,
                                g.bnd_u8rows) * g.u8_img;
    }
    for (int p = t; p < g.cv_qh * g.cv_qw; p += NT) {
      const int qy = p / g.cv_qw;
      gtbl[p] = static_cast<int32_t>(qy * g.cv_ys + (p - qy * g.cv_qw) * g.cv_xs);
    }
    __syncthreads();
  } else if constexpr (GATH == 2) {
    const int segn = static_cast<int>(n0 / g.gseg);
    coffB = -static_cast<int64_t>(segn) * g.gseg;
    for (int r = t; r < nk * kX6BK; r += NT)
      gtbl[r] = g.gidx[static_cast<int64_t>(kb * kX6BK + r) * g.gw + segn];
    __syncthreads();
  }
  // plain operands load through buffer resources (X6Stage::load_buf): config-2 GEMM set
  // 715 -> 682 us (profiles/r04/exp_x6_bufld); the pointer form stays for the inline-asm
  // experiment (OCPPO_X6_ASMLD)
#ifdef OCPPO_X6_ASMLD
  constexpr bool kBuf = false;
#else
  constexpr bool kBuf = GATH == 0;
#endif
  typename SA::Buf bufA;
  typename SB::Buf bufB;
  if constexpr (kBuf) {
    SA::buf_setup(A, g.sam, g.sak, m0, kb * kX6BK, t, bufA);
    SB::buf_setup(B, g.sbn, g.sbk, n0, kb * kX6BK, t, bufB);
  }
  auto loadA = [&](int k0, floatx4 (&r)[SA::kPer][4]) {
    if constexpr (GATH == 1) SA::load_rows(A, roffA, k0, t, r);
    else if constexpr (GATH == 3) SA::load_rows(A, roffA, static_cast<int>(x6_cv_seg(g, k0)), t, r, &g);
    else if constexpr (GATH == 5) SA::load_u8_rows(g.u8, roffA, gtbl, k0, t, r, g);
    else if constexpr (GATH == 7) SA::load_rows_bounded(A, g, roffA, qyA, qxA, k0, t, r);
    else if constexpr (kBuf)
      SA::load_buf(bufA, t, static_cast<int32_t>(4 * (AKC ? (k0 - kb * kX6BK)
                                                        : (k0 - kb * kX6BK) * g.sak)), r);
    else SA::load(A, g.sam, g.sak, m0, k0, t, r);
  };
  auto loadB = [&](int k0, floatx4 (&r)[SB::kPer][4]) {
    if constexpr (GATH == 2) SB::load_ktbl(B, g.sbk, gtbl, kb * kX6BK, coffB, n0, k0, t, r);
    else if constexpr (GATH == 4) SB::load_conv_k(B, g, nsegB, gtbl, cbB, cpB, t, r);  // k0: next
    else if constexpr (GATH == 6) SB::load_u8_k(g.u8, g, nsegB, gtbl, cbB, cpB, cbaseB, t, r);
    else if constexpr (kBuf)
      SB::load_buf(bufB, t, static_cast<int32_t>(4 * (BKC ? (k0 - kb * kX6BK)
                                                        : (k0 - kb * kX6BK) * g.sbk)), r);
    else SB::load(B, g.sbn, g.sbk, n0, k0, t, r);
  };

  floatx4 hi[FM][FN], lo[LO ? FM : 1][LO ? FN : 1];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) hi[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  if constexpr (LO) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) lo[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  // MFMAs of the step held in LDS (an exact operand: its lead plane only, three products)
  constexpr bool AEX = GATH == 5, BEX = GATH == 6;
  auto compute = [&]() {
    bf16x8 af[FM][3];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int pl = 0; pl < (AEX ? 1 : 3); ++pl)
        af[i][pl] = x6_frag(la + pl * SA::kPlane, wm * 16 * FM + 16 * i + fr, fc);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bf16x8 bf[3];
#pragma unroll
      for (int pl = 0; pl < (BEX ? 1 : 3); ++pl)
        bf[pl] = x6_frag(lb + pl * SB::kPlane, wn * 16 * FN + 16 * j + fr, fc);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (AEX || BEX) x6_mfma3<AEX>(af[i], bf, hi[i][j]);
        else x6_mfma6<LO>(af[i], bf, hi[i][j], lo[LO ? i : 0][LO ? j : 0]);
      }
    }
  };
  floatx4 ra[SA::kPer][4];
  if constexpr (PIPE) {
    // Two LDS stages, ONE barrier per K step, the fragment reads pipelined across it:
    //   * step kt's MFMAs for block columns [0, FN - 1) from stage kt % 2, each column followed
    //     by its share of the split + stash of step kt + 1 (raw tiles loaded during step kt - 1)
    //     into the other stage -- one basic block, so the split's VALU and LDS writes issue in
    //     the MFMAs' shadow instead of in a phase of their own between two barriers;
    //   * the barrier; then step kt + 2's loads (into the registers just stashed: one set,
    //     clamped to the last step, so no branch), and the LAST column's MFMAs of step kt, each
    //     A block's MFMAs followed by the read of that block's fragments of step kt + 1 from the
    //     stage just completed -- so the next step starts on fragments already in registers
    //     instead of every wave waiting on its reads behind the barrier.
    // The stash is unconditional (the last step rewrites a stage nobody reads again).
    // BPL: B arrives pre-split (X6StagePl: its stash is a 16-B copy per chunk, no VALU)
    static_assert(!LO && GATH == 0 && WGE == 0 && FN >= 2,
                  "pipelined loop: the plain family, >= 2 block columns per wave");
    using PB = X6StagePl<BN, NT>;
    constexpr int kStage = 3 * SA::kPlane + 3 * SB::kPlane;
    constexpr int kRowsA = SA::kPR * SA::kPer,
                  kRows = kRowsA + (BPL ? PB::kPer : SB::kPR * SB::kPer);
    floatx4 rb[BPL ? 1 : SB::kPer][4];
    u32x4 pb[BPL ? PB::kPer : 1];
    auto loadBB = [&](int k0) {
      if constexpr (BPL) PB::load(g.bpl, g.bpl_ld, g.bpl_ps, n0, k0, t, pb);
      else loadB(k0, rb);
    };
    // stash unit q of the step held in registers: A rows first, then B rows / plane chunks
    auto stash_unit = [&](unsigned char* st, int q) {
      if (q < kRowsA)
        SA::template stash_row<kProbeA>(st, t, ra, q / SA::kPR, q % SA::kPR);
      else if constexpr (BPL)
        PB::stash_chunk(st + 3 * SA::kPlane, t, pb, q - kRowsA);
      else
        SB::template stash_row<kProbeB>(st + 3 * SA::kPlane, t, rb, (q - kRowsA) / SB::kPR,
                                        (q - kRowsA) % SB::kPR);
    };
    constexpr int kSj = FN - 1;  // columns carrying the stash
    loadA(kb * kX6BK, ra);
    loadBB(kb * kX6BK);
#pragma unroll
    for (int q = 0; q < kRows; ++q) stash_unit(lds, q);
    loadA((kb + (nk > 1 ? 1 : 0)) * kX6BK, ra);
    loadBB((kb + (nk > 1 ? 1 : 0)) * kX6BK);
    __syncthreads();
    X6_STAMP(g, 1, static_cast<int64_t>(__builtin_readcyclecounter()));
    auto readA = [&](const unsigned char* st, int i, bf16x8 (&a)[3]) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[pl] = x6_frag(st + pl * SA::kPlane, wm * 16 * FM + 16 * i + fr, fc);
    };
    auto readB = [&](const unsigned char* st, int j, bf16x8 (&b)[3]) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[pl] = x6_frag(st + 3 * SA::kPlane + pl * SB::kPlane, wn * 16 * FN + 16 * j + fr, fc);
    };
    bf16x8 af[FM][3], bf0[3];
#pragma unroll
    for (int i = 0; i < FM; ++i) readA(lds, i, af[i]);
    readB(lds, 0, bf0);
    auto pstep = [&](int kt, const unsigned char* cur, unsigned char* nxt) {
#pragma unroll
      for (int j = 0; j < FN - 1; ++j) {
        bf16x8 bf[3];
        if (j == 0) {
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) bf[pl] = bf0[pl];
        } else {
          readB(cur, j, bf);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) x6_mfma6<false>(af[i], bf, hi[i][j], lo[0][0]);
#ifndef OCPPO_X6P_PROBE_NOSTASH  // probe builds only: the loop without its split and stash
#pragma unroll
        for (int q = j * kRows / kSj; q < (j + 1) * kRows / kSj; ++q) stash_unit(nxt, q);
#endif
      }
      bf16x8 bl[3];
      readB(cur, FN - 1, bl);
      __syncthreads();
#ifndef OCPPO_X6P_PROBE_NOLOAD
      const int kl = kt + 2 < nk ? kt + 2 : nk - 1;
      loadA((kb + kl) * kX6BK, ra);
      loadBB((kb + kl) * kX6BK);
#endif
      readB(nxt, 0, bf0);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        x6_mfma6<false>(af[i], bl, hi[i][FN - 1], lo[0][0]);
        readA(nxt, i, af[i]);
      }
    };
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      pstep(kt, lds, lds + kStage);
      pstep(kt + 1, lds + kStage, lds);
    }
    if (kt < nk) pstep(kt, lds, lds + kStage);
    X6_STAMP(g, 2, static_cast<int64_t>(__builtin_readcyclecounter()));
  } else if constexpr (BPL) {
    // A two K steps ahead (register sets ra / qa, as below), the pre-split B one step ahead:
    // its loads of step kt + 1 are issued before A's of step kt + 2, so the stash of step
    // kt + 1 waits for them without draining A's
    static_assert(PF2 && !LO, "the pre-split B path is built for the shipped family");
    using PB = X6StagePl<BN, NT>;
    const uint16_t* __restrict__ Bp = g.bpl;
    u32x4 pb[PB::kPer];
    floatx4 qa[SA::kPer][4];
    loadA(kb * kX6BK, ra);
    PB::load(Bp, g.bpl_ld, g.bpl_ps, n0, kb * kX6BK, t, pb);
    if (nk > 1) loadA((kb + 1) * kX6BK, qa);
    SA::template stash<kProbeA, AEX>(la, t, ra);
    PB::stash(lb, t, pb);
    __syncthreads();
    auto step = [&](int kt, floatx4 (&ldA)[SA::kPer][4], floatx4 (&stA)[SA::kPer][4],
                    u32x4 (&pbr)[PB::kPer]) {
      if (kt + 1 < nk) PB::load(Bp, g.bpl_ld, g.bpl_ps, n0, (kb + kt + 1) * kX6BK, t, pbr);
      if (kt + 2 < nk) loadA((kb + kt + 2) * kX6BK, ldA);
      compute();
      __syncthreads();
      if (kt + 1 < nk) {
        SA::template stash<kProbeA, AEX>(la, t, stA);
        PB::stash(lb, t, pbr);
      }
      __syncthreads();
    };
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      step(kt, ra, qa, pb);
      step(kt + 1, qa, ra, pb);
    }
    if (kt < nk) step(kt, ra, qa, pb);
  } else if constexpr (!PF2) {
    floatx4 rb[SB::kPer][4];
    SA::load(A, g.sam, g.sak, m0, kb * kX6BK, t, ra);
    SB::load(B, g.sbn, g.sbk, n0, kb * kX6BK, t, rb);
    SA::template stash<kProbeA, AEX>(la, t, ra);
    SB::template stash<kProbeB, BEX>(lb, t, rb);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) {
        SA::load(A, g.sam, g.sak, m0, (kb + kt + 1) * kX6BK, t, ra);
        SB::load(B, g.sbn, g.sbk, n0, (kb + kt + 1) * kX6BK, t, rb);
      }
      compute();
      __syncthreads();
      if (more) {
        SA::template stash<kProbeA, AEX>(la, t, ra);
        SB::template stash<kProbeB, BEX>(lb, t, rb);
      }
      __syncthreads();
    }
  } else {
    // set (ra, rb) holds even steps, (qa, qb) odd ones; at step kt the loads of step kt + 2 go
    // into the set step kt came from (already in LDS), then step kt + 1 is stashed
    // OCPPO_X6_ASMLD: the operand loads as inline asm with counted waits (the compiler's own
    // wait insertion loses the order of loads carried around the loop and drains the newer set
    // at every step); measured no faster (tools/exp_gemm_x6.py), so off by default
#ifdef OCPPO_X6_ASMLD
    constexpr bool ASM = SA::kUniform && SB::kUniform;
#else
    constexpr bool ASM = false;
#endif
    constexpr int kLoads = 4 * (SA::kPer + SB::kPer);  // loads per step per thread
    static_assert(!ASM || kLoads == 8, "x6_vmwait counts assume 8 loads per step");
    floatx4 rb[SB::kPer][4], qa[SA::kPer][4], qb[SB::kPer][4];
    if constexpr (GATH != 0 || kBuf) {
      loadA(kb * kX6BK, ra);
      loadB(kb * kX6BK, rb);
      if (nk > 1) {
        loadA((kb + 1) * kX6BK, qa);
        loadB((kb + 1) * kX6BK, qb);
      }
    } else {
      SA::template load<ASM>(A, g.sam, g.sak, m0, kb * kX6BK, t, ra);
      SB::template load<ASM>(B, g.sbn, g.sbk, n0, kb * kX6BK, t, rb);
      if (nk > 1) {
        SA::template load<ASM>(A, g.sam, g.sak, m0, (kb + 1) * kX6BK, t, qa);
        SB::template load<ASM>(B, g.sbn, g.sbk, n0, (kb + 1) * kX6BK, t, qb);
      }
    }
    if constexpr (ASM) {
      if (nk > 1) {
        x6_vmwait<8>(ra);
        x6_vmwait<8>(rb);
      } else {
        x6_vmwait<0>(ra);
        x6_vmwait<0>(rb);
      }
    }
    SA::template stash<kProbeA, AEX>(la, t, ra);
    SB::template stash<kProbeB, BEX>(lb, t, rb);
    __syncthreads();
    auto step = [&](int kt, floatx4 (&ldA)[SA::kPer][4], floatx4 (&ldB)[SB::kPer][4],
                    floatx4 (&stA)[SA::kPer][4], floatx4 (&stB)[SB::kPer][4]) {
      const bool issue = kt + 2 < nk;
      if (issue) {
        if constexpr (GATH != 0 || kBuf) {
          loadA((kb + kt + 2) * kX6BK, ldA);
          loadB((kb + kt + 2) * kX6BK, ldB);
        } else {
          SA::template load<ASM>(A, g.sam, g.sak, m0, (kb + kt + 2) * kX6BK, t, ldA);
          SB::template load<ASM>(B, g.sbn, g.sbk, n0, (kb + kt + 2) * kX6BK, t, ldB);
        }
      }
      compute();
      __syncthreads();
      if (kt + 1 < nk) {
        if constexpr (ASM) {  // step kt + 1's loads are older than the ones just issued
          if (issue) {
            x6_vmwait<8>(stA);
            x6_vmwait<8>(stB);
          } else {
            x6_vmwait<0>(stA);
            x6_vmwait<0>(stB);
          }
        }
        SA::template stash<kProbeA, AEX>(la, t, stA);
        SB::template stash<kProbeB, BEX>(lb, t, stB);
      }
      __syncthreads();
    };
    // both steps of a pair in one loop body with no branch between them (a conditional second
    // step let the compiler fold the pair into one step with register copies, which put a
    // vmcnt(0) before every step's loads: one step of prefetch, not two)
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      step(kt, ra, rb, qa, qb);
      step(kt + 1, qa, qb, ra, rb);
    }
    if (kt < nk) step(kt, ra, rb, qa, qb);
  }

  if constexpr (PIPE) {
    // stream-K: a later part of a split tile hands its accumulators over; the first part takes
    // them before its epilogue. Slots are [block (i, j)][thread] float4s (coalesced both ways);
    // the parts of one tile run on one XCD (x6p_streamk), whose L2 holds the slot: the data as
    // plain stores, drained (vmcnt) before the flag, which is written and polled at agent scope
    constexpr int kSlot = FM * FN * NT;  // float4 per slot
    if (seg && pl_.seg_mode == 1) {
      floatx4* ws = reinterpret_cast<floatx4*>(g.skws) + static_cast<int64_t>(pl_.seg_slot) * kSlot;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) ws[(i * FN + j) * NT + t] = hi[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) __hip_atomic_store(g.skflag + pl_.seg_slot, 1, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (seg && pl_.seg_mode == 2) {
      // the later parts of this tile are the first segments of the next ranks of this XCD (the
      // ones whose non-empty ranges start inside it)
      const X6pGeom G = x6p_geom(g, pl_.seg_slot, gridDim.x);
      const int64_t tl = rem - G.t0;
      for (int r = G.rank + 1; r < G.P; ++r) {
        const int64_t sr = static_cast<int64_t>(r) * G.I / G.P;
        if (sr >= (tl + 1) * G.nk) break;
        if (static_cast<int64_t>(r + 1) * G.I / G.P == sr) continue;  // an empty range
        const int slot = G.xcd + 8 * r;  // that rank's blockIdx
        if (t == 0) {  // bounded wait: a lost part ends in wrong numbers, never in a hang
          for (int it = 0; it < (1 << 22); ++it) {
            if (__hip_atomic_load(g.skflag + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
              break;
            __builtin_amdgcn_s_sleep(2);
          }
        }
        __syncthreads();
        const floatx4* ws = reinterpret_cast<const floatx4*>(g.skws) + static_cast<int64_t>(slot) * kSlot;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const floatx4 v = ws[(i * FN + j) * NT + t];
            hi[i][j] += v;
          }
        if (t == 0) __hip_atomic_store(g.skflag + slot, 0, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // epilogue: MFMA result C[4 fc + r][fr] of block (i, j)
#ifdef OCPPO_X6_ASMLD
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no inline-asm load left in flight
#endif
  float* __restrict__ Cp = g.c + s * g.split_c;
  const int wr0 = m0 + wm * 16 * FM, wc0 = n0 + wn * 16 * FN;
  if constexpr (WGE > 0) {
    // the layer below's backward (relu_bias_wgrad's arithmetic on this tile): gp = mask > 0 ?
    // acc : 0 is never stored; per column, db = sum_rows gp and dw[k] = sum_rows gp x[row, k],
    // rows of a lane in order, then the 4 lane row groups (xor 16, 32), then the wave rows in
    // order; one record slice per tile (record = row tile, columns n0 ..). WGE = K padded.
    constexpr int KP = WGE, XLD = KP + 1, NV = KP + 1;
    static_assert(WGM * BN * XLD * 4 <= x6_lds_bytes<FM, FN, WGM, WGN, AKC, BKC>() &&
                      BM * XLD * 4 <= x6_lds_bytes<FM, FN, WGM, WGN, AKC, BKC>(), "wgrad LDS");
    const int K1 = g.wk;
    float* xs = reinterpret_cast<float*>(lds);  // [BM][XLD], zero-padded to KP; the K loop
    for (int e = t; e < BM * KP; e += NT) {     // ended with a barrier
      const int r = e / KP, k = e - r * KP;
      xs[r * XLD + k] = k < K1 ? g.wx[static_cast<int64_t>(m0 + r) * g.ldwx + k] : 0.f;
    }
    __syncthreads();
    float acc[FN][NV];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[j][v] = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lrow = wm * 16 * FM + 16 * i + 4 * fc + r;
        const int64_t row = m0 + lrow;
        float xr[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) xr[k] = xs[lrow * XLD + k];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const float gp = g.mask[row * g.ldm + wc0 + 16 * j + fr] <= 0.f ? 0.f : hi[i][j][r];
          acc[j][0] += gp;
#pragma unroll
          for (int k = 0; k < KP; ++k) acc[j][1 + k] = fmaf(gp, xr[k], acc[j][1 + k]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        acc[j][v] += __shfl_xor(acc[j][v], 16, kWave);
        acc[j][v] += __shfl_xor(acc[j][v], 32, kWave);
      }
    __syncthreads();  // xs reads done: the LDS holds the wave-row partials next
    float* red = reinterpret_cast<float*>(lds);  // [WGM - 1][BN][XLD]
    if (wm > 0 && fc == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lc = wn * 16 * FN + 16 * j + fr;
#pragma unroll
        for (int v = 0; v < NV; ++v) red[((wm - 1) * BN + lc) * XLD + v] = acc[j][v];
      }
    }
    __syncthreads();
    if (wm == 0 && fc == 0) {
      float* rec = g.wrec + static_cast<int64_t>(tm) * g.wnpw;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lc = wn * 16 * FN + 16 * j + fr;
        const int col = n0 + lc;
        const int cgi = col / kWgRecCols;
        float* rc = rec + static_cast<int64_t>(cgi) * kWgRecCols * NV + (col - cgi * kWgRecCols);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          float sv = acc[j][v];
#pragma unroll
          for (int q = 0; q + 1 < WGM; ++q) sv += red[(q * BN + lc) * XLD + v];
          rc[static_cast<int64_t>(v) * kWgRecCols] = sv;
        }
      }
    }
    return;
  }
  // output row offsets: r ldc, or a convolution stride class's rows (GATH 3 / 7, cv_out)
  int64_t orow[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wr0 + 16 * i + 4 * fc + r;
      orow[i][r] = static_cast<int64_t>(row) * g.ldc;
      if constexpr (GATH == 3 || GATH == 7) {
        if (g.cv_out) {
          int b, qy, qx;
          x6_cv_split(g, row, b, qy, qx);
          orow[i][r] = b * g.co_sb + qy * g.co_ys + qx * g.co_xs + g.co_off;
        }
      }
    }
  // output column offset of column col (a stride class's channel under cv_out)
  auto ocol_of = [&](int col) -> int64_t {
    if constexpr (GATH == 3 || GATH == 7) {
      if (g.cv_out) {
        const int c = col / g.co_cw, py = c / g.co_cs;
        return py * g.co_cy + (c - py * g.co_cs) * g.co_cx + (col - c * g.co_cw);
      }
    }
    return col;
  };
  if (g.mask || g.mbits_in) {
    // threshold_backward(acc, mask, 0) and the tile's column sums: rows of a lane (i, r) in
    // order, then the wave's 4 row groups (xor 16, 32), then the two wave rows through LDS
    const uint64_t bits = bits_in;
    float colsum[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = wc0 + 16 * j + fr;
      const int64_t ocol = ocol_of(col);
      float cs = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = wr0 + 16 * i + 4 * fc + r;
          const float acc = LO ? hi[i][j][r] + lo[LO ? i : 0][LO ? j : 0][r] : hi[i][j][r];
          // the mask shares the output's layout under cv_out (the convolution data gradient)
          bool cvo = false;
          if constexpr (GATH == 3 || GATH == 7) cvo = g.cv_out != 0;
          const bool on = g.mbits_in ? ((bits >> ((i * FN + j) * 4 + r)) & 1) != 0
                                     : g.mask[cvo ? orow[i][r] + ocol : row * g.ldm + col] > 0.f;
          const float v = on ? acc : 0.f;
          Cp[orow[i][r] + ocol] = v;
          cs += v;
        }
      }
      cs += __shfl_xor(cs, 16, kWave);
      cs += __shfl_xor(cs, 32, kWave);
      colsum[j] = cs;
    }
    float* red = reinterpret_cast<float*>(lds);  // [WGM - 1][BN]; the K loop ended with a barrier
    if (wm > 0 && fc == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) red[(wm - 1) * BN + wn * 16 * FN + 16 * j + fr] = colsum[j];
    }
    __syncthreads();
    if (wm == 0 && fc == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int lc = wn * 16 * FN + 16 * j + fr;
        float v = colsum[j];
#pragma unroll
        for (int q = 0; q + 1 < WGM; ++q) v += red[q * BN + lc];  // wave rows in order
        const int64_t dr = pl_.db_base + static_cast<int64_t>(pl_.db_mult) * tm;
        g.dbp[dr * g.N + n0 + lc] = v;
        if (pl_.db_mult == 2) g.dbp[(dr + 1) * g.N + n0 + lc] = 0.f;
      }
    }
    return;
  }
  static_assert(FM * FN * 4 <= 64, "one 64-bit mask word per thread and tile");
  uint64_t bits = 0;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = wc0 + 16 * j + fr;
    const float bv = g.bias ? g.bias[col] : 0.f;
    const int64_t ocol = ocol_of(col);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = LO ? hi[i][j][r] + lo[LO ? i : 0][LO ? j : 0][r] : hi[i][j][r];
        if constexpr (GATH == 5) v = v / g.cdiv;
        if (g.bias) v += bv;
        if (g.relu) v = relu_f(v);
        Cp[orow[i][r] + ocol] = v;
        bits |= static_cast<uint64_t>(!(v <= 0.f)) << ((i * FN + j) * 4 + r);
      }
    }
  }
  if (!g.mbits_out) return;
  if (!g.mbits_rows) {
    g.mbits_out[tile_id * NT + t] = bits;
    return;
  }
  if constexpr (FN % 2 == 0) {
    // row-major words: the ballot of fragment (i, j, r) holds, for lane group fc, the 16 columns
    // 16 j + [0, 16) of row 16 i + 4 fc + r; word (row, p) = columns 32 p + [0, 32) of the wave's
    // 16 FM rows x 16 FN columns, assembled by the lane that stores it
    constexpr int WPR = FN / 2, WORDS = 16 * FM * WPR;
    uint32_t* rows = reinterpret_cast<uint32_t*>(g.mbits_out);
    const int64_t ldw = g.N / 32;
#pragma unroll
    for (int q = 0; q < (WORDS + 63) / 64; ++q) {
      const int w = lane + 64 * q;
      const int wrow = w / WPR, p = w - wrow * WPR;
      const int li = wrow >> 4, lfc = (wrow >> 2) & 3, lr = wrow & 3;
      uint32_t word = 0;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint64_t bal = __ballot((bits >> ((i * FN + j) * 4 + r)) & 1);
            const uint32_t half = static_cast<uint32_t>(bal >> (16 * lfc)) & 0xffffu;
            if (li == i && lr == r && p == (j >> 1)) word |= half << (16 * (j & 1));
          }
        }
      }
      if (w < WORDS) rows[(wr0 + wrow) * ldw + (wc0 >> 5) + p] = word;
    }
  }
}

template <int FM, int FN, int WGM, int WGN, bool AKC, bool BKC, bool LO, bool PF2, bool BPL = false,
          int GATH = 0, int WGE = 0>
__global__ __launch_bounds__(64 * WGM * WGN, OCPPO_X6_OCC) void gemm_x6_kernel(X6Args g) {
  __shared__ __attribute__((aligned(16)))
  unsigned char lds[x6_lds_bytes<FM, FN, WGM, WGN, AKC, BKC>()];
  __shared__ int32_t gtbl[(GATH == 2 || GATH >= 4) ? kX6GTbl : 1];
  const int u = x6_remap(blockIdx.x, gridDim.x);
  if (u >= g.units) return;
  x6_unit<FM, FN, WGM, WGN, AKC, BKC, LO, PF2, BPL, GATH, WGE>(
      g, lds, u, X6Place{g.tiles_m, 0, 0, 1, 0}, gtbl);
}

// The pipelined family (variants 57-60, x6_unit PIPE): two LDS stages per workgroup, so one
// workgroup per CU (the 8-wave forms: two waves per SIMD, 256 registers each; the 4-wave form:
// one wave per SIMD, 512 registers)
template <int FM, int FN, int WGM, int WGN, bool AKC, bool BKC, int OCC, bool BPL = false,
          bool SK = false>
__global__ __launch_bounds__(64 * WGM * WGN, OCC) void gemm_x6p_kernel(X6Args g) {
  __shared__ __attribute__((aligned(16)))
  unsigned char lds[2 * x6_lds_bytes<FM, FN, WGM, WGN, AKC, BKC>()];
  X6_STAMP(g, 0, static_cast<int64_t>(__builtin_readcyclecounter()));
  X6_STAMP(g, 4, static_cast<int64_t>(__builtin_amdgcn_s_memrealtime()));
  if constexpr (SK) {
    // stream-K: this workgroup's range of its XCD's K steps, tile segment by tile segment
    const X6pGeom G = x6p_geom(g, blockIdx.x, gridDim.x);
    int64_t s = static_cast<int64_t>(G.rank) * G.I / G.P;
    const int64_t e = static_cast<int64_t>(G.rank + 1) * G.I / G.P;
    while (s < e) {
      const int tl = static_cast<int>(s / G.nk), k0 = static_cast<int>(s - static_cast<int64_t>(tl) * G.nk);
      const int k1 = static_cast<int>(e - s < G.nk - k0 ? k0 + (e - s) : G.nk);
      X6Place pl{g.tiles_m, 0, 0, 1, 0};
      pl.seg_mode = k0 > 0 ? 1 : (k1 < G.nk ? 2 : 0);
      pl.seg_tile = G.t0 + tl;
      pl.seg_kb = k0;
      pl.seg_nk = k1 - k0;
      pl.seg_slot = blockIdx.x;
      x6_unit<FM, FN, WGM, WGN, AKC, BKC, false, true, BPL, 0, 0, true>(g, lds, 0, pl);
      s += k1 - k0;
      __syncthreads();  // the next segment's prologue rewrites the LDS stages
    }
  } else {
    const int u = x6_remap(blockIdx.x, gridDim.x);
    if (u >= g.units) return;
    x6_unit<FM, FN, WGM, WGN, AKC, BKC, false, true, BPL, 0, 0, true>(
        g, lds, u, X6Place{g.tiles_m, 0, 0, 1, 0});
  }
#ifdef OCPPO_X6_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  X6_STAMP(g, 3, static_cast<int64_t>(__builtin_readcyclecounter()));
  X6_STAMP(g, 5, static_cast<int64_t>(__builtin_amdgcn_s_memrealtime()));
#endif
}

template <int FM, int FN, int WGM, int WGN, int OCC>
static void launch_x6p_t(hipStream_t s, bool akc, bool bkc, X6Args& g) {
  g.tiles_m = g.M / (16 * FM * WGM);
  g.tiles_n = g.N / (16 * FN * WGN);
  const dim3 grid(g.units), block(64 * WGM * WGN);
  if constexpr (OCC == 2 && FM == 4) {  // 57, 58: the stream-K forms
    if (g.sk) {
      if (g.bpl)
        hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, true, true, OCC, true, true>), grid,
                           block, 0, s, g);
      else if (akc && bkc)
        hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, true, true, OCC, false, true>),
                           grid, block, 0, s, g);
      else if (akc)
        hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, true, false, OCC, false, true>),
                           grid, block, 0, s, g);
      else if (bkc)
        hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, false, true, OCC, false, true>),
                           grid, block, 0, s, g);
      else
        hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, false, false, OCC, false, true>),
                           grid, block, 0, s, g);
      return;
    }
  }
  if (g.bpl)  // pre-split B (the caller checked akc)
    hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, true, true, OCC, true>), grid, block, 0,
                       s, g);
  else if (akc && bkc)
    hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, true, true, OCC>), grid, block, 0, s, g);
  else if (akc)
    hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, true, false, OCC>), grid, block, 0, s, g);
  else if (bkc)
    hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, false, true, OCC>), grid, block, 0, s, g);
  else
    hipLaunchKernelGGL((gemm_x6p_kernel<FM, FN, WGM, WGN, false, false, OCC>), grid, block, 0, s, g);
}

// Mixed tiles: workgroups [0, nbig) take the 128 x 128 tiles of rows [0, mbig) (dispatched
// first, the longest units), the rest the 64 x 128 tiles of rows [mbig, M) as slots free up;
// each range keeps its own XCD remap (nbig is a multiple of 8, so XCD b & 7 is the same in both)
template <bool AKC, bool BKC, bool BPL = false>
__global__ __launch_bounds__(256, OCPPO_X6_OCC) void gemm_x6_mixed_kernel(X6Args g) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[x6_lds_bytes<4, 4, 2, 2, AKC, BKC>()];
  const int nbig = (g.mbig / 128) * g.tiles_n;
  const int b = blockIdx.x;
  if (b < nbig) {
    x6_unit<4, 4, 2, 2, AKC, BKC, false, true, BPL>(g, lds, x6_remap(b, nbig),
                                                    X6Place{g.mbig / 128, 0, 0, 2, 0});
  } else {
    const int small = (g.M - g.mbig) / 64;
    const int u = x6_remap(b - nbig, gridDim.x - nbig);
    if (u >= small * g.tiles_n) return;
    x6_unit<2, 4, 2, 2, AKC, BKC, false, true, BPL>(
        g, lds, u, X6Place{small, g.mbig, g.mbig / 64, 1, static_cast<int64_t>(nbig)});
  }
}

template <bool AKC, bool BKC>
static void launch_x6_mixed1(hipStream_t s, X6Args& g) {
  if (g.bpl)
    hipLaunchKernelGGL((gemm_x6_mixed_kernel<true, true, true>), dim3(g.units), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_x6_mixed_kernel<AKC, BKC>), dim3(g.units), dim3(256), 0, s, g);
}

// Rows in 128-row tiles for an [M x N] mixed product. With 256 < T <= 384 tiles of 128 x 128
// (T / 256 CUs: some CUs run two, the rest one), 256 of them — one per CU — and the rest as
// 2 (T - 256) tiles of 64 x 128 that fill the second slot of every CU: one wave of <= 512
// workgroups with no CU holding two big tiles (tools/exp_gemm_x6.py --mbig: [11520 x 512] from
// K = 1024 80.4 -> 70.3 us); otherwise every row in 128-row tiles (at 720 tiles no split beat it).
// The caller may pass its own split (the mbig argument, >= 0: experiments and tests).
static int x6_mixed_mbig(int M, int N) {
  const int tn = N / 128, tiles = (M / 128) * tn;
  if (tiles > 256 && tiles <= 384 && 256 % tn == 0) return (256 / tn) * 128;
  return (M / 128) * 128 == M && tiles % 8 == 0 ? M : 0;
}

template <int FM, int FN, int WGM, int WGN, bool LO, bool PF2>
static void launch_x6_t(hipStream_t s, bool akc, bool bkc, X6Args& g) {
  g.tiles_m = g.M / (16 * FM * WGM);
  g.tiles_n = g.N / (16 * FN * WGN);
  const dim3 grid(g.units), block(64 * WGM * WGN);
  if constexpr (PF2 && !LO && WGM * WGN == 4) {
    if (g.bpl) {  // pre-split B (the caller checked akc)
      hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, true, true, false, true, true>), grid,
                         block, 0, s, g);
      return;
    }
  }
  if (akc && bkc)
    hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, true, true, LO, PF2>), grid, block, 0, s, g);
  else if (akc)
    hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, true, false, LO, PF2>), grid, block, 0, s, g);
  else if (bkc)
    hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, false, true, LO, PF2>), grid, block, 0, s, g);
  else
    hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, false, false, LO, PF2>), grid, block, 0, s, g);
}

// Tile configs (FM, FN, WGM, WGN): tile = 16 FM WGM rows x 16 FN WGN columns
struct X6Tile {
  int fm, fn, wgm, wgn;
};
constexpr X6Tile kX6Tiles[] = {{4, 4, 2, 2}, {2, 4, 2, 2}, {4, 2, 2, 2}, {2, 2, 2, 2},
                               {4, 2, 2, 4}, {2, 2, 2, 4}, {2, 4, 4, 2}, {2, 2, 4, 2}};
// the pipelined family, variants 57-60: 256 x 128 and 128 x 256 (8 waves), 128 x 128 (4 waves,
// one per SIMD), 128 x 128 (8 waves)
constexpr X6Tile kX6PTiles[] = {{4, 4, 4, 2}, {4, 4, 2, 4}, {4, 4, 2, 2}, {2, 4, 4, 2}};

// variant: shape (bits 0-2) | PF2 (bit 3) | one accumulator (bit 4); instantiated: every shape
// with PF2 + one accumulator (the product family), shapes 0-3 with one-step loads (+/- LO)
static bool launch_x6(hipStream_t s, int tile, bool akc, bool bkc, X6Args& g) {
  const int shape = tile & 7;
  switch (tile) {  // the pipelined family
    case 57: launch_x6p_t<4, 4, 4, 2, 2>(s, akc, bkc, g); return true;
    case 58: launch_x6p_t<4, 4, 2, 4, 2>(s, akc, bkc, g); return true;
    case 59: launch_x6p_t<4, 4, 2, 2, 1>(s, akc, bkc, g); return true;
    case 60: launch_x6p_t<2, 4, 4, 2, 2>(s, akc, bkc, g); return true;
    default: break;
  }
  if (tile & 32) {  // mixed 128 x 128 / 64 x 128 tiles (variant 56 only)
    if (tile != 56) return false;
    g.tiles_n = g.N / 128;
    g.tiles_m = 0;
    const int nbig = (g.mbig / 128) * g.tiles_n;
    g.units = nbig + ((g.M - g.mbig) / 64) * g.tiles_n;
    if (akc && bkc) launch_x6_mixed1<true, true>(s, g);
    else if (akc) launch_x6_mixed1<true, false>(s, g);
    else if (bkc) launch_x6_mixed1<false, true>(s, g);
    else launch_x6_mixed1<false, false>(s, g);
    return true;
  }
  const bool pf2 = tile & 8, one = tile & 16;
  if (pf2 && one) {
    switch (shape) {
      case 0: launch_x6_t<4, 4, 2, 2, false, true>(s, akc, bkc, g); return true;
      case 1: launch_x6_t<2, 4, 2, 2, false, true>(s, akc, bkc, g); return true;
      case 2: launch_x6_t<4, 2, 2, 2, false, true>(s, akc, bkc, g); return true;
      case 3: launch_x6_t<2, 2, 2, 2, false, true>(s, akc, bkc, g); return true;
      case 4: launch_x6_t<4, 2, 2, 4, false, true>(s, akc, bkc, g); return true;
      case 5: launch_x6_t<2, 2, 2, 4, false, true>(s, akc, bkc, g); return true;
      case 6: launch_x6_t<2, 4, 4, 2, false, true>(s, akc, bkc, g); return true;
      default: launch_x6_t<2, 2, 4, 2, false, true>(s, akc, bkc, g); return true;
    }
  }
  if (pf2 || shape > 3) return false;
  switch (shape + (one ? 4 : 0)) {
    case 0: launch_x6_t<4, 4, 2, 2, true, false>(s, akc, bkc, g); return true;
    case 1: launch_x6_t<2, 4, 2, 2, true, false>(s, akc, bkc, g); return true;
    case 2: launch_x6_t<4, 2, 2, 2, true, false>(s, akc, bkc, g); return true;
    case 3: launch_x6_t<2, 2, 2, 2, true, false>(s, akc, bkc, g); return true;
    case 4: launch_x6_t<4, 4, 2, 2, false, false>(s, akc, bkc, g); return true;
    case 5: launch_x6_t<2, 4, 2, 2, false, false>(s, akc, bkc, g); return true;
    case 6: launch_x6_t<4, 2, 2, 2, false, false>(s, akc, bkc, g); return true;
    default: launch_x6_t<2, 2, 2, 2, false, false>(s, akc, bkc, g); return true;
  }
}

// gathered products on the 128 x 128 tile (variant 24): mode 1 (forward, k-contiguous A and B or
// B pre-split), mode 2 (weight gradient, m-contiguous A, n-contiguous gathered B)
static void launch_x6_gather(hipStream_t s, int mode, X6Args& g) {
  g.tiles_m = g.M / 128;
  g.tiles_n = g.N / 128;
  const dim3 grid(g.units), block(256);
  if (mode == 1 && g.bpl)
    hipLaunchKernelGGL((gemm_x6_kernel<4, 4, 2, 2, true, true, false, true, true, 1>), grid, block,
                       0, s, g);
  else if (mode == 1)
    hipLaunchKernelGGL((gemm_x6_kernel<4, 4, 2, 2, true, true, false, true, false, 1>), grid, block,
                       0, s, g);
  else
    hipLaunchKernelGGL((gemm_x6_kernel<4, 4, 2, 2, false, false, false, true, false, 2>), grid,
                       block, 0, s, g);
}

// ---------------------------------------------------------------------------------------------
// ocppo_split_planes: an f32 matrix (or its transpose) as the three bf16 planes gemm_x6 stages
// as its B operand (x6_split2: bitwise the pieces the kernel would form itself). Up to
// kSplitJobs matrices per launch, each cut into 64 x 64 tiles read as rows of 256 B and written
// (transposed through LDS when asked) as bf16 pairs.
constexpr int kSplitJobs = 8;
struct SplitJob {
  const float* src;
  int64_t ld;
  int R, C, trans, tiles_c, tile0;
  uint16_t* dst;
};
struct SplitJobs {
  SplitJob j[kSplitJobs];
  int n;
};

__global__ __launch_bounds__(256) void split_planes_kernel(SplitJobs J) {
  const int b = blockIdx.x;
  int ji = 0;
  while (ji + 1 < J.n && b >= J.j[ji + 1].tile0) ++ji;
  const SplitJob jb = J.j[ji];
  const int tl = b - jb.tile0, tr = tl / jb.tiles_c, tc = tl - tr * jb.tiles_c;
  const int r0 = 64 * tr, c0 = 64 * tc;
  __shared__ float tile[64][65];
  if ((jb.C & 3) == 0 && (jb.ld & 3) == 0 && (reinterpret_cast<uintptr_t>(jb.src) & 15) == 0) {
    // 16-B loads: 4 per thread, all issued before the LDS stores
    float4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + 256 * i, r = e >> 4, c = 4 * (e & 15);
      v[i] = r0 + r < jb.R && c0 + c < jb.C
                 ? *reinterpret_cast<const float4*>(jb.src + static_cast<int64_t>(r0 + r) * jb.ld + c0 + c)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + 256 * i, r = e >> 4, c = 4 * (e & 15);
      tile[r][c] = v[i].x;
      tile[r][c + 1] = v[i].y;
      tile[r][c + 2] = v[i].z;
      tile[r][c + 3] = v[i].w;
    }
  } else {
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int r = e >> 6, c = e & 63;
      tile[r][c] = r0 + r < jb.R && c0 + c < jb.C
                       ? jb.src[static_cast<int64_t>(r0 + r) * jb.ld + c0 + c] : 0.f;
    }
  }
  __syncthreads();
  const int oR = jb.trans ? jb.C : jb.R, oC = jb.trans ? jb.R : jb.C;
  const int64_t ps = static_cast<int64_t>(oR) * oC;
  for (int e = threadIdx.x; e < 64 * 16; e += 256) {  // 4 output elements (8 B per plane) each
    const int orow = e >> 4, oq = e & 15;
    x6f2 v01, v23;
    if (jb.trans) {
      v01 = x6f2{tile[4 * oq][orow], tile[4 * oq + 1][orow]};
      v23 = x6f2{tile[4 * oq + 2][orow], tile[4 * oq + 3][orow]};
    } else {
      v01 = x6f2{tile[orow][4 * oq], tile[orow][4 * oq + 1]};
      v23 = x6f2{tile[orow][4 * oq + 2], tile[orow][4 * oq + 3]};
    }
    const int gr = (jb.trans ? c0 : r0) + orow, gc = (jb.trans ? r0 : c0) + 4 * oq;
    if (gr >= oR || gc >= oC) continue;  // oC % 8 == 0: a quad is inside or outside whole
    uint32_t a0, a1, a2, b0, b1, b2;
    x6_split2(v01, a0, a1, a2);
    x6_split2(v23, b0, b1, b2);
    uint2* d = reinterpret_cast<uint2*>(jb.dst + static_cast<int64_t>(gr) * oC + gc);
    d[0] = uint2{a0, b0};
    d[ps / 4] = uint2{a1, b1};
    d[ps / 2] = uint2{a2, b2};
  }
}

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_split_planes(ocppo_stream_t stream, int n, const float* const* src,
                                  const int64_t* ld, const int64_t* rows, const int64_t* cols,
                                  const int* trans, void* const* dst) {
  OCPPO_REQUIRE(n >= 1 && n <= kSplitJobs && src && ld && rows && cols && trans && dst,
                "ocppo_split_planes: n=%d jobs (1..%d) and every array", n, kSplitJobs);
  SplitJobs J{};
  J.n = n;
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    OCPPO_REQUIRE(src[i] && dst[i] && rows[i] >= 1 && cols[i] >= 1 && ld[i] >= cols[i] &&
                      rows[i] <= 65536 && cols[i] <= 65536 &&
                      (trans[i] ? rows[i] : cols[i]) % 8 == 0 &&
                      reinterpret_cast<uintptr_t>(dst[i]) % 16 == 0,
                  "ocppo_split_planes: job %d (%lld x %lld, ld %lld, trans %d): the planes' rows "
                  "must be multiples of 8 elements, 16-B aligned", i, (long long)rows[i],
                  (long long)cols[i], (long long)ld[i], trans[i]);
    const int tc = static_cast<int>((cols[i] + 63) / 64), tr = static_cast<int>((rows[i] + 63) / 64);
    J.j[i] = SplitJob{src[i], ld[i], static_cast<int>(rows[i]), static_cast<int>(cols[i]),
                      trans[i] ? 1 : 0, tc, tiles, static_cast<uint16_t*>(dst[i])};
    tiles += tc * tr;
  }
  clear_stale_error();
  hipLaunchKernelGGL(split_planes_kernel, dim3(tiles), dim3(256), 0, as_stream(stream), J);
  return check_launch("ocppo_split_planes");
}

#ifdef OCPPO_X6_BOUNDS
static uint32_t* g_x6_bnd = nullptr;
static int64_t g_x6_bnd_x = 0, g_x6_bnd_u8 = 0, g_x6_bnd_u8rows = 0;
// bounds-check builds only: the violation record (>= 6 uint32, device) and the extents of the
// next convolution launch's gathered sources, from the pointers it is passed (x elements; u8
// bytes and stack rows)
extern "C" __attribute__((visibility("default"))) int ocppo_x6_probe_set_bounds(
    uint32_t* rec, int64_t x_elems, int64_t u8_bytes, int64_t u8_rows) {
  g_x6_bnd = rec;
  g_x6_bnd_x = x_elems;
  g_x6_bnd_u8 = u8_bytes;
  g_x6_bnd_u8rows = u8_rows;
  return OCPPO_OK;
}
static void x6_bounds_args(X6Args& g) {
  g.bnd = g_x6_bnd;
  g.bnd_x = g_x6_bnd_x;
  g.bnd_u8 = g_x6_bnd_u8;
  g.bnd_u8rows = g_x6_bnd_u8rows;
}
static void img_bounds_args(uint32_t*& bnd, int64_t& rows) {
  bnd = g_x6_bnd;
  rows = g_x6_bnd_u8rows;
}
#else
static void x6_bounds_args(X6Args&) {}
static void img_bounds_args(uint32_t*&, int64_t&) {}
#endif

#ifdef OCPPO_X6_STAMPS
static int64_t* g_x6_stamps = nullptr;
// probe builds only: the stamps buffer (>= 8 int64 per workgroup) of the following launches
extern "C" __attribute__((visibility("default"))) int ocppo_x6_probe_set_stamps(int64_t* p) {
  g_x6_stamps = p;
  return OCPPO_OK;
}
#endif

// A unit's operand window (<= 256 rows x its K range, either layout) addressed by the 32-bit
// buffer offsets of X6Stage::load_buf
static bool x6_windows_ok(int64_t sam, int64_t sak, int64_t sbn, int64_t sbk, int64_t K,
                          int64_t splits, bool b_planes) {
  const int64_t ks = ((K / kX6BK + splits - 1) / splits + 1) * kX6BK;
  auto win = [&](int64_t srow, int64_t sk) { return 4 * (256 * srow + ks * sk + 256); };
  return win(sam, sak) < INT32_MAX && (b_planes || win(sbn, sbk) < INT32_MAX);
}

// Stream-K launches of the pipelined tiles: one workgroup per CU (a multiple of 8: every XCD's
// share equal), workspace = a partial-accumulator slot + an int flag per workgroup
static int x6p_sk_grid() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8)
      n = 256;
    cus = n / 8 * 8;
  }
  return cus;
}
static int64_t x6p_slot_bytes(int tile) {
  const X6Tile tc = kX6PTiles[tile - 57];
  return static_cast<int64_t>(tc.fm) * tc.fn * 64 * tc.wgm * tc.wgn * 16;
}

extern "C" size_t ocppo_gemm_x6_sk_workspace_bytes(int tile) {
  if (tile != 57 && tile != 58) return 0;
  const int grid = x6p_sk_grid();
  return static_cast<size_t>(grid) * x6p_slot_bytes(tile) + static_cast<size_t>(grid) * 4;
}

extern "C" int ocppo_gemm_x6(ocppo_stream_t stream, const float* a, int64_t sam, int64_t sak,
                             const float* b, int64_t sbn, int64_t sbk, float* c, int64_t ldc,
                             int64_t M, int64_t N, int64_t K, int64_t splits, int64_t split_c,
                             const float* bias, int relu,
                             const float* mask, int64_t ldm, float* dbp, uint64_t* mbits_out,
                             const uint64_t* mbits_in, int tile, int mbig,
                             const void* b_planes, int64_t bp_ld, int64_t bp_stride,
                             void* sk_workspace, size_t sk_workspace_bytes) {
  OCPPO_REQUIRE(M >= 1 && N >= 1 && K >= 1 && splits >= 1 && M <= INT32_MAX && N <= INT32_MAX &&
                    K <= INT32_MAX,
                "ocppo_gemm_x6: bad sizes M=%lld N=%lld K=%lld splits=%lld", (long long)M,
                (long long)N, (long long)K, (long long)splits);
  OCPPO_REQUIRE(a && (b || b_planes) && c, "ocppo_gemm_x6: null pointer");
  OCPPO_REQUIRE((sak == 1 && sam >= K && sam % 4 == 0) || (sam == 1 && sak >= M && sak % 4 == 0),
                "ocppo_gemm_x6: A strides (%lld, %lld): one must be 1, the other a multiple of 4",
                (long long)sam, (long long)sak);
  OCPPO_REQUIRE(b_planes != nullptr ||
                    (sbk == 1 && sbn >= K && sbn % 4 == 0) || (sbn == 1 && sbk >= N && sbk % 4 == 0),
                "ocppo_gemm_x6: B strides (%lld, %lld): one must be 1, the other a multiple of 4",
                (long long)sbn, (long long)sbk);
  OCPPO_REQUIRE(b_planes == nullptr ||
                    (sak == 1 && bp_ld >= K && bp_ld % 8 == 0 && bp_stride >= bp_ld * N &&
                     bp_stride % 8 == 0 && reinterpret_cast<uintptr_t>(b_planes) % 16 == 0 &&
                     ((tile >= 24 && tile < 28) || tile == 56 || tile == 57 || tile == 58)),
                "ocppo_gemm_x6: pre-split B needs a k-contiguous A, 16-B aligned k-contiguous "
                "planes (ld %lld, stride %lld) and a tile of 24..27, 56, 57 or 58",
                (long long)bp_ld,
                (long long)bp_stride);
  OCPPO_REQUIRE(ldc >= N, "ocppo_gemm_x6: ldc=%lld < N", (long long)ldc);
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(a) % 16 == 0 && reinterpret_cast<uintptr_t>(b) % 16 == 0,
                "ocppo_gemm_x6: A and B must be 16-B aligned");
  OCPPO_REQUIRE(x6_windows_ok(sam, sak, sbn, sbk, K, splits, b_planes != nullptr),
                "ocppo_gemm_x6: an operand window of one tile exceeds 2 GiB (32-bit buffer "
                "offsets): split the product");
  if (b_planes) b = nullptr;
  OCPPO_REQUIRE(K % kX6BK == 0 && K / kX6BK >= splits,
                "ocppo_gemm_x6: K=%lld must be a multiple of %d with >= 1 step per split",
                (long long)K, kX6BK);
  OCPPO_REQUIRE(tile >= 0 && tile < 64, "ocppo_gemm_x6: tile=%d", tile);
  const bool pipe = tile >= 57 && tile <= 60;
  OCPPO_REQUIRE(tile != 56 || splits == 1, "ocppo_gemm_x6: mixed tiles need splits == 1");
  OCPPO_REQUIRE(!(tile & 32) || tile == 56 || pipe, "ocppo_gemm_x6: tile=%d not built", tile);
  OCPPO_REQUIRE(mbig == -1 || (tile == 56 && mbig >= 0),
                "ocppo_gemm_x6: mbig=%d (-1, or a split of the mixed tile)", mbig);
  const X6Tile tc = tile >= 57 && tile <= 60 ? kX6PTiles[tile - 57]
                    : kX6Tiles[(tile & 32) ? 1 : (tile & 7)];  // mixed: divisibility of 64 x 128
  const int64_t bm = 16 * tc.fm * tc.wgm, bn = 16 * tc.fn * tc.wgn;
  OCPPO_REQUIRE(M % bm == 0 && N % bn == 0,
                "ocppo_gemm_x6: M=%lld, N=%lld must be multiples of the %lld x %lld tile",
                (long long)M, (long long)N, (long long)bm, (long long)bn);
  OCPPO_REQUIRE(splits == 1 || (bias == nullptr && !relu),
                "ocppo_gemm_x6: bias / ReLU epilogues need splits == 1");
  OCPPO_REQUIRE((mask == nullptr && mbits_in == nullptr) ||
                    (splits == 1 && bias == nullptr && !relu && dbp &&
                     (mbits_in != nullptr || ldm >= N)),
                "ocppo_gemm_x6: the mask epilogue needs splits == 1, no bias / ReLU, dbp, ldm >= N");
  OCPPO_REQUIRE(mbits_out == nullptr || (splits == 1 && mask == nullptr && mbits_in == nullptr),
                "ocppo_gemm_x6: mbits_out needs splits == 1 and no mask epilogue");
  const int64_t units = splits * (M / bm) * (N / bn);
  OCPPO_REQUIRE(units <= INT32_MAX / 2, "ocppo_gemm_x6: too large");
  OCPPO_REQUIRE(!(relu & OCPPO_X6_MBITS_ROWS) || ((relu & 1) && mbits_out != nullptr),
                "ocppo_gemm_x6: the row-major bitmask needs the ReLU epilogue and mbits_out");
  X6Args g{a, sam, sak, b, sbn, sbk, c, ldc, bias, relu & 1, (int)M, (int)N, (int)K,
           0, 0, (int)units, (int)splits, split_c, mask, ldm, dbp, mbits_out, mbits_in, 0,
           static_cast<const uint16_t*>(b_planes), bp_ld, bp_stride};
  g.mbits_rows = (relu & OCPPO_X6_MBITS_ROWS) ? 1 : 0;
#ifdef OCPPO_X6_STAMPS
  g.stamps = g_x6_stamps;
#endif
  if (sk_workspace) {
    OCPPO_REQUIRE((tile == 57 || tile == 58) && splits == 1 &&
                      sk_workspace_bytes >= ocppo_gemm_x6_sk_workspace_bytes(tile) &&
                      reinterpret_cast<uintptr_t>(sk_workspace) % 256 == 0,
                  "ocppo_gemm_x6: stream-K needs tile 57 or 58, splits == 1 and a 256-B aligned "
                  "workspace of ocppo_gemm_x6_sk_workspace_bytes (%zu given)", sk_workspace_bytes);
    const int grid = x6p_sk_grid();
    const X6Tile tc = kX6PTiles[tile - 57];
    const int64_t T = (M / (16 * tc.fm * tc.wgm)) * (N / (16 * tc.fn * tc.wgn));
    OCPPO_REQUIRE(T >= 8, "ocppo_gemm_x6: stream-K needs >= 8 tiles (one range per XCD)");
    g.sk = 1;
    g.skws = static_cast<float*>(sk_workspace);
    g.skflag = reinterpret_cast<int*>(static_cast<char*>(sk_workspace) +
                                      static_cast<int64_t>(grid) * x6p_slot_bytes(tile));
    g.units = grid;
  }
  if (tile == 56) {
    g.mbig = mbig >= 0 ? mbig : x6_mixed_mbig((int)M, (int)N);
    OCPPO_REQUIRE(g.mbig >= 0 && g.mbig <= M && g.mbig % 128 == 0 && ((g.mbig / 128) * (N / 128)) % 8 == 0,
                  "ocppo_gemm_x6: mixed split at row %d", g.mbig);
  }
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const bool akc = sak == 1, bkc = sbk == 1;
  OCPPO_REQUIRE(launch_x6(s, tile, akc, bkc, g), "ocppo_gemm_x6: variant %d not built", tile);
  return check_launch("ocppo_gemm_x6");
}

// ocppo_gemm_x6 with one operand's rows gathered through a row table (include/ocppo.h)
extern "C" int ocppo_gemm_x6_gather(ocppo_stream_t stream, const float* a, int64_t sam,
                                    int64_t sak, const float* b, int64_t sbn, int64_t sbk,
                                    float* c, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                    int64_t splits, int64_t split_c, const float* bias, int relu,
                                    const void* b_planes, const int32_t* gidx, int64_t gw,
                                    int64_t gseg, int mode) {
  OCPPO_REQUIRE(M >= 128 && N >= 128 && K >= 32 && splits >= 1 && M <= INT32_MAX &&
                    N <= INT32_MAX && K <= INT32_MAX && M % 128 == 0 && N % 128 == 0 &&
                    K % kX6BK == 0 && (K / kX6BK) % splits == 0,
                "ocppo_gemm_x6_gather: bad sizes M=%lld N=%lld K=%lld splits=%lld (128 x 128 "
                "tiles, K / 32 steps split evenly)", (long long)M, (long long)N, (long long)K,
                (long long)splits);
  OCPPO_REQUIRE(a && (b || b_planes) && c && gidx, "ocppo_gemm_x6_gather: null pointer");
  OCPPO_REQUIRE(mode == 1 || mode == 2, "ocppo_gemm_x6_gather: mode %d (1: A rows, 2: B rows)",
                mode);
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(a) % 16 == 0 && reinterpret_cast<uintptr_t>(b) % 16 == 0,
                "ocppo_gemm_x6_gather: A and B must be 16-B aligned");
  OCPPO_REQUIRE(ldc >= N && (splits == 1 || (bias == nullptr && !relu)),
                "ocppo_gemm_x6_gather: ldc >= N; bias / ReLU need splits == 1");
  const int64_t kps = K / splits;  // K per split
  if (mode == 1) {
    // A(m, k) = a[gidx[m * gw + k / gseg] * sam + k % gseg]: each split's K range in one segment
    OCPPO_REQUIRE(sak == 1 && sam % 4 == 0 && gw >= 1 && gseg % kX6BK == 0 && gw * gseg == K &&
                      gseg % kps == 0,
                  "ocppo_gemm_x6_gather: mode 1 needs a k-contiguous A (row stride %% 4 == 0), "
                  "K = gw x gseg and every split inside one segment (gw=%lld gseg=%lld K=%lld "
                  "splits=%lld)", (long long)gw, (long long)gseg, (long long)K, (long long)splits);
    OCPPO_REQUIRE(b_planes != nullptr || (sbk == 1 && sbn >= K && sbn % 4 == 0),
                  "ocppo_gemm_x6_gather: mode 1 needs a k-contiguous B or its planes");
  } else {
    // B(n, k) = b[gidx[k * gw + n / gseg] * sbk + n % gseg]: each 128-column tile in one segment
    OCPPO_REQUIRE(sbn == 1 && sbk % 4 == 0 && gw >= 1 && gseg % 128 == 0 && gw * gseg == N &&
                      kps <= kX6GTbl && b_planes == nullptr,
                  "ocppo_gemm_x6_gather: mode 2 needs an n-contiguous B (row stride %% 4 == 0), "
                  "N = gw x gseg with gseg %% 128 == 0, K / splits <= %d rows and no planes",
                  kX6GTbl);
    OCPPO_REQUIRE(sam == 1 && sak >= M && sak % 4 == 0,
                  "ocppo_gemm_x6_gather: mode 2 needs an m-contiguous A");
  }
  const int64_t units = splits * (M / 128) * (N / 128);
  OCPPO_REQUIRE(units <= INT32_MAX / 2, "ocppo_gemm_x6_gather: too large");
  X6Args g{a, sam, sak, b_planes ? nullptr : b, sbn, sbk, c, ldc, bias, relu ? 1 : 0, (int)M,
           (int)N, (int)K, 0, 0, (int)units, (int)splits, split_c, nullptr, 0, nullptr, nullptr,
           nullptr, 0, static_cast<const uint16_t*>(b_planes), K, N * K, gidx, gw, gseg};
  clear_stale_error();
  launch_x6_gather(as_stream(stream), mode, g);
  return check_launch("ocppo_gemm_x6_gather");
}

namespace ocppo {
void wgrad_record(ocppo_deferred_finish_t* out, const float* partials, int G, int64_t N, int K,
                  float* dw, float* db);  // ocppo_linear_bwd.hip
}

// dX of a layer above a Linear+ReLU with the lower layer's whole backward in the epilogue
extern "C" int ocppo_gemm_x6_wgrad(ocppo_stream_t stream, const float* a, int64_t sam,
                                   int64_t sak, const float* b, int64_t sbn, int64_t sbk,
                                   int64_t M, int64_t N, int64_t K, const float* mask,
                                   int64_t ldm, const float* x, int64_t ldx, int64_t K1,
                                   float* dw, float* db, float* records, int64_t records_floats,
                                   int tile, ocppo_deferred_finish_t* finish) {
  OCPPO_REQUIRE(tile == 24 || tile == 27, "ocppo_gemm_x6_wgrad: tile %d (24 or 27)", tile);
  const X6Tile tc = kX6Tiles[tile & 7];
  const int64_t bm = 16 * tc.fm * tc.wgm, bn = 16 * tc.fn * tc.wgn;
  OCPPO_REQUIRE(M >= bm && N >= bn && M % bm == 0 && N % bn == 0 && K >= 32 && K % kX6BK == 0 &&
                    M <= INT32_MAX && N <= INT32_MAX && K <= INT32_MAX && K1 >= 1 && K1 <= 16,
                "ocppo_gemm_x6_wgrad: bad sizes M=%lld N=%lld K=%lld K1=%lld", (long long)M,
                (long long)N, (long long)K, (long long)K1);
  OCPPO_REQUIRE(a && b && mask && x && dw && db && records && finish,
                "ocppo_gemm_x6_wgrad: null pointer");
  OCPPO_REQUIRE(sak == 1 && sam >= K && sam % 4 == 0 && sbn == 1 && sbk >= N && sbk % 4 == 0 &&
                    ldm >= N && ldx >= K1,
                "ocppo_gemm_x6_wgrad: a k-contiguous A, an n-contiguous B (a dX product), "
                "ldm >= N, ldx >= K1");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(a) % 16 == 0 && reinterpret_cast<uintptr_t>(b) % 16 == 0,
                "ocppo_gemm_x6_wgrad: A and B must be 16-B aligned");
  OCPPO_REQUIRE(x6_windows_ok(sam, sak, sbn, sbk, K, 1, false),
                "ocppo_gemm_x6_wgrad: an operand window of one tile exceeds 2 GiB");
  const int64_t tiles_m = M / bm;
  const int64_t npw = ((N + kWgRecCols - 1) / kWgRecCols) * kWgRecCols * (wg_kp(K1) + 1);
  OCPPO_REQUIRE(records_floats >= tiles_m * npw,
                "ocppo_gemm_x6_wgrad: records need %lld floats", (long long)(tiles_m * npw));
  X6Args g{a, sam, sak, b, sbn, sbk, nullptr, N, nullptr, 0, (int)M, (int)N, (int)K,
           (int)tiles_m, (int)(N / bn), (int)(tiles_m * (N / bn)), 1, 0, mask, ldm, nullptr,
           nullptr, nullptr, 0, nullptr, 0, 0, nullptr, 0, 0, x, ldx, (int)K1, records, npw};
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const dim3 grid(g.units), block(64 * tc.wgm * tc.wgn);
  // the 64 x 64 tile (the fastest for the PPObj second layer's dX [11520 x 256] from K = 512,
  // tools/exp_gemm_x6.py) and the 128 x 128 one, K1 padded to 4 / 8 / 12 / 16
#define OCPPO_X6W(FM_, FN_, KP_)                                                                  \
  hipLaunchKernelGGL((gemm_x6_kernel<FM_, FN_, 2, 2, true, false, false, true, false, 0, KP_>),   \
                     grid, block, 0, s, g)
  const int kp = wg_kp(K1);
  if (tile == 27) {
    if (kp == 4) OCPPO_X6W(2, 2, 4); else if (kp == 8) OCPPO_X6W(2, 2, 8);
    else if (kp == 12) OCPPO_X6W(2, 2, 12); else OCPPO_X6W(2, 2, 16);
  } else {
    if (kp == 4) OCPPO_X6W(4, 4, 4); else if (kp == 8) OCPPO_X6W(4, 4, 8);
    else if (kp == 12) OCPPO_X6W(4, 4, 12); else OCPPO_X6W(4, 4, 16);
  }
#undef OCPPO_X6W
  if (int rc = check_launch("ocppo_gemm_x6_wgrad")) return rc;
  ocppo::wgrad_record(finish, records, static_cast<int>(tiles_m), N, static_cast<int>(K1), dw, db);
  return OCPPO_OK;
}

// ---------------------------------------------------------------------------------------------
// ocppo_conv_x6: NHWC convolutions (no padding, square stride) as implicit GEMMs on the x6
// products (the NatureCNN trunk, cleanrl/architectures/ppo.py:20-31, in the rollout forward at
// ppo_atari_oc.py:506 and the update at :566-606): no im2col buffer -- the loader reads each
// operand row's kernel-row segments (KW x C contiguous floats of the NHWC input) straight from the
// activation (X6Args cv_*). Three products per layer, all deterministic (no atomics; split-K
// partials summed in split order):
//   forward      y[r, co] = act(sum_k x(r, k) W[co, k] + b[co])       mode 0, GATH 3
//   weight grad  dW[co, k] = sum_r gp[r, co] x(r, k)                  mode 1, GATH 4 + sum_parts
//   data grad    the forward form over the zero-padded gradient with the flipped weight, one
//                launch per stride class (output rows through cv_out)  mode 0, GATH 3
// Tiles (FM, FN, WGM, WGN): 0 = 128 x 32 (2 waves), 1 = 32 x 128 (2 waves), 2 = 128 x 64,
// 3 = 64 x 64, 4 = 64 x 128, 5 = 128 x 128 (4 waves), 6 = 32 x 64 (2 waves: the rollout's few
// hundred rows per image batch still fill the CUs).
namespace ocppo {
constexpr X6Tile kConvTiles[] = {{4, 2, 2, 1}, {2, 4, 1, 2}, {4, 2, 2, 2}, {2, 2, 2, 2},
                                 {2, 4, 2, 2}, {4, 4, 2, 2}, {2, 2, 1, 2}};

template <int FM, int FN, int WGM, int WGN, int GATH>
static void launch_conv_t(hipStream_t s, X6Args& g) {
  g.tiles_m = g.M / (16 * FM * WGM);
  g.tiles_n = g.N / (16 * FN * WGN);
  constexpr bool KC = GATH == 3 || GATH == 5 || GATH == 7;  // rows forms: k-contiguous; wgrad: neither
  if constexpr (GATH == 3 || GATH == 7) {
    if (g.bpl) {  // the weight pre-split (ocppo_split_planes): B's stash is a copy, no split
      hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, true, true, false, true, true, GATH>),
                         dim3(g.units), dim3(64 * WGM * WGN), 0, s, g);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_x6_kernel<FM, FN, WGM, WGN, KC, KC, false, true, false, GATH>),
                     dim3(g.units), dim3(64 * WGM * WGN), 0, s, g);
}

static bool launch_conv(hipStream_t s, int mode, int tile, X6Args& g) {
  if (mode == 2) {  // the first convolution from u8 frame stacks: forward / weight gradient
    if (tile == 0) launch_conv_t<4, 2, 2, 1, 5>(s, g);
    else if (tile == 2) launch_conv_t<4, 2, 2, 2, 5>(s, g);
    else return false;
    return true;
  }
  if (mode == 3) {
    if (tile == 1) launch_conv_t<2, 4, 1, 2, 6>(s, g);
    else if (tile == 4) launch_conv_t<2, 4, 2, 2, 6>(s, g);
    else return false;
    return true;
  }
  if (mode == 4) {  // the data gradient from the unpadded output gradient (bounded rows)
    switch (tile) {
      case 2: launch_conv_t<4, 2, 2, 2, 7>(s, g); return true;
      case 3: launch_conv_t<2, 2, 2, 2, 7>(s, g); return true;
      case 5: launch_conv_t<4, 4, 2, 2, 7>(s, g); return true;
      case 6: launch_conv_t<2, 2, 1, 2, 7>(s, g); return true;
      default: return false;
    }
  }
  if (mode == 0) {
    switch (tile) {
      case 0: launch_conv_t<4, 2, 2, 1, 3>(s, g); return true;
      case 2: launch_conv_t<4, 2, 2, 2, 3>(s, g); return true;
      case 3: launch_conv_t<2, 2, 2, 2, 3>(s, g); return true;
      case 5: launch_conv_t<4, 4, 2, 2, 3>(s, g); return true;
      case 6: launch_conv_t<2, 2, 1, 2, 3>(s, g); return true;
      default: return false;
    }
  }
  switch (tile) {
    case 1: launch_conv_t<2, 4, 1, 2, 4>(s, g); return true;
    case 3: launch_conv_t<2, 2, 2, 2, 4>(s, g); return true;
    case 4: launch_conv_t<2, 4, 2, 2, 4>(s, g); return true;
    case 5: launch_conv_t<4, 4, 2, 2, 4>(s, g); return true;
    default: return false;
  }
}

// out[e] = sum_s part[s n + e] for any S: 16 groups of 64 lanes per 64 outputs, group q adding
// splits [q S / 16, (q + 1) S / 16) in order in f64, the groups added in order (fixed: bitwise
// reproducible), one f32 rounding
constexpr int kSumGroups = 16;
__global__ __launch_bounds__(64 * kSumGroups) void sum_parts_kernel(const float* __restrict__ part,
                                                                    int S, int64_t n,
                                                                    float* __restrict__ out,
                                                                    double div) {
  __shared__ double red[kSumGroups][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  const int s0 = q * S / kSumGroups, s1 = (q + 1) * S / kSumGroups;
  double acc = 0.0;
  if (e < n) {
#pragma unroll 8
    for (int sp = s0; sp < s1; ++sp) acc += static_cast<double>(part[static_cast<int64_t>(sp) * n + e]);
  }
  red[q][lane] = acc;
  __syncthreads();
  if (q == 0 && e < n) {
    double v = red[0][lane];
#pragma unroll
    for (int r = 1; r < kSumGroups; ++r) v += red[r][lane];
    out[e] = static_cast<float>(v / div);
  }
}

// ---------------------------------------------------------------------------------------------
// The first NatureCNN convolution (8 x 8 taps, stride 4, 32 output channels) from the u8 frame
// stacks with each IMAGE staged in LDS once (ocppo_conv_x6_u8 mode 0, tile 7). The tile loop
// above gathers every window from L2 (the 8 x 8 / 4 windows overlap 4x, and each loaded byte
// feeds only 32 output channels); here a workgroup copies a whole C x H x W stack into LDS with
// LDS-DMA (global_load_lds, 16 B per lane: no VGPRs, no wait in the compute path) while it
// computes the previous image (two image buffers), and every window row of 8 taps is then two
// dword reads from LDS converted to bf16 in registers (a byte is exact in bf16). Persistent: a
// workgroup takes images blockIdx.x, + gridDim.x, ...; the weight's three bf16 pieces stay in
// registers for all of them (split once per workgroup with x6_split2, the tile loop's own split).
// Same products in the same order as the tile loop (tile 0 / 2): per output element the K steps
// of 32 taps in order, each as the three MFMAs a0 b0, a0 b2, a0 b1 (x6_mfma3<true>) with the
// same lane <-> tap assignment, then / cdiv, + bias, ReLU: bitwise the same output
// (tests/test_conv_gpu.py).
constexpr int kImgCO = 32;   // output channels (two 16-column blocks)
constexpr int kImgKW = 8;    // taps per kernel row = one 8-bf16 fragment chunk
constexpr int kImgStride = 4;
constexpr int kImgChunk = 1024;  // bytes one global_load_lds wave instruction writes

struct ConvImgArgs {
  const uint8_t* src;
  const int64_t* idx;
  const float* w;     // [32, ldw], taps (c, ky, kx)
  int64_t ldw;
  const float* bias;  // [32] or null
  float* out;         // [B * P, 32]
  int B, H, W, OW, P;  // P = OH * OW output positions per image (P % 16 == 0)
  int relu;
  float cdiv;
  uint32_t* mbits;    // [B * P] or null: bit co of word r = out[r, co] > 0 (the ReLU mask)
  uint32_t* bnd;      // bounds-check builds: the violation record (else null) and the stack rows
  int64_t bnd_rows;
};

__device__ __forceinline__ uint32_t img_bf16x2(uint32_t v, int half) {
  // bytes 2 half, 2 half + 1 of v -> two bf16 (the upper halves of their exact f32 values)
  const float f0 = static_cast<float>(half ? (v >> 16) & 0xffu : v & 0xffu);
  const float f1 = static_cast<float>(half ? v >> 24 : (v >> 8) & 0xffu);
  return __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
}

// NW waves per workgroup: 4 (two workgroups per CU: one's image copy beside the other's MFMAs)
// for minibatch-sized batches, 8 for a batch of at most one image per CU (the rollout: the
// image's 25 row tiles over twice the waves)
template <int C, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_u8_img_kernel(ConvImgArgs a) {
  constexpr int KS = 2 * C;  // K steps of 32 taps: two per channel (kernel rows 0-3, 4-7)
  extern __shared__ __attribute__((aligned(16))) unsigned char conv_img_raw[];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int fr = lane & 15, fc = lane >> 4;
  const int64_t bytes = static_cast<int64_t>(C) * a.H * a.W;  // % 16 == 0 (host check)
  const int nchunks = static_cast<int>((bytes + kImgChunk - 1) / kImgChunk);
  const int64_t ibuf = static_cast<int64_t>(nchunks) * kImgChunk;  // one image buffer
  // one image's bytes -> buffer `buf`: wave wv copies chunks wv, wv + 4, ... (lane-linear 16 B)
  auto issue = [&](int64_t row, int buf) {
    const uint8_t* s = a.src + row * bytes;
    for (int ch = wv; ch < nchunks; ch += NW) {
      const int64_t off = static_cast<int64_t>(ch) * kImgChunk + 16 * lane;
      if (off < bytes)
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const void*>(s + off),
            (__attribute__((address_space(3))) void*)(conv_img_raw + buf * ibuf +
                                                      static_cast<int64_t>(ch) * kImgChunk),
            16, 0, 0);
    }
  };
  int b = blockIdx.x;
  if (b >= a.B) return;
  const int grid = static_cast<int>(gridDim.x);
  // the stack rows of this workgroup's images, 64 iterations at a time in one register (lane L:
  // iteration w0 + L), read back with readlane: uniform values without a vector load (and its
  // vmcnt wait, which would drain the LDS-DMA in flight) inside the loop
  auto window = [&](int it0) -> int64_t {
    const int bb = b + (it0 + lane) * grid;
    return bb < a.B ? bnd_check(a.bnd, kBndU8Row, a.idx[bb], 1, a.bnd_rows) : 0;
  };
  auto row_of = [&](int64_t win, int l) -> int64_t {
    const uint64_t u = static_cast<uint64_t>(win);
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(u), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(u >> 32), l);
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  int64_t win = window(0);
  issue(row_of(win, 0), 0);  // the first image's copy overlaps the weight split below
  // the weight's pieces: bw[j][kt][pl] = 8 taps k = 32 kt + 8 fc + e of output channel 16 j + fr
  bf16x8 bw[2][KS][3];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int kt = 0; kt < KS; ++kt) {
      const float* wr = a.w + static_cast<int64_t>(16 * j + fr) * a.ldw + 32 * kt + 8 * fc;
      const floatx4 lo = *reinterpret_cast<const floatx4*>(wr);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(wr + 4);
      uint32_t p[4][3];
      x6_split2(x6f2{lo[0], lo[1]}, p[0][0], p[0][1], p[0][2]);
      x6_split2(x6f2{lo[2], lo[3]}, p[1][0], p[1][1], p[1][2]);
      x6_split2(x6f2{hi[0], hi[1]}, p[2][0], p[2][1], p[2][2]);
      x6_split2(x6f2{hi[2], hi[3]}, p[3][0], p[3][1], p[3][2]);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        bw[j][kt][pl] = __builtin_bit_cast(bf16x8, u32x4{p[0][pl], p[1][pl], p[2][pl], p[3][pl]});
    }
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias[j] = a.bias ? a.bias[16 * j + fr] : 0.f;
  const int tiles = a.P / 16;
  for (int it = 0; b < a.B; b += gridDim.x, ++it) {
    // this image's copy (and every wave's reads of the buffer the next copy reuses) are done:
    // vmcnt(0) retires this wave's LDS-DMA (the compiler inserts no wait for it here), the
    // barrier everyone's
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int cur = it & 1;
    if (b + grid < a.B) {
      if (((it + 1) & 63) == 0) win = window(it + 1);  // (the copies in flight: none)
      issue(row_of(win, (it + 1) & 63), cur ^ 1);  // the next image's copy beside these MFMAs
    }
    const unsigned char* img = conv_img_raw + cur * ibuf;
    for (int tile = wv; tile < tiles; tile += NW) {
      const int pa = 16 * tile + fr;  // this lane's A row: output position (oy, ox)
      const int oy = pa / a.OW, ox = pa - oy * a.OW;
      const unsigned char* r0 = img + kImgStride * (oy * a.W + ox);
      floatx4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      // taps 32 kt + 8 fc + e = channel kt / 2, kernel row 4 (kt % 2) + fc, column e; the next
      // step's window row is read before this step's MFMAs
      auto row_words = [&](int kt, uint32_t& w0, uint32_t& w1) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(
            r0 + ((kt >> 1) * a.H + 4 * (kt & 1) + fc) * a.W);
        w0 = q[0];
        w1 = q[1];
      };
      uint32_t u0, u1;
      row_words(0, u0, u1);
#pragma unroll
      for (int kt = 0; kt < KS; ++kt) {
        uint32_t n0 = 0, n1 = 0;
        if (kt + 1 < KS) row_words(kt + 1, n0, n1);
        const bf16x8 af = __builtin_bit_cast(
            bf16x8, u32x4{img_bf16x2(u0, 0), img_bf16x2(u0, 1), img_bf16x2(u1, 0),
                          img_bf16x2(u1, 1)});
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][kt][0], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][kt][2], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[j][kt][1], acc[j], 0, 0, 0);
        }
        u0 = n0;
        u1 = n1;
      }
      // C/D layout: column fr of block j, rows 4 fc + r of the tile
      float ov[2][4];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[j][r] / a.cdiv;
          if (a.bias) v += bias[j];
          if (a.relu) v = relu_f(v);
          ov[j][r] = v;
          a.out[(static_cast<int64_t>(b) * a.P + 16 * tile + 4 * fc + r) * kImgCO + 16 * j + fr] = v;
        }
      if (a.mbits) {
        // row 4 fc + r's 32 mask bits: lanes 16 fc .. 16 fc + 15 of the two blocks' ballots
        uint32_t wd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint64_t b0 = __ballot(ov[0][r] > 0.f), b1 = __ballot(ov[1][r] > 0.f);
          wd[r] = static_cast<uint32_t>((b0 >> (16 * fc)) & 0xffffu) |
                  (static_cast<uint32_t>((b1 >> (16 * fc)) & 0xffffu) << 16);
        }
        if (fr == 0)
          *reinterpret_cast<uint4*>(a.mbits + static_cast<int64_t>(b) * a.P + 16 * tile + 4 * fc) =
              uint4{wd[0], wd[1], wd[2], wd[3]};
      }
    }
  }
}

// The first convolution's WEIGHT gradient with each image staged in LDS once (ocppo_conv_x6_u8
// mode 1, tile 8): dW[co, tap] = sum over images b and positions p of gp[b, p, co] u_b(p, tap) /
// divisor. The tile loop (GATH 6) walks the K = B OH OW rows through 32-row steps and gathers
// every window byte from L2; here K is taken image by image: a workgroup copies image b's u8
// stack's bytes into registers one image ahead (each thread the 9 dwords of one row segment per
// channel), then per channel writes them to LDS as 8 tap-column rows T[kx][y][ox] = img[c][y][4 ox
// + kx] (ox padded to 24), so that the 8 positions a lane feeds one MFMA for a fixed
// tap are 16 contiguous bytes; the kx and kx + 4 rows come from the same dwords (one window byte
// per phase q = kx % 4): 64 byte conversions per thread and channel. (An LDS-DMA copy of the raw
// image, as in the forward, made the compiler drain it before every T write.) K steps of 32 positions (rows of 24, so a lane's 8
// never cross an output row; 15 steps for a 20 x 20 output) are dealt to the 4 waves; a wave
// keeps the partial dW of its K steps for all 256 taps x 32 channels (32 accumulator blocks) over
// all its workgroup's images, and the gradient rows of its K steps in registers (split into the
// three bf16 pieces, x6_split2). Products per block and step: u0 g0, u0 g2, u0 g1 (x6_mfma3's
// order). Each wave writes its partial [32 co][256 taps] to workspace slot 4 blockIdx.x + wave;
// sum_parts_kernel then adds the 4 grid partials in slot order in f64 and divides once:
// deterministic (not the tile loop's summation order; tests compare with a float64 convolution).
// With mbits (the forward's ReLU bitmask, conv_u8_img_kernel) gp is the UNMASKED output gradient:
// each image's P mask words ride with its bytes (registers one image ahead, then LDS), a lane
// zeroes its gradient rows where the mask bit is clear before the split (relu_bias_grad's
// threshold_backward, so the products are those of the masked gradient, bitwise), and with dbp
// the masked rows' per-channel sums (the bias gradient) are kept per lane, reduced over the wave's
// row groups and written to dbp [4 grid, 32]: no masked copy of the gradient ever reaches HBM.
constexpr int kWgRow = 24;  // ox padded to a multiple of 8

struct ConvWgImgArgs {
  const uint8_t* src;
  const int64_t* idx;
  const float* gp;  // [B P, ldg]
  int64_t ldg;
  float* part;      // [4 grid, 32, 256]
  int B;
  const uint32_t* mbits;  // [B P] or null
  float* dbp;             // [4 grid, 32] or null
  uint32_t* bnd;          // bounds-check builds (as ConvImgArgs)
  int64_t bnd_rows;
};

template <int C, int H, int W, int OH, int OW>
__global__ __launch_bounds__(256, 1) void conv_u8_wgrad_img_kernel(ConvWgImgArgs a) {
  static_assert(W == kImgStride * (OW - 1) + kImgKW && H == kImgStride * (OH - 1) + kImgKW,
                "8 x 8 taps, stride 4, no padding");
  static_assert(OW <= kWgRow && (OH * kWgRow) % 32 == 0 && W % 4 == 0, "geometry");
  constexpr int P = OH * OW, KS = OH * kWgRow / 32, KSW = (KS + 3) / 4;  // K steps, per wave
  constexpr int64_t bytes = static_cast<int64_t>(C) * H * W;
  constexpr int kItems = H * (kWgRow / 8);  // T rows x 8-position groups per channel
  static_assert(kItems <= 256, "one T item per thread and channel");
  constexpr int kTRow = kWgRow * 2;  // bytes per T row
  constexpr int kTChan = 8 * H * kTRow;  // bytes per channel
  // [c][kx][y][24] bf16: every channel of the image at once (129 KB of the CU's 160)
  __shared__ __attribute__((aligned(16))) uint16_t T[C * 8 * H * kWgRow];
  // the image's mask words (a step's last 8-position group may read up to 7 past P: those
  // positions' gradient rows are zero whatever the word holds)
  static_assert(P <= 512, "two mask words per thread");
  __shared__ __attribute__((aligned(16))) uint32_t Mw[P + 8];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int fr = lane & 15, fc = lane >> 4;
  const int iy = t / (kWgRow / 8), ig = t - iy * (kWgRow / 8);  // this thread's T item
  const int grid = static_cast<int>(gridDim.x);
  // image bb's window dwords of this thread's item: raw[c][i] = dword i of row iy of channel c
  // from column 4 (8 ig + i) (phase q of it = img[c][iy][4 (8 ig + i) + q])
  uint32_t raw[C][9];
  auto load_raw = [&](int bb) {
    const bool ok = bb < a.B && t < kItems;
    const int64_t row = bb < a.B ? bnd_check(a.bnd, kBndU8Row, a.idx[bb], 1, a.bnd_rows) : 0;
    const uint8_t* sp = a.src + row * bytes + iy * W;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int col = 4 * (8 * ig + i);
        raw[c][i] = (ok && col + 4 <= W)
                        ? *reinterpret_cast<const uint32_t*>(sp + c * H * W + col)
                        : 0u;
      }
  };
  // the gradient rows of this wave's K step q: gr[q][j][e] = position k = 32 ks + 8 fc + e of
  // output channel 16 j + fr (zero in the row padding)
  float gr[KSW][2][8];
  auto load_g = [&](int bb, int q) {
    const int ks = wv + 4 * q;
    const int k0 = 32 * ks + 8 * fc, oy = k0 / kWgRow, ox0 = k0 - oy * kWgRow;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = bb < a.B && ks < KS && ox0 + e < OW;
        gr[q][j][e] =
            ok ? a.gp[(static_cast<int64_t>(bb) * P + oy * OW + ox0 + e) * a.ldg + 16 * j + fr]
               : 0.f;
      }
  };
  // image bb's mask words t, t + 256
  uint32_t mr[2];
  const bool masked = a.mbits != nullptr;
  auto load_m = [&](int bb) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = t + 256 * i;
      mr[i] = (masked && bb < a.B && p < P) ? a.mbits[static_cast<int64_t>(bb) * P + p] : 0u;
    }
  };
  float dbs[2] = {0.f, 0.f};  // this lane's masked gradient sums, channels fr, 16 + fr
  floatx4 acc[C * 4][2];  // tap block (c, 16-tap group) x channel block
#pragma unroll
  for (int i = 0; i < C * 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // every register set is refilled for the next image as soon as this image has consumed it, so
  // the loads run beside the rest of this image's work
  int b = blockIdx.x;
  load_raw(b);
  load_m(b);
#pragma unroll
  for (int q = 0; q < KSW; ++q) load_g(b, q);
  for (; b < a.B; b += grid) {
    __syncthreads();  // the previous image's T / Mw readers done
    if (masked) {
      Mw[t] = mr[0];
      if (t + 256 < P) Mw[t + 256] = mr[1];
    }
    if (t < kItems) {
      // T[c][kx][iy][8 ig + e] = img[c][iy][4 (8 ig + e) + kx] = phase kx % 4 of dword e + kx / 4
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int kx = 0; kx < 8; ++kx) {
          const int q = kx & 3, m = kx >> 2;
          // (the padding positions ox >= OW take whatever finite byte values the dwords hold:
          // their gradient rows are zero, so they add exact zeros -- no selects here)
          uint32_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float f0 = static_cast<float>((raw[c][2 * e + m] >> (8 * q)) & 0xffu);
            const float f1 = static_cast<float>((raw[c][2 * e + 1 + m] >> (8 * q)) & 0xffu);
            o[e] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
          }
          *reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(T) + c * kTChan +
                                    (kx * H + iy) * kTRow + 16 * ig) = uint4{o[0], o[1], o[2], o[3]};
        }
    }
    load_raw(b + grid);  // the next image's bytes, in flight during this image's MFMAs
    load_m(b + grid);
    __syncthreads();
    // this wave's K steps x all 256 taps (channel c's 4 blocks of 16: tap = 16 tb + fr -> ky =
    // 2 tb + fr / 8, kx = fr % 8)
#pragma unroll
    for (int q = 0; q < KSW; ++q) {
      const int ks = wv + 4 * q;
      if (ks >= KS) break;  // wave-uniform
      if (masked) {
        // positions oy OW + ox0 .. + 7 (ox0 % 8 == 0, OW % 4 == 0: 16-B aligned words)
        const int k0 = 32 * ks + 8 * fc, oy = k0 / kWgRow, ox0 = k0 - oy * kWgRow;
        const uint4 m0 = *reinterpret_cast<const uint4*>(Mw + oy * OW + ox0);
        const uint4 m1 = *reinterpret_cast<const uint4*>(Mw + oy * OW + ox0 + 4);
        const uint32_t mw[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (((mw[e] >> (16 * j + fr)) & 1u) == 0u) gr[q][j][e] = 0.f;
      }
      if (a.dbp) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 8; ++e) dbs[j] += gr[q][j][e];
      }
      bf16x8 gf[2][3];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        uint32_t pc[4][3];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          x6_split2(x6f2{gr[q][j][2 * e], gr[q][j][2 * e + 1]}, pc[e][0], pc[e][1], pc[e][2]);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          gf[j][pl] = __builtin_bit_cast(bf16x8, u32x4{pc[0][pl], pc[1][pl], pc[2][pl], pc[3][pl]});
      }
      load_g(b + grid, q);  // the next image's rows of this step
      const int k0 = 32 * ks + 8 * fc, oy = k0 / kWgRow, ox0 = k0 - oy * kWgRow;
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) {
          const int ky = 2 * tb + (fr >> 3), kx = fr & 7;
          const uint4 tv = *reinterpret_cast<const uint4*>(
              reinterpret_cast<const unsigned char*>(T) + c * kTChan +
              (kx * H + kImgStride * oy + ky) * kTRow + 2 * ox0);
          const bf16x8 af = __builtin_bit_cast(bf16x8, u32x4{tv.x, tv.y, tv.z, tv.w});
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            floatx4& ac = acc[4 * c + tb][j];
            ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, gf[j][0], ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, gf[j][2], ac, 0, 0, 0);
            ac = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, gf[j][1], ac, 0, 0, 0);
          }
        }
    }
  }
  // this wave's partial, transposed to [co][tap]: block (i, j) element (tap 16 i + 4 fc + r,
  // co 16 j + fr)
  float* pw = a.part + (static_cast<int64_t>(blockIdx.x) * 4 + wv) * (kImgCO * C * 64);
#pragma unroll
  for (int i = 0; i < C * 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pw[(16 * j + fr) * (C * 64) + 16 * i + 4 * fc + r] = acc[i][j][r];
  if (a.dbp) {
    // the wave's 4 row groups (xor 16, 32), then slot 4 blockIdx.x + wave like the weight's
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float s = dbs[j];
      s += __shfl_xor(s, 16, kWave);
      s += __shfl_xor(s, 32, kWave);
      if (fc == 0) a.dbp[(static_cast<int64_t>(blockIdx.x) * 4 + wv) * kImgCO + 16 * j + fr] = s;
    }
  }
}

// A convolution forward of FEW rows (the rollout's batch: ocppo_conv_x6 mode 0, tile 7) with the
// K steps split over the NW waves of a workgroup. The tile loop walks a tile's K steps one after
// another on 2 waves, so at 256 envs (20736 / 12544 rows of NatureCNN's second / third layer)
// each launch is a chain of 16-18 dependent load -> split -> MFMA steps (27.7 us). Here a
// workgroup owns a 32 x 16 FN output tile and wave w of NW takes K steps w, w + NW, ... (NW = 4:
// fastest of 4 / 8 / 16 at 256 envs, tools/exp_conv_rows.py), each wave's partial is
// summed with the other waves' through LDS in wave order (deterministic), then + bias, ReLU.
// Same x6 products per K step as the tile loop (x6_split2 pieces, x6_mfma6's order); the sum over
// K steps is grouped by wave instead of running in order: not the tile loop's bits, f32-level
// (tests/test_conv_gpu.py compares with a float64 convolution). Operand rows / taps through the
// same implicit-GEMM geometry (x6_cv_row / x6_cv_seg); KW C % 32 == 0 so 8 taps of a lane are
// contiguous.
#ifndef OCPPO_ROWS_NW  // waves per workgroup (experiments: tools/exp_conv_rows.py)
#define OCPPO_ROWS_NW 4
#endif
constexpr int kRowsNW = OCPPO_ROWS_NW;

// BPL: the weight's three bf16 pieces pre-split (ocppo_split_planes, once per rollout: the
// weights are fixed within it) -- the same pieces x6_split2 would form, read instead of split
template <int FN, bool BPL>
__global__ __launch_bounds__(64 * kRowsNW) void conv_x6_rows_kernel(X6Args g) {
  constexpr int NB = 2 * FN;  // 16 x 16 blocks of the 32 x 16 FN tile
  __shared__ __attribute__((aligned(16))) floatx4 red[kRowsNW][NB][kWave];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int fr = lane & 15, fc = lane >> 4;
  const int m0 = 32 * static_cast<int>(blockIdx.x);
  const float* __restrict__ x = g.a;
  const float* __restrict__ w = g.b;
  int64_t arow[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) arow[i] = x6_cv_row(g, m0 + 16 * i + fr);
  const int steps = g.K / kX6BK;
  floatx4 acc[2][FN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // one K step's operand values of this lane: A rows 16 i + fr, B columns 16 j + fr, taps
  // 32 kt + 8 fc .. + 8
  float4 va[2][2], vb[FN][2];
  uint4 vp[BPL ? FN : 1][3];
  auto load = [&](int kt, float4 (&a)[2][2], float4 (&b)[FN][2]) {
    const int k = kX6BK * kt + 8 * fc;
    const int64_t seg = x6_cv_seg(g, k);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float4* p = reinterpret_cast<const float4*>(x + x6_bnd(g, kBndX, arow[i] + seg, 8,
                                                                   g.bnd_x));
      a[i][0] = p[0];
      a[i][1] = p[1];
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (BPL) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          vp[j][pl] = *reinterpret_cast<const uint4*>(
              g.bpl + pl * g.bpl_ps + static_cast<int64_t>(16 * j + fr) * g.bpl_ld + k);
      } else {
        const float4* p =
            reinterpret_cast<const float4*>(w + static_cast<int64_t>(16 * j + fr) * g.sbn + k);
        b[j][0] = p[0];
        b[j][1] = p[1];
      }
    }
  };
  auto pieces = [&](const float4 (&v)[2], bf16x8 (&f)[3]) {
    uint32_t p[4][3];
    x6_split2(x6f2{v[0].x, v[0].y}, p[0][0], p[0][1], p[0][2]);
    x6_split2(x6f2{v[0].z, v[0].w}, p[1][0], p[1][1], p[1][2]);
    x6_split2(x6f2{v[1].x, v[1].y}, p[2][0], p[2][1], p[2][2]);
    x6_split2(x6f2{v[1].z, v[1].w}, p[3][0], p[3][1], p[3][2]);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      f[pl] = __builtin_bit_cast(bf16x8, u32x4{p[0][pl], p[1][pl], p[2][pl], p[3][pl]});
  };
  int kt = wv;
  if (kt < steps) load(kt, va, vb);
  for (; kt < steps; kt += kRowsNW) {
    bf16x8 af[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i) pieces(va[i], af[i]);
#pragma unroll
    for (int j = 0; j < FN; ++j) {  // B's pieces block by block (fewer live registers)
      bf16x8 bfr[3];
      if constexpr (BPL) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) bfr[pl] = __builtin_bit_cast(bf16x8, vp[j][pl]);
      } else {
        pieces(vb[j], bfr);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) x6_mfma6<false>(af[i], bfr, acc[i][j], acc[i][j]);
    }
    if (kt + kRowsNW < steps) load(kt + kRowsNW, va, vb);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) red[wv][i * FN + j][lane] = acc[i][j];
  __syncthreads();
  // block blk = (i, j): the waves' partials in wave order, then bias, ReLU; C/D layout: column
  // fr of the block, rows 4 fc + r
  for (int blk = wv; blk < NB; blk += kRowsNW) {
    floatx4 s = red[0][blk][lane];
#pragma unroll
    for (int q = 1; q < kRowsNW; ++q) s += red[q][blk][lane];
    const int i = blk / FN, j = blk - i * FN;
    const int col = 16 * j + fr;
    const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = s[r] + bv;
      if (g.relu) v = relu_f(v);
      g.c[static_cast<int64_t>(m0 + 16 * i + 4 * fc + r) * g.ldc + col] = v;
    }
  }
}

static int conv_u8_img_grid(int B) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    cus = n;
  }
  return B < 2 * cus ? B : 2 * cus;
}

}  // namespace ocppo

extern "C" int ocppo_conv_x6(ocppo_stream_t stream, int mode, const float* x, const int64_t* geom,
                             const float* w, int64_t ldw, float* c, int64_t ldc, int64_t M,
                             int64_t N, int64_t K, int64_t splits, const float* bias, int relu,
                             const int64_t* out_geom, int tile, float* out, const int64_t* pad,
                             const float* mask, float* dbp, const uint16_t* w_planes,
                             uint32_t* mbits_rows) {
  OCPPO_REQUIRE(mode == 0 || mode == 1, "ocppo_conv_x6: mode %d (0 rows, 1 weight gradient)", mode);
  OCPPO_REQUIRE(tile >= 0 && tile < 8, "ocppo_conv_x6: tile %d", tile);
  OCPPO_REQUIRE(x && geom && w && c, "ocppo_conv_x6: null pointer");
  const int64_t qh = geom[0], qw = geom[1], sb = geom[2], ys = geom[3], xs = geom[4],
                segs = geom[5], gseg = geom[6];
  if (tile == 7) {  // few rows: K steps split over the waves of a workgroup (conv_x6_rows_kernel)
    OCPPO_REQUIRE(mode == 0 && (N == 32 || N == 64) && M >= 32 && M % 32 == 0 && K >= kX6BK &&
                      K % kX6BK == 0 && splits == 1 && !out_geom && !pad && !mask && !dbp &&
                      !mbits_rows &&
                      gseg % kX6BK == 0 && ldw >= K && ldw % 4 == 0 && ldc >= N &&
                      M <= INT32_MAX && K <= INT32_MAX && qh >= 1 && qw >= 1 &&
                      M % (qh * qw) == 0 && M < (int64_t{1} << 24) && sb % 4 == 0 &&
                      ys % 4 == 0 && xs % 4 == 0 && segs % 4 == 0 &&
                      reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(w) % 16 == 0,
                  "ocppo_conv_x6: tile 7 needs mode 0, N = 32 or 64, 32 | M, 32 | K, kernel-row "
                  "segments of a multiple of 32, splits 1, no output map / pad / mask (M=%lld "
                  "N=%lld K=%lld)", (long long)M, (long long)N, (long long)K);
    X6Args g{};
    g.a = x;
    g.b = w;
    g.sbn = ldw;
    g.sbk = 1;
    g.c = c;
    g.ldc = ldc;
    g.M = (int)M;
    g.N = (int)N;
    g.K = (int)K;
    g.splits = 1;
    g.bias = bias;
    g.relu = relu ? 1 : 0;
    g.cv_qh = (int)qh;
    g.cv_qw = (int)qw;
    g.cv_sb = sb;
    g.cv_ys = ys;
    g.cv_xs = xs;
    g.cv_segs = segs;
    g.cv_gseg = (int)gseg;
    x6_bounds_args(g);
    if (w_planes) {
      OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(w_planes) % 16 == 0,
                    "ocppo_conv_x6: w_planes must be 16-B aligned");
      g.bpl = w_planes;
      g.bpl_ld = K;
      g.bpl_ps = N * K;
    }
    clear_stale_error();
    const dim3 grid(static_cast<unsigned>(M / 32)), block(64 * kRowsNW);
    hipStream_t s = as_stream(stream);
    if (N == 64 && w_planes)
      hipLaunchKernelGGL((conv_x6_rows_kernel<4, true>), grid, block, 0, s, g);
    else if (N == 64)
      hipLaunchKernelGGL((conv_x6_rows_kernel<4, false>), grid, block, 0, s, g);
    else if (w_planes)
      hipLaunchKernelGGL((conv_x6_rows_kernel<2, true>), grid, block, 0, s, g);
    else
      hipLaunchKernelGGL((conv_x6_rows_kernel<2, false>), grid, block, 0, s, g);
    return check_launch("ocppo_conv_x6 (tile 7)");
  }
  OCPPO_REQUIRE(!w_planes || (mode == 0 && reinterpret_cast<uintptr_t>(w_planes) % 16 == 0 &&
                                K % 8 == 0),
                "ocppo_conv_x6: w_planes needs mode 0 (16-B aligned, K %% 8 == 0)");
  OCPPO_REQUIRE(!mbits_rows || (mode == 0 && relu && splits == 1 && !out_geom && !pad && !mask &&
                                N % 32 == 0 && ldc == N && kConvTiles[tile].fn % 2 == 0 &&
                                reinterpret_cast<uintptr_t>(mbits_rows) % 4 == 0),
                "ocppo_conv_x6: mbits_rows needs the forward with relu, splits 1, ldc == N, "
                "32 | N and a tile of an even number of block columns");
  const X6Tile tc = kConvTiles[tile];
  const int64_t bm = 16 * tc.fm * tc.wgm, bn = 16 * tc.fn * tc.wgn;
  OCPPO_REQUIRE(M >= bm && N >= bn && M % bm == 0 && N % bn == 0 && K >= kX6BK && K % kX6BK == 0 &&
                    splits >= 1 && K / kX6BK >= splits && M <= INT32_MAX && N <= INT32_MAX &&
                    K <= INT32_MAX,
                "ocppo_conv_x6: bad sizes M=%lld N=%lld K=%lld splits=%lld (tile %lld x %lld)",
                (long long)M, (long long)N, (long long)K, (long long)splits, (long long)bm,
                (long long)bn);
  OCPPO_REQUIRE(qh >= 1 && qw >= 1 && gseg >= 4 && gseg % 4 == 0 && sb % 4 == 0 && ys % 4 == 0 &&
                    xs % 4 == 0 && segs % 4 == 0 && sb >= 0 && ys >= 0 && xs >= 0 && segs >= 0,
                "ocppo_conv_x6: bad geometry (qh %lld qw %lld sb %lld ys %lld xs %lld segs %lld "
                "gseg %lld: strides multiples of 4 floats)", (long long)qh, (long long)qw,
                (long long)sb, (long long)ys, (long long)xs, (long long)segs, (long long)gseg);
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0,
                "ocppo_conv_x6: x and w must be 16-B aligned");
  const int64_t rows = mode == 0 ? M : K;  // the convolution rows (b, qy, qx)
  OCPPO_REQUIRE(rows % (qh * qw) == 0 && rows < (int64_t{1} << 24),
                "ocppo_conv_x6: %lld rows: a whole number of %lld x %lld images, < 2^24",
                (long long)rows, (long long)qh, (long long)qw);
  X6Args g{};
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.splits = (int)splits;
  g.units = (int)(splits * (M / bm) * (N / bn));
  g.cv_qh = (int)qh;
  g.cv_qw = (int)qw;
  g.cv_sb = sb;
  g.cv_ys = ys;
  g.cv_xs = xs;
  g.cv_segs = segs;
  g.cv_gseg = (int)gseg;
  if (mode == 0) {
    // A = x gathered, B = W [N, K] (row stride ldw), C [M, N] (ldc) or a stride class's rows
    OCPPO_REQUIRE(gseg % kX6BK == 0 && ldw >= K && ldw % 4 == 0 &&
                      (splits == 1 || (bias == nullptr && !relu && !out_geom && ldc == N)) &&
                      (out_geom != nullptr || ldc >= N),
                  "ocppo_conv_x6: the rows form needs kernel-row segments of a multiple of 32, "
                  "a k-contiguous W (ldw %lld >= K, %% 4), splits == 1, ldc >= N", (long long)ldw);
    g.a = x;
    g.sak = 1;
    g.b = w;
    g.sbn = ldw;
    g.sbk = 1;
    g.c = c;
    g.ldc = ldc;
    g.split_c = M * N;  // splits > 1: partials [splits, M, N] (ocppo_sum_splits_act adds them)
    if (w_planes) {  // B = w pre-split into three bf16 planes [3, N, K]
      g.bpl = w_planes;
      g.bpl_ld = K;
      g.bpl_ps = N * K;
    }
    if (mbits_rows) {  // the ReLU mask as a row-major bitmask [M, N / 32] (relu_bias_grad_bits)
      g.mbits_out = reinterpret_cast<uint64_t*>(mbits_rows);
      g.mbits_rows = 1;
    }
    g.bias = bias;
    g.relu = relu ? 1 : 0;
    if (mask) {  // the layer below's ReLU backward: c = mask > 0 ? acc : 0, column sums -> dbp
      OCPPO_REQUIRE(dbp && splits == 1 && bias == nullptr && !relu,
                    "ocppo_conv_x6: the mask epilogue needs dbp, splits == 1, no bias / ReLU");
      g.mask = mask;
      g.ldm = ldc;
      g.dbp = dbp;
    }
    if (out_geom) {
      g.cv_out = 1;
      g.co_sb = out_geom[0];
      g.co_ys = out_geom[1];
      g.co_xs = out_geom[2];
      g.co_off = out_geom[3];
      g.co_cw = static_cast<int>(out_geom[4]);
      g.co_cs = static_cast<int>(out_geom[5]);
      g.co_cy = out_geom[6];
      g.co_cx = out_geom[7];
      OCPPO_REQUIRE(g.co_cw >= 1 && g.co_cs >= 1 && N % g.co_cw == 0 &&
                        N / g.co_cw <= static_cast<int64_t>(g.co_cs) * g.co_cs,
                    "ocppo_conv_x6: output columns: %lld classes of %d", (long long)(N / g.co_cw),
                    g.co_cw);
    }
  } else {
    // A(m = co, k = r) = gp[r ldw + m], B(n, k = r) = x gathered; partials [splits, M, N] in c,
    // summed in split order into out [M, N]
    OCPPO_REQUIRE(out && ldw >= M && ldw % 4 == 0 && bias == nullptr && !relu && !out_geom &&
                      qh * qw <= kX6GTbl && N <= gseg * ((segs > 0) ? (INT32_MAX / segs) : 1),
                  "ocppo_conv_x6: the weight-gradient form needs out, an m-contiguous gradient "
                  "(ldw %lld >= M, %% 4), no epilogue, <= %d pixels per image", (long long)ldw,
                  kX6GTbl);
    OCPPO_REQUIRE((qh - 1) * ys + (qw - 1) * xs < INT32_MAX, "ocppo_conv_x6: image too large");
    g.a = w;
    g.sam = 1;
    g.sak = ldw;
    g.b = x;
    g.sbn = 1;
    g.c = c;
    g.ldc = N;
    g.split_c = M * N;
  }
  x6_bounds_args(g);
  int lmode = mode;
  if (pad) {
    // x is the UNPADDED gradient [B, ih, iw, C]; geom's strides describe the padded one it stands
    // for (ys = (iw + 2 pw) C would be the padded row): rebuilt here for the unpadded source
    OCPPO_REQUIRE(mode == 0 && splits == 1 && pad[0] >= 0 && pad[1] >= 0 && pad[2] >= 1 &&
                      pad[3] >= 1 && pad[4] >= 4 && pad[4] % 4 == 0 && gseg % pad[4] == 0,
                  "ocppo_conv_x6: pad = {ph, pw, ih, iw, C} (the rows form only)");
    g.cv_ph = (int)pad[0];
    g.cv_pw = (int)pad[1];
    g.cv_ih = (int)pad[2];
    g.cv_iw = (int)pad[3];
    g.cv_c = (int)pad[4];
    g.cv_sb = pad[2] * pad[3] * pad[4];
    g.cv_ys = pad[3] * pad[4];
    g.cv_xs = pad[4];
    g.cv_segs = pad[3] * pad[4];
    lmode = 4;
  }
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  OCPPO_REQUIRE(launch_conv(s, lmode, tile, g), "ocppo_conv_x6: tile %d not built for mode %d",
                tile, mode);
  if (int rc = check_launch("ocppo_conv_x6")) return rc;
  if (mode == 1) {
    const int64_t n = M * N;
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64 * kSumGroups), 0,
                       s, c, (int)splits, n, out, 1.0);
    return check_launch("ocppo_conv_x6 (sum_parts)");
  }
  return OCPPO_OK;
}

extern "C" int ocppo_conv_x6_u8(ocppo_stream_t stream, int mode, const uint8_t* src,
                                const int64_t* idx, int64_t C, int64_t H, int64_t W, int64_t KH,
                                int64_t KW, int64_t stride, const float* w, int64_t ldw, float* c,
                                int64_t M, int64_t N, int64_t K, int64_t splits, const float* bias,
                                int relu, float divisor, int tile, float* out, uint32_t* mbits,
                                float* dbp, float* db) {
  OCPPO_REQUIRE(mode == 0 || mode == 1, "ocppo_conv_x6_u8: mode %d (0 rows, 1 weight gradient)",
                mode);
  OCPPO_REQUIRE(src && idx && w && c && (mode == 0 || out), "ocppo_conv_x6_u8: null pointer");
  OCPPO_REQUIRE(C >= 1 && KH >= 1 && KW >= 1 && stride >= 1 && H >= KH && W >= KW &&
                    (H - KH) % stride == 0 && (W - KW) % stride == 0 && KW % 4 == 0 &&
                    W % 4 == 0 && stride % 4 == 0 && divisor > 0.f,
                "ocppo_conv_x6_u8: geometry C=%lld H=%lld W=%lld KH=%lld KW=%lld stride=%lld "
                "(KW, W, stride multiples of 4; no padding)", (long long)C, (long long)H,
                (long long)W, (long long)KH, (long long)KW, (long long)stride);
  const int64_t OH = (H - KH) / stride + 1, OW = (W - KW) / stride + 1, taps = C * KH * KW;
  const int64_t rows = mode == 0 ? M : K;
  if (tile == 7) {  // the image-staged forward (conv_u8_img_kernel)
    const int64_t P = OH * OW, bytes = C * H * W;
    OCPPO_REQUIRE(mode == 0 && C == 4 && KH == kImgKW && KW == kImgKW && stride == kImgStride &&
                      N == kImgCO && K == taps && splits == 1 && P % 16 == 0 && M % P == 0 &&
                      M / P <= INT32_MAX && bytes % 16 == 0 &&
                      2 * ((bytes + kImgChunk - 1) / kImgChunk) * kImgChunk <= 64 * 1024 &&
                      ldw >= K && ldw % 4 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(w) % 16 == 0 && M / P >= 1,
                  "ocppo_conv_x6_u8: tile 7 (image-staged) needs mode 0, C = 4, 8 x 8 taps, "
                  "stride 4, 32 output channels, 16 | OH OW, a 16-B aligned src with 16 | C H W, "
                  "two image buffers of C H W (1 KiB-rounded) <= 64 KB (C=%lld H=%lld W=%lld N=%lld M=%lld)", (long long)C,
                  (long long)H, (long long)W, (long long)N, (long long)M);
    OCPPO_REQUIRE(!dbp && !db && (!mbits || (relu && reinterpret_cast<uintptr_t>(mbits) % 16 == 0)),
                  "ocppo_conv_x6_u8: tile 7 takes mbits (16-B aligned, with relu) and no dbp / db");
    ConvImgArgs ia{src, idx, w, ldw, bias, c, static_cast<int>(M / P), static_cast<int>(H),
                   static_cast<int>(W), static_cast<int>(OW), static_cast<int>(P), relu ? 1 : 0,
                   divisor, mbits, nullptr, 0};
    img_bounds_args(ia.bnd, ia.bnd_rows);
    clear_stale_error();
    const size_t ibuf = static_cast<size_t>((bytes + kImgChunk - 1) / kImgChunk) * kImgChunk;
    const int grid = conv_u8_img_grid(ia.B);
    if (grid <= conv_u8_img_grid(1 << 30) / 2)  // at most one image per CU: 8 waves each
      hipLaunchKernelGGL((conv_u8_img_kernel<4, 8>), dim3(grid), dim3(512), 2 * ibuf,
                         as_stream(stream), ia);
    else
      hipLaunchKernelGGL((conv_u8_img_kernel<4, 4>), dim3(grid), dim3(256), 2 * ibuf,
                         as_stream(stream), ia);
    return check_launch("ocppo_conv_x6_u8 (image-staged)");
  }
  if (tile == 8) {  // the image-staged weight gradient (conv_u8_wgrad_img_kernel)
    constexpr int64_t kC = 4, kH = 84, kW = 84;
    const int64_t P = OH * OW, bytes = C * H * W;
    OCPPO_REQUIRE(mode == 1 && C == kC && H == kH && W == kW && KH == kImgKW && KW == kImgKW &&
                      stride == kImgStride && M == kImgCO && N == taps && K % P == 0 &&
                      K / P <= INT32_MAX && splits >= 4 && splits % 4 == 0 &&
                      splits / 4 <= 65536 && ldw >= M && ldw % 4 == 0 && bias == nullptr &&
                      !relu && reinterpret_cast<uintptr_t>(src) % 16 == 0 && bytes % 16 == 0,
                  "ocppo_conv_x6_u8: tile 8 (image-staged weight gradient) needs mode 1, "
                  "4 x 84 x 84 stacks, 8 x 8 taps, stride 4, 32 output channels, splits = 4 x "
                  "workgroups, a 16-B aligned src (C=%lld H=%lld W=%lld M=%lld K=%lld splits=%lld)",
                  (long long)C, (long long)H, (long long)W, (long long)M, (long long)K,
                  (long long)splits);
    OCPPO_REQUIRE((dbp == nullptr) == (db == nullptr) &&
                      (!mbits || reinterpret_cast<uintptr_t>(mbits) % 16 == 0),
                  "ocppo_conv_x6_u8: tile 8 takes dbp and db together, a 16-B aligned mbits");
    ConvWgImgArgs wa{src, idx, w, ldw, c, static_cast<int>(K / P), mbits, dbp, nullptr, 0};
    img_bounds_args(wa.bnd, wa.bnd_rows);
    clear_stale_error();
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL((conv_u8_wgrad_img_kernel<4, 84, 84, 20, 20>),
                       dim3(static_cast<unsigned>(splits / 4)), dim3(256), 0, s, wa);
    if (int rc = check_launch("ocppo_conv_x6_u8 (image-staged weight gradient)")) return rc;
    const int64_t n = M * N;
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64 * kSumGroups), 0,
                       s, c, (int)splits, n, out, static_cast<double>(divisor));
    if (int rc = check_launch("ocppo_conv_x6_u8 (sum_parts)")) return rc;
    if (!db) return OCPPO_OK;
    hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(64 * kSumGroups), 0, s, dbp, (int)splits,
                       int64_t{kImgCO}, db, 1.0);
    return check_launch("ocppo_conv_x6_u8 (bias gradient)");
  }
  OCPPO_REQUIRE(!mbits && !dbp && !db, "ocppo_conv_x6_u8: mbits / dbp / db need tile 7 or 8");
  const X6Tile tc = kConvTiles[tile >= 0 && tile < 7 ? tile : 0];
  const int64_t bm = 16 * tc.fm * tc.wgm, bn = 16 * tc.fn * tc.wgn;
  OCPPO_REQUIRE(M % bm == 0 && N % bn == 0 && K % kX6BK == 0 && splits >= 1 &&
                    K / kX6BK >= splits && rows % (OH * OW) == 0 && rows < (int64_t{1} << 24) &&
                    (mode == 0 ? (N <= INT32_MAX && K == taps && taps / 4 <= kX6GTbl)
                               : (N == taps && OH * OW <= kX6GTbl)),
                "ocppo_conv_x6_u8: bad sizes M=%lld N=%lld K=%lld splits=%lld", (long long)M,
                (long long)N, (long long)K, (long long)splits);
  OCPPO_REQUIRE(mode == 0 ? (ldw >= K && ldw % 4 == 0 && splits == 1)
                          : (ldw >= M && ldw % 4 == 0 && bias == nullptr && !relu),
                "ocppo_conv_x6_u8: operand strides / epilogue (ldw %lld)", (long long)ldw);
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(src) % 4 == 0 && reinterpret_cast<uintptr_t>(w) % 16 == 0,
                "ocppo_conv_x6_u8: src 4-B and w 16-B aligned");
  X6Args g{};
  g.M = (int)M;
  g.N = (int)N;
  g.K = (int)K;
  g.splits = (int)splits;
  g.units = (int)(splits * (M / bm) * (N / bn));
  g.cv_qh = (int)OH;
  g.cv_qw = (int)OW;
  g.cv_ys = stride * W;
  g.cv_xs = stride;
  g.u8 = src;
  g.u8_idx = idx;
  g.u8_img = C * H * W;
  g.u8_hw = H * W;
  g.u8_w = W;
  g.u8_khw = (int)(KH * KW);
  g.u8_kw = (int)KW;
  g.u8_nimg = (int)(rows / (OH * OW));
  g.cdiv = divisor;
  x6_bounds_args(g);
  if (mode == 0) {  // y = act(sum_k u(r, k) w[n, k] / divisor + bias)
    g.sak = 1;
    g.b = w;
    g.sbn = ldw;
    g.sbk = 1;
    g.c = c;
    g.ldc = N;
    g.bias = bias;
    g.relu = relu ? 1 : 0;
  } else {  // dW[m, n] = sum_r gp[r ldw + m] u(r, n) / divisor: split partials, ordered sum
    g.a = w;
    g.sam = 1;
    g.sak = ldw;
    g.sbn = 1;
    g.c = c;
    g.ldc = N;
    g.split_c = M * N;
  }
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  OCPPO_REQUIRE(launch_conv(s, mode + 2, tile, g), "ocppo_conv_x6_u8: tile %d not built for mode %d",
                tile, mode);
  if (int rc = check_launch("ocppo_conv_x6_u8")) return rc;
  if (mode == 1) {
    const int64_t n = M * N;
    hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64 * kSumGroups), 0,
                       s, c, (int)splits, n, out, static_cast<double>(divisor));
    return check_launch("ocppo_conv_x6_u8 (sum_parts)");
  }
  return OCPPO_OK;
}

