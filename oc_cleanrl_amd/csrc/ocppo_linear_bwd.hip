// Backward of a Linear(+ReLU) layer's elementwise part in ONE pass over the output gradient:
//   gp = threshold_backward(g, out, 0)   (out <= 0 ? 0 : g; skipped without ReLU: gp = g)
//   db = gp.sum(0)                       (the bias gradient)
// i.e. what autograd runs for `nn.ReLU()` after `nn.Linear` plus the Linear's bias grad inside
// `loss.backward()` of cleanrl/ppo_atari_oc.py:605, for the PPObj layers of
// architectures/ppo.py:60-84 (and the NatureCNN head :44-46). ATen does it as two passes
// (threshold_backward reads g and out and writes gp; sum reads gp again, with a column reduction
// that runs at ~2 TB/s on [12288, 1024]); here g and out are read once, gp written once.
//
// Deterministic column reduction without atomics on data: the rows are cut into `chunks` equal
// ranges; workgroup (stripe, chunk) owns a stripe of 4L columns x one row range (L lanes per row,
// 4 adjacent columns per lane, 16-B accesses, 64/L rows per wave instruction; 4 waves split the
// rows), sums its rows in a fixed order, combines waves and row-lanes through LDS in a fixed
// order and publishes its partial column sums with write-through (sc1) stores; the last
// workgroup of a stripe to arrive on the stripe's ticket (one 128-B line per stripe) sums the
// `chunks` partials of each column: the 256 threads split the chunks into 256/(4L) ordered groups
// per column (32 loads in flight each), then add the group sums in group order. rb_plan picks L,
// the stripes and the chunks (<= 64 for wide N) so a launch has >= 512 workgroups where the rows
// allow it (tools/exp_relu_bias.py: chunk caps 16 / 32 / 64 / 128 measured, 64 best). Hand-off per
// MI355X_MICROARCH.md "Valid forms" row 1 (sc1 stores, every storing wave's vmcnt(0), barrier,
// one agent-scope atomic add; the last arriver reads with sc1 loads). Tickets re-arm themselves.
// Roofline: HBM / Infinity-Cache stream, 12 B per element (relu) or 4 B (no relu) + 4 B per
// partial; no flops to speak of.
#include <cstring>

#include "ocppo_common.h"

namespace ocppo {

constexpr int kRbMaxStripes = 64;
constexpr int kRbMaxChunks = 512;
#ifndef OCPPO_RB_CHUNKS
#define OCPPO_RB_CHUNKS 64
#endif
constexpr int kRbChunks = OCPPO_RB_CHUNKS;  // wide-N chunk cap
constexpr size_t kRbTicketBytes = kRbMaxStripes * 128;

// Launch plan: L lanes per row (4 columns each: a stripe is 4L columns, 64/L rows per wave
// instruction), `stripes` column stripes x `chunks` row chunks workgroups.
struct RbPlan {
  int L, stripes, chunks;
};

inline RbPlan rb_plan(int64_t R, int64_t N) {
  const int64_t q = N / 4;
  RbPlan p;
  // narrow N (N/4 divides 64, e.g. conv channels 32 / 64): several rows per wave instruction
  p.L = (q < 64 && 64 % q == 0) ? static_cast<int>(q) : 64;
  p.stripes = static_cast<int>((N + 4 * p.L - 1) / (4 * p.L));
  const int64_t by_rows = (R + 31) / 32;  // >= 32 rows per chunk
  if (p.stripes == 1 && p.L < 64) {
    // tall narrow (NHWC conv outputs): ~64K elements per workgroup, 128..512 chunks
    int64_t c = (R * N + 65535) / 65536;
    if (c < 128) c = 128;
    if (c > kRbMaxChunks) c = kRbMaxChunks;
    if (c > by_rows) c = by_rows;
    p.chunks = static_cast<int>(c < 1 ? 1 : c);
    return p;
  }
  // <= kRbChunks chunks per stripe (the last arriver's loads of a column are ONE batch in flight
  // per thread group); narrower stripes (down to 8 lanes = 32 columns, 128-B row pieces) until the
  // launch has >= 512 workgroups (two per CU) when the rows allow it
  const int64_t c = by_rows < kRbChunks ? by_rows : kRbChunks;
  while (static_cast<int64_t>(p.stripes) * c < 512 && p.L > 8) {
    const int L2 = p.L / 2;
    const int s2 = static_cast<int>((N + 4 * L2 - 1) / (4 * L2));
    if (s2 > kRbMaxStripes) break;
    p.L = L2;
    p.stripes = s2;
  }
  p.chunks = static_cast<int>(c < 1 ? 1 : c);
  return p;
}

// TAIL = false: every workgroup stores its partial column sums (plain stores) and is done; the
// chunk sums are left to a later kernel of the same stream (ocppo_sum_splits_db, which runs after
// the layer's split-K weight gradient anyway): no ticket, no last-arriver tail on this launch.
// MB: the ReLU mask read as a row-major bitmask (bit c % 32 of word r N / 32 + c / 32 = out[r, c]
// > 0, the producing forward's epilogue: ocppo_conv_x6 mbits_out) instead of the f32 output --
// 4 B -> 1 bit of mask traffic per element
template <bool RELU, bool TAIL = true, bool MB = false>
__global__ __launch_bounds__(256) void relu_bias_grad_kernel(const float* __restrict__ g,
                                                             const float* __restrict__ out,
                                                             float* __restrict__ gp,
                                                             float* __restrict__ db, int64_t R,
                                                             int64_t N, int L, int chunks,
                                                             unsigned* __restrict__ tickets,
                                                             float* __restrict__ partials,
                                                             const uint32_t* __restrict__ mbits =
                                                                 nullptr) {
  __shared__ float4 red[4][64];
  __shared__ float tail[256];
  __shared__ int s_last;
  const int SW = 4 * L;  // columns per stripe
  const int nstripes = static_cast<int>((N + SW - 1) / SW);
  const int stripe = blockIdx.x % nstripes;
  const int chunk = blockIdx.x / nstripes;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int RP = 64 / L;
  const int lrow = lane / L, lcol = lane - lrow * L;
  const int64_t c0 = static_cast<int64_t>(stripe) * SW + 4 * lcol;
  const bool live = c0 < N;  // N % 4 == 0: a lane's 4 columns are all live or all dead
  const int64_t rows_per = (R + chunks - 1) / chunks;
  const int64_t r0 = chunk * rows_per;
  const int64_t r1 = r0 + rows_per < R ? r0 + rows_per : R;
  const int64_t step = 4 * RP;  // rows per block-wide sweep (4 waves x RP rows)

  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t wpr = N / 32;                       // MB: mask words per row
  const int msh = static_cast<int>(c0 & 31);        // MB: this lane's 4 bits in its word
  auto mask4 = [&](float4& a, int64_t r) {
    const uint32_t w = mbits[r * wpr + (c0 >> 5)] >> msh;
    a.x = (w & 1u) ? a.x : 0.f; a.y = (w & 2u) ? a.y : 0.f;
    a.z = (w & 4u) ? a.z : 0.f; a.w = (w & 8u) ? a.w : 0.f;
  };
  if (live) {
    int64_t r = r0 + wv * RP + lrow;
    // two rows in flight per lane and iteration
    for (; r + step < r1; r += 2 * step) {
      float4 a = *reinterpret_cast<const float4*>(g + r * N + c0);
      float4 b = *reinterpret_cast<const float4*>(g + (r + step) * N + c0);
      if constexpr (MB) {
        mask4(a, r);
        mask4(b, r + step);
        *reinterpret_cast<float4*>(gp + r * N + c0) = a;
        *reinterpret_cast<float4*>(gp + (r + step) * N + c0) = b;
      } else if (RELU) {
        const float4 oa = *reinterpret_cast<const float4*>(out + r * N + c0);
        const float4 ob = *reinterpret_cast<const float4*>(out + (r + step) * N + c0);
        a.x = oa.x <= 0.f ? 0.f : a.x; a.y = oa.y <= 0.f ? 0.f : a.y;
        a.z = oa.z <= 0.f ? 0.f : a.z; a.w = oa.w <= 0.f ? 0.f : a.w;
        b.x = ob.x <= 0.f ? 0.f : b.x; b.y = ob.y <= 0.f ? 0.f : b.y;
        b.z = ob.z <= 0.f ? 0.f : b.z; b.w = ob.w <= 0.f ? 0.f : b.w;
        *reinterpret_cast<float4*>(gp + r * N + c0) = a;
        *reinterpret_cast<float4*>(gp + (r + step) * N + c0) = b;
      }
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
      acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
    }
    for (; r < r1; r += step) {
      float4 a = *reinterpret_cast<const float4*>(g + r * N + c0);
      if constexpr (MB) {
        mask4(a, r);
        *reinterpret_cast<float4*>(gp + r * N + c0) = a;
      } else if (RELU) {
        const float4 oa = *reinterpret_cast<const float4*>(out + r * N + c0);
        a.x = oa.x <= 0.f ? 0.f : a.x; a.y = oa.y <= 0.f ? 0.f : a.y;
        a.z = oa.z <= 0.f ? 0.f : a.z; a.w = oa.w <= 0.f ? 0.f : a.w;
        *reinterpret_cast<float4*>(gp + r * N + c0) = a;
      }
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
  }
  red[wv][lane] = acc;
  __syncthreads();
  // column j of the stripe: waves in order, then the RP row-lanes of its lane column in order
  const int j = threadIdx.x;
  const int64_t col = static_cast<int64_t>(stripe) * SW + j;
  const bool mine = j < SW && col < N;
  if (mine) {
    const int jc = j >> 2, comp = j & 3;
    float s = 0.f;
    for (int w = 0; w < 4; ++w)
      for (int q = 0; q < RP; ++q) {
        const float4 v = red[w][q * L + jc];
        s += comp == 0 ? v.x : comp == 1 ? v.y : comp == 2 ? v.z : v.w;
      }
    if (TAIL)
      __hip_atomic_store(&partials[static_cast<int64_t>(chunk) * N + col], s, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else
      partials[static_cast<int64_t>(chunk) * N + col] = s;
  }
  if (!TAIL) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ticket = tickets + stripe * 32;
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == static_cast<unsigned>(chunks - 1);
  }
  __syncthreads();
  if (!s_last) return;
  // the 256 threads as 256/SW groups of the stripe's SW columns: group gi sums chunks
  // [gi*cpg, (gi+1)*cpg) of its column in chunk order (32 loads in flight per batch), then the
  // groups' sums are added in group order -- a fixed order, so db is deterministic
  {
    const int NG = 256 / SW;
    const int jj = threadIdx.x % SW, gi = threadIdx.x / SW;
    const int64_t colj = static_cast<int64_t>(stripe) * SW + jj;
    const int cpg = (chunks + NG - 1) / NG;
    const int cb = gi * cpg;
    const int ce = cb + cpg < chunks ? cb + cpg : chunks;
    float s = 0.f;
    if (colj < N) {
      for (int c = cb; c < ce; c += 32) {
        float v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k)
          v[k] = c + k < ce ? __hip_atomic_load(&partials[static_cast<int64_t>(c + k) * N + colj],
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : 0.f;
#pragma unroll
        for (int k = 0; k < 32; ++k) s += v[k];
      }
    }
    tail[threadIdx.x] = s;
    __syncthreads();
    if (gi == 0 && colj < N) {
      float t = tail[jj];
      for (int g2 = 1; g2 < NG; ++g2) t += tail[g2 * SW + jj];
      db[colj] = t;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ocppo

using namespace ocppo;

extern "C" size_t ocppo_relu_bias_grad_workspace_bytes(int64_t R, int64_t N) {
  if (R < 1 || N < 1) return kRbTicketBytes;
  return kRbTicketBytes + static_cast<size_t>(rb_plan(R, N).chunks) * N * sizeof(float);
}

extern "C" int ocppo_relu_bias_grad(ocppo_stream_t stream, const float* g, const float* out,
                                    float* gp, float* db, int64_t R, int64_t N, void* workspace,
                                    size_t workspace_bytes) {
  OCPPO_REQUIRE(R >= 0 && N >= 4 && N % 4 == 0 && N <= kRbMaxStripes * 256,
                "ocppo_relu_bias_grad: bad sizes R=%lld N=%lld (N %% 4 == 0, 4 <= N <= 16384)",
                (long long)R, (long long)N);
  OCPPO_REQUIRE(g && db && workspace && (!out || gp), "ocppo_relu_bias_grad: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                    (!out || (reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                              reinterpret_cast<uintptr_t>(gp) % 16 == 0)) &&
                    reinterpret_cast<uintptr_t>(workspace) % 256 == 0,
                "ocppo_relu_bias_grad: g/out/gp must be 16-B aligned, workspace 256-B aligned");
  OCPPO_REQUIRE(workspace_bytes >= ocppo_relu_bias_grad_workspace_bytes(R, N),
                "ocppo_relu_bias_grad: workspace too small (%zu < %zu)", workspace_bytes,
                ocppo_relu_bias_grad_workspace_bytes(R, N));
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (R == 0) {
    (void)hipMemsetAsync(db, 0, N * sizeof(float), s);
    return check_launch("ocppo_relu_bias_grad");
  }
  const RbPlan p = rb_plan(R, N);
  unsigned* tickets = static_cast<unsigned*>(workspace);
  float* partials = reinterpret_cast<float*>(static_cast<char*>(workspace) + kRbTicketBytes);
  const dim3 grid(static_cast<unsigned>(p.stripes * p.chunks)), block(256);
  if (out)
    hipLaunchKernelGGL(relu_bias_grad_kernel<true>, grid, block, 0, s, g, out, gp, db, R, N,
                       p.L, p.chunks, tickets, partials);
  else
    hipLaunchKernelGGL(relu_bias_grad_kernel<false>, grid, block, 0, s, g, out, gp, db, R, N,
                       p.L, p.chunks, tickets, partials);
  return check_launch("ocppo_relu_bias_grad");
}

extern "C" int ocppo_relu_bias_grad_bits(ocppo_stream_t stream, const float* g,
                                         const uint32_t* mbits, float* gp, float* db, int64_t R,
                                         int64_t N, void* workspace, size_t workspace_bytes) {
  OCPPO_REQUIRE(R >= 1 && N >= 32 && N % 32 == 0 && N <= kRbMaxStripes * 256,
                "ocppo_relu_bias_grad_bits: bad sizes R=%lld N=%lld (N %% 32 == 0, 32 <= N <= "
                "16384)", (long long)R, (long long)N);
  OCPPO_REQUIRE(g && mbits && gp && db && workspace, "ocppo_relu_bias_grad_bits: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(gp) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(mbits) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(workspace) % 256 == 0,
                "ocppo_relu_bias_grad_bits: g/gp 16-B aligned, mbits 4-B, workspace 256-B");
  OCPPO_REQUIRE(workspace_bytes >= ocppo_relu_bias_grad_workspace_bytes(R, N),
                "ocppo_relu_bias_grad_bits: workspace too small (%zu < %zu)", workspace_bytes,
                ocppo_relu_bias_grad_workspace_bytes(R, N));
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const RbPlan p = rb_plan(R, N);
  unsigned* tickets = static_cast<unsigned*>(workspace);
  float* partials = reinterpret_cast<float*>(static_cast<char*>(workspace) + kRbTicketBytes);
  const dim3 grid(static_cast<unsigned>(p.stripes * p.chunks)), block(256);
  hipLaunchKernelGGL((relu_bias_grad_kernel<true, true, true>), grid, block, 0, s, g, nullptr, gp,
                     db, R, N, p.L, p.chunks, tickets, partials, mbits);
  return check_launch("ocppo_relu_bias_grad_bits");
}

extern "C" int64_t ocppo_relu_bias_grad_chunks(int64_t R, int64_t N) {
  if (R < 1 || N < 4) return 1;
  return rb_plan(R, N).chunks;
}

extern "C" int ocppo_relu_bias_grad_partial(ocppo_stream_t stream, const float* g,
                                            const float* out, float* gp, float* partials,
                                            int64_t R, int64_t N) {
  OCPPO_REQUIRE(R >= 1 && N >= 4 && N % 4 == 0 && N <= kRbMaxStripes * 256,
                "ocppo_relu_bias_grad_partial: bad sizes R=%lld N=%lld (R >= 1, N %% 4 == 0, "
                "4 <= N <= 16384)", (long long)R, (long long)N);
  OCPPO_REQUIRE(g && partials && (!out || gp), "ocppo_relu_bias_grad_partial: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                    (!out || (reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                              reinterpret_cast<uintptr_t>(gp) % 16 == 0)),
                "ocppo_relu_bias_grad_partial: g/out/gp must be 16-B aligned");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const RbPlan p = rb_plan(R, N);
  const dim3 grid(static_cast<unsigned>(p.stripes * p.chunks)), block(256);
  if (out)
    hipLaunchKernelGGL((relu_bias_grad_kernel<true, false>), grid, block, 0, s, g, out, gp,
                       nullptr, R, N, p.L, p.chunks, nullptr, partials);
  else
    hipLaunchKernelGGL((relu_bias_grad_kernel<false, false>), grid, block, 0, s, g, out, gp,
                       nullptr, R, N, p.L, p.chunks, nullptr, partials);
  return check_launch("ocppo_relu_bias_grad_partial");
}

// ---- forward epilogue: y = act(y + b) in place over [R, N] rows (e.g. an NHWC convolution
// output, N = channels), the bias add + ReLU ATen runs as two passes after a bias-less conv.
namespace ocppo {
template <bool RELU>
__global__ __launch_bounds__(256) void bias_act_kernel(float* __restrict__ y,
                                                       const float* __restrict__ b, int64_t R,
                                                       int64_t N) {
  const int64_t groups = R * (N / 4);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; q < groups;
       q += stride) {
    const int64_t c = (q % (N / 4)) * 4;
    float4 v = reinterpret_cast<float4*>(y)[q];
    const float4 bb = *reinterpret_cast<const float4*>(b + c);
    v.x = v.x + bb.x; v.y = v.y + bb.y; v.z = v.z + bb.z; v.w = v.w + bb.w;
    if (RELU) {
      v = relu_f4(v);
    }
    reinterpret_cast<float4*>(y)[q] = v;
  }
}
}  // namespace ocppo

extern "C" int ocppo_bias_act(ocppo_stream_t stream, float* y, const float* b, int64_t R,
                              int64_t N, int relu) {
  OCPPO_REQUIRE(R >= 0 && N >= 4 && N % 4 == 0, "ocppo_bias_act: bad sizes R=%lld N=%lld",
                (long long)R, (long long)N);
  if (R == 0) return OCPPO_OK;
  OCPPO_REQUIRE(y && b, "ocppo_bias_act: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(y) % 16 == 0 && reinterpret_cast<uintptr_t>(b) % 16 == 0,
                "ocppo_bias_act: y and b must be 16-B aligned");
  clear_stale_error();
  const dim3 grid(grid_for(R * (N / 4), 256)), block(256);
  if (relu)
    hipLaunchKernelGGL(bias_act_kernel<true>, grid, block, 0, as_stream(stream), y, b, R, N);
  else
    hipLaunchKernelGGL(bias_act_kernel<false>, grid, block, 0, as_stream(stream), y, b, R, N);
  return check_launch("ocppo_bias_act");
}

// ---- the same epilogue written out in NCHW order: out[b, c, p] = act(y[b, p, c] + bias[c]) for an
// NHWC convolution output y [B, P, C] (P = H*W) whose consumer flattens in NCHW order (nn.Flatten
// before a Linear): one image per workgroup through LDS (row stride C + 1: conflict-free reads
// down a channel), coalesced reads of y and writes of out -- the layout copy rides in the pass.
namespace ocppo {
constexpr int kBaNchwMaxElems = 12288;  // P * (C + 1) floats of LDS (48 KB)

template <bool RELU>
__global__ __launch_bounds__(256) void bias_act_nchw_kernel(const float* __restrict__ y,
                                                            const float* __restrict__ bias,
                                                            int P, int C,
                                                            float* __restrict__ out) {
  extern __shared__ float tile[];
  const int64_t img = blockIdx.x;
  const float* src = y + img * P * C;
  float* dst = out + img * P * C;
  const int ld = C + 1;
  for (int i = threadIdx.x; i < P * C; i += 256) {
    const int p = i / C, c = i - p * C;
    tile[p * ld + c] = src[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < P * C; i += 256) {
    const int c = i / P, p = i - c * P;
    float v = tile[p * ld + c] + bias[c];
    if (RELU) v = relu_f(v);
    dst[i] = v;
  }
}
}  // namespace ocppo

extern "C" int ocppo_bias_act_nchw(ocppo_stream_t stream, const float* y, const float* b,
                                   int64_t B, int64_t P, int64_t C, int relu, float* out) {
  OCPPO_REQUIRE(B >= 0 && P >= 1 && C >= 1 && P * (C + 1) <= ocppo::kBaNchwMaxElems &&
                    B <= INT32_MAX,
                "ocppo_bias_act_nchw: bad sizes B=%lld P=%lld C=%lld (P * (C + 1) <= %d)",
                (long long)B, (long long)P, (long long)C, ocppo::kBaNchwMaxElems);
  if (B == 0) return OCPPO_OK;
  OCPPO_REQUIRE(y && b && out, "ocppo_bias_act_nchw: null pointer");
  OCPPO_REQUIRE(y != out, "ocppo_bias_act_nchw: out must not alias y");
  clear_stale_error();
  const dim3 grid(static_cast<unsigned>(B)), block(256);
  const size_t lds = static_cast<size_t>(P) * (C + 1) * sizeof(float);
  if (relu)
    hipLaunchKernelGGL(ocppo::bias_act_nchw_kernel<true>, grid, block, lds, as_stream(stream), y,
                       b, (int)P, (int)C, out);
  else
    hipLaunchKernelGGL(ocppo::bias_act_nchw_kernel<false>, grid, block, lds, as_stream(stream),
                       y, b, (int)P, (int)C, out);
  return check_launch("ocppo_bias_act_nchw");
}

// ---- split-K combine of a weight gradient: out[i] = part[0][i] + part[1][i] + ... (split order,
// added in float64 and rounded once, as in sum_splits_db_kernel below)
// The update's tall-skinny weight-gradient GEMMs dW = g'^T x (inside loss.backward(),
// ppo_atari_oc.py:605, for the PPObj Linear layers of architectures/ppo.py:60-84) run as a
// batched GEMM over S row chunks; this sums the S partial [n] blocks straight into the
// parameter's slot of the flat grad buffer in one streaming pass (S loads of 16 B in flight per
// lane), where ATen's sum(0) kernel runs at ~1.5-3 TB/s on these shapes.
// Roofline: HBM / Infinity-Cache stream, (S + 1) * 4 B per output element.
namespace ocppo {
template <int S>
__global__ __launch_bounds__(256) void sum_splits_kernel(const float4* __restrict__ part,
                                                         int64_t n4, float4* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    float4 v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = part[s * n4 + i];
    double ax = v[0].x, ay = v[0].y, az = v[0].z, aw = v[0].w;  // f64 fold, one rounding
#pragma unroll
    for (int s = 1; s < S; ++s) {
      ax += v[s].x; ay += v[s].y; az += v[s].z; aw += v[s].w;
    }
    out[i] = make_float4(static_cast<float>(ax), static_cast<float>(ay), static_cast<float>(az),
                         static_cast<float>(aw));
  }
}
}  // namespace ocppo

// The deferred bias gradient of ocppo_relu_bias_grad_partial, summed in the same launch as the
// weight gradient's split-K combine: blocks [0, nsb) combine the weight splits, blocks
// [nsb, nsb + ceil(N / 16)) each own 16 columns of db: 4 column quads x 64 chunk groups, each
// thread summing its chunks in order, then the 64 group sums by a fixed butterfly inside each
// wave and the 4 wave sums in order: one pass, deterministic. (16 columns per block: the frame scatter's 720 chunk partials at [11520 x 512]
// take two load batches per thread instead of six.) Both folds add in float64 and round once:
// a bias gradient is a column sum over ~10^4 rows with heavy cancellation, and a left fold of
// 90-720 f32 partials rounded at every step cost it up to 1.6e-4 of its largest element against
// the reference's own 2e-5 (tests/test_config2_golden_gpu.py, against the f64 twin); the split
// combine of the weight gradient likewise (S <= 16 adds per element; HBM-bound either way).
constexpr int kDbQuads = 4;
constexpr int kDbGroups = 64;
struct d4 {
  double x, y, z, w;
};
template <int S>
__device__ __forceinline__ void sum_splits_db_block(const float4* __restrict__ part, int64_t n4,
                                                    float4* __restrict__ out, int nsb,
                                                    const float* __restrict__ dbp, int chunks,
                                                    int64_t N, float* __restrict__ db, int blk) {
  if (blk < nsb) {
    const int64_t stride = static_cast<int64_t>(nsb) * blockDim.x;
    for (int64_t i = static_cast<int64_t>(blk) * blockDim.x + threadIdx.x; i < n4;
         i += stride) {
      float4 v[S];
#pragma unroll
      for (int s = 0; s < S; ++s) v[s] = part[s * n4 + i];
      double ax = v[0].x, ay = v[0].y, az = v[0].z, aw = v[0].w;
#pragma unroll
      for (int s = 1; s < S; ++s) {
        ax += v[s].x; ay += v[s].y; az += v[s].z; aw += v[s].w;
      }
      out[i] = make_float4(static_cast<float>(ax), static_cast<float>(ay),
                           static_cast<float>(az), static_cast<float>(aw));
    }
    return;
  }
  __shared__ d4 red[256 / kWave][kDbQuads];
  const int cb = blk - nsb;
  const int q = threadIdx.x % kDbQuads, gi = threadIdx.x / kDbQuads;  // column quad, chunk group
  const int64_t col = static_cast<int64_t>(cb) * (4 * kDbQuads) + 4 * q;
  const int cpg = (chunks + kDbGroups - 1) / kDbGroups;
  const int c0 = gi * cpg, c1 = c0 + cpg < chunks ? c0 + cpg : chunks;
  d4 acc{0.0, 0.0, 0.0, 0.0};
  if (col < N) {
    for (int c = c0; c < c1; c += 8) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[k] = c + k < c1 ? *reinterpret_cast<const float4*>(dbp + (c + k) * N + col)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
      }
    }
  }
  // the 16 chunk groups of a wave (lanes 4 apart) by a butterfly, then the 4 waves in order
#pragma unroll
  for (int o = kDbQuads; o < kWave; o *= 2) {
    acc.x += __shfl_xor(acc.x, o); acc.y += __shfl_xor(acc.y, o);
    acc.z += __shfl_xor(acc.z, o); acc.w += __shfl_xor(acc.w, o);
  }
  const int wid = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) < kDbQuads) red[wid][q] = acc;
  __syncthreads();
  if (threadIdx.x < kDbQuads && col < N) {
    d4 t = red[0][q];
    for (int k = 1; k < 256 / kWave; ++k) {
      const d4 v = red[k][q];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    *reinterpret_cast<float4*>(db + col) =
        make_float4(static_cast<float>(t.x), static_cast<float>(t.y), static_cast<float>(t.z),
                    static_cast<float>(t.w));
  }
}

template <int S>
__global__ __launch_bounds__(256) void sum_splits_db_kernel(const float4* __restrict__ part,
                                                            int64_t n4, float4* __restrict__ out,
                                                            int nsb, const float* __restrict__ dbp,
                                                            int chunks, int64_t N,
                                                            float* __restrict__ db) {
  sum_splits_db_block<S>(part, n4, out, nsb, dbp, chunks, N, db, blockIdx.x);
}

extern "C" int ocppo_sum_splits_db(ocppo_stream_t stream, const float* part, int64_t S, int64_t n,
                                   float* out, const float* db_partials, int64_t chunks, int64_t N,
                                   float* db) {
  OCPPO_REQUIRE(n >= 4 && n % 4 == 0 && (S == 1 || S == 2 || S == 4 || S == 8 || S == 16) &&
                    N >= 4 && N % 4 == 0 && chunks >= 1,
                "ocppo_sum_splits_db: bad sizes S=%lld n=%lld N=%lld chunks=%lld", (long long)S,
                (long long)n, (long long)N, (long long)chunks);
  OCPPO_REQUIRE(part && out && db_partials && db, "ocppo_sum_splits_db: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(part) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(db_partials) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(db) % 16 == 0,
                "ocppo_sum_splits_db: pointers must be 16-B aligned");
  clear_stale_error();
  const int64_t n4 = n / 4;
  const int nsb = grid_for(n4, 256);
  const int ndb = static_cast<int>((N + 4 * kDbQuads - 1) / (4 * kDbQuads));
  const dim3 grid(nsb + ndb), block(256);
  hipStream_t s = as_stream(stream);
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int c = static_cast<int>(chunks);
  switch (S) {
    case 1: hipLaunchKernelGGL(sum_splits_db_kernel<1>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db); break;
    case 2: hipLaunchKernelGGL(sum_splits_db_kernel<2>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db); break;
    case 4: hipLaunchKernelGGL(sum_splits_db_kernel<4>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db); break;
    case 8: hipLaunchKernelGGL(sum_splits_db_kernel<8>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db); break;
    default: hipLaunchKernelGGL(sum_splits_db_kernel<16>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db); break;
  }
  return check_launch("ocppo_sum_splits_db");
}

extern "C" int ocppo_sum_splits(ocppo_stream_t stream, const float* part, int64_t S, int64_t n,
                                float* out) {
  OCPPO_REQUIRE(n >= 0 && n % 4 == 0 && (S == 1 || S == 2 || S == 4 || S == 8 || S == 16),
                "ocppo_sum_splits: bad sizes S=%lld n=%lld (S in {1,2,4,8,16}, n %% 4 == 0)",
                (long long)S, (long long)n);
  if (n == 0) return OCPPO_OK;
  OCPPO_REQUIRE(part && out, "ocppo_sum_splits: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(part) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out) % 16 == 0,
                "ocppo_sum_splits: part and out must be 16-B aligned");
  clear_stale_error();
  const int64_t n4 = n / 4;
  const dim3 grid(grid_for(n4, 256)), block(256);
  hipStream_t s = as_stream(stream);
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4* o4 = reinterpret_cast<float4*>(out);
  switch (S) {
    case 1: hipLaunchKernelGGL(sum_splits_kernel<1>, grid, block, 0, s, p4, n4, o4); break;
    case 2: hipLaunchKernelGGL(sum_splits_kernel<2>, grid, block, 0, s, p4, n4, o4); break;
    case 4: hipLaunchKernelGGL(sum_splits_kernel<4>, grid, block, 0, s, p4, n4, o4); break;
    case 8: hipLaunchKernelGGL(sum_splits_kernel<8>, grid, block, 0, s, p4, n4, o4); break;
    default: hipLaunchKernelGGL(sum_splits_kernel<16>, grid, block, 0, s, p4, n4, o4); break;
  }
  return check_launch("ocppo_sum_splits");
}

// ---- split-K combine of a forward product with its epilogue: out[m, n] = act(sum_s part[s, m, n]
// + bias[n]) (the S partials added in split order in float64, rounded once, then torch's
// _addmm_activation order: + bias, then ReLU). The update's decoder forward [4096 x 512] from
// K = 2048 (architectures/ppo.py:77-80) has 128 output tiles: gemm_x6 runs it as 4 K splits of 128
// tiles each (512 workgroups) and this pass finishes it. Roofline: HBM stream, (S + 1) * 4 B per
// output element.
namespace ocppo {
template <int S>
__global__ __launch_bounds__(256) void sum_splits_act_kernel(const float4* __restrict__ part,
                                                             int64_t n4, int64_t N4,
                                                             const float4* __restrict__ bias,
                                                             int relu, float4* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4;
       i += stride) {
    float4 v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) v[s] = part[s * n4 + i];
    double ax = v[0].x, ay = v[0].y, az = v[0].z, aw = v[0].w;
#pragma unroll
    for (int s = 1; s < S; ++s) {
      ax += v[s].x; ay += v[s].y; az += v[s].z; aw += v[s].w;
    }
    float4 r = make_float4(static_cast<float>(ax), static_cast<float>(ay),
                           static_cast<float>(az), static_cast<float>(aw));
    if (bias) {
      const float4 b = bias[i % N4];
      r.x += b.x; r.y += b.y; r.z += b.z; r.w += b.w;
    }
    if (relu) {
      r = relu_f4(r);
    }
    out[i] = r;
  }
}
}  // namespace ocppo

extern "C" int ocppo_sum_splits_act(ocppo_stream_t stream, const float* part, int64_t S,
                                    int64_t M, int64_t N, const float* bias, int relu,
                                    float* out) {
  OCPPO_REQUIRE(M >= 0 && N >= 4 && N % 4 == 0 && (S == 1 || S == 2 || S == 4 || S == 8 || S == 16),
                "ocppo_sum_splits_act: bad sizes S=%lld M=%lld N=%lld (S in {1,2,4,8,16}, "
                "N %% 4 == 0)", (long long)S, (long long)M, (long long)N);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(part && out, "ocppo_sum_splits_act: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(part) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(out) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(bias) % 16 == 0,
                "ocppo_sum_splits_act: part, out and bias must be 16-B aligned");
  clear_stale_error();
  const int64_t n4 = M * N / 4;
  const dim3 grid(grid_for(n4, 256)), block(256);
  hipStream_t s = as_stream(stream);
  const float4* p4 = reinterpret_cast<const float4*>(part);
  const float4* b4 = reinterpret_cast<const float4*>(bias);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int r = relu ? 1 : 0;
  switch (S) {
    case 1: hipLaunchKernelGGL(sum_splits_act_kernel<1>, grid, block, 0, s, p4, n4, N / 4, b4, r, o4); break;
    case 2: hipLaunchKernelGGL(sum_splits_act_kernel<2>, grid, block, 0, s, p4, n4, N / 4, b4, r, o4); break;
    case 4: hipLaunchKernelGGL(sum_splits_act_kernel<4>, grid, block, 0, s, p4, n4, N / 4, b4, r, o4); break;
    case 8: hipLaunchKernelGGL(sum_splits_act_kernel<8>, grid, block, 0, s, p4, n4, N / 4, b4, r, o4); break;
    default: hipLaunchKernelGGL(sum_splits_act_kernel<16>, grid, block, 0, s, p4, n4, N / 4, b4, r, o4); break;
  }
  return check_launch("ocppo_sum_splits_act");
}

// ---- first-layer backward in ONE pass: ReLU-backward + bias gradient + weight gradient -----------
// For a Linear(+ReLU) layer whose input needs no gradient and has few features (the PPObj
// encoder's first layer on the object frames, F = 6 / 12 -> 256, architectures/ppo.py:60-84,
// inside loss.backward() of ppo_atari_oc.py:605) the elementwise pass and the weight-gradient GEMM
// read the same rows, and gp is consumed by nothing else:
//   gp[r, n] = out[r, n] <= 0 ? 0 : g[r, n]      (never written)
//   db[n]    = sum_r gp[r, n]
//   dw[n, k] = sum_r gp[r, n] * x[r, k]           (k < K <= 16)
// Autograd runs threshold_backward (writes gp), a split-K GEMM over gp (a long K = R reduction
// into a tiny [N, K] output: ~3 TFLOP/s) and a sum: 3 launches, gp written and read back. Here a
// workgroup (stripe, chunk) owns 4L columns x a row range, each lane keeps 4 columns x (K + 1)
// running sums (fmaf, rows in a fixed order), waves and row-lanes are combined through LDS in a
// fixed order, partials published with sc1 stores, and the stripe's last arriver (ticket per
// stripe, re-arming) sums the chunks in chunk order: deterministic, no data atomics.
// Roofline: HBM stream, 8 B (relu; 4 B without) per element of g + 4K B per row of x.
namespace ocppo {

constexpr int kWgL = 8;  // lanes per row: 32-column stripes (whole 128-B lines), 8 rows per instruction
constexpr int kWgMaxChunks = 64;
constexpr int kWgMaxStripes = 512;  // N <= 16384
constexpr size_t kWgTicketBytes = kWgMaxStripes * 128;

inline int wg_chunks(int64_t R, int64_t N) {
  const int64_t stripes = (N + 4 * kWgL - 1) / (4 * kWgL);
  int64_t c = (512 + stripes - 1) / stripes;  // ~512 workgroups
  if (c > kWgMaxChunks) c = kWgMaxChunks;
  const int64_t by_rows = (R + 63) / 64;      // >= 64 rows per chunk
  if (c > by_rows) c = by_rows;
  return static_cast<int>(c < 1 ? 1 : c);
}

// Row-major form: a workgroup owns a contiguous range of rows x 256 columns (lane = 4 adjacent
// columns, 16-B loads; the waves take every kWrWaves-th row), so every row of x is read once per
// column group, out of LDS (staged kWrStage rows at a time). Each lane keeps 4 columns x (K + 1)
// running sums (fmaf, rows in order). Fixed grid (round 3): wr_layout picks about 128 row
// ranges per column group, so the records -- ONE per workgroup, the waves combined through LDS
// in wave order -- are O(grid), not O(R / 64); a second launch adds them with a fixed-shape tree
// (relu_bias_wgrad_finish_kernel). Deterministic, no atomics.
#ifndef OCPPO_WR_WAVES  // experiments (tools/build_variant.py) move these
#define OCPPO_WR_WAVES 8
#endif
#ifndef OCPPO_WR_GRID
#define OCPPO_WR_GRID 256
#endif
constexpr int kWrCols = kWgRecCols;  // columns per workgroup (64 lanes x 4)
constexpr int kWrWaves = OCPPO_WR_WAVES;  // 2 waves per SIMD: enough loads in flight per CU
constexpr int kWrU = 8;            // rows in flight per wave
constexpr int kWrStage = 128;      // rows of x staged in LDS at a time
constexpr int kWrGrid = OCPPO_WR_GRID;  // row ranges per column group (at most)

// rows per workgroup: a multiple of the wave count, >= 32
inline int64_t wr_rows_per_wg(int64_t R) {
  int64_t rpw = (R + kWrGrid - 1) / kWrGrid;
  if (rpw < 32) rpw = 32;
  return (rpw + kWrWaves - 1) / kWrWaves * kWrWaves;
}

template <bool RELU, int KP>
__global__ __launch_bounds__(64 * kWrWaves) void relu_bias_wgrad_rows_kernel(
    const float* __restrict__ g, const float* __restrict__ out, const float* __restrict__ x,
    int64_t ldx, int64_t R, int64_t N, int K, int64_t rows_per_wg, float* __restrict__ partials) {
  constexpr int NV = KP + 1;
  // per wave an image [NV][256 columns]: a lane's 4 columns of one value are one float4, so
  // consecutive lanes store / load consecutive 16 B (no bank conflicts)
  extern __shared__ __attribute__((aligned(16))) float wr_red[];  // [waves][NV][256]
  __shared__ float xs[kWrStage][KP];                               // staged rows of x
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int cg = blockIdx.y;
  const int64_t c0 = static_cast<int64_t>(cg) * kWrCols + 4 * lane;
  const bool live = c0 < N;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_wg;
  const int64_t r1 = r0 + rows_per_wg < R ? r0 + rows_per_wg : R;
  float sb[4] = {0.f, 0.f, 0.f, 0.f};
  float sw[4][KP];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < KP; ++k) sw[j][k] = 0.f;
  for (int64_t s0 = r0; s0 < r1; s0 += kWrStage) {  // block-uniform trip count
    const int64_t s1 = s0 + kWrStage < r1 ? s0 + kWrStage : r1;
    __syncthreads();  // the previous stage's rows are consumed
    for (int i = threadIdx.x; i < kWrStage * KP; i += 64 * kWrWaves) {
      const int rr = i / KP, k = i - rr * KP;
      xs[rr][k] = (s0 + rr < s1 && k < K) ? x[(s0 + rr) * ldx + k] : 0.f;
    }
    __syncthreads();
    for (int64_t rb = s0 + wv; rb < s1; rb += kWrWaves * kWrU) {
      float4 a[kWrU];
#pragma unroll
      for (int u = 0; u < kWrU; ++u) {
        const int64_t r = rb + kWrWaves * u;
        const bool ok = r < s1 && live;
        a[u] = ok ? *reinterpret_cast<const float4*>(g + r * N + c0)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (RELU) {
#pragma unroll
        for (int u = 0; u < kWrU; ++u) {
          const int64_t r = rb + kWrWaves * u;
          const float4 o = (r < s1 && live) ? *reinterpret_cast<const float4*>(out + r * N + c0)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
          a[u].x = o.x <= 0.f ? 0.f : a[u].x; a[u].y = o.y <= 0.f ? 0.f : a[u].y;
          a[u].z = o.z <= 0.f ? 0.f : a[u].z; a[u].w = o.w <= 0.f ? 0.f : a[u].w;
        }
      }
#pragma unroll
      for (int u = 0; u < kWrU; ++u) {
        const int64_t r = rb + kWrWaves * u;
        if (r >= s1) break;  // wave-uniform; rows past the stage carry zeros anyway
        const float* xr = xs[r - s0];
        const float av[4] = {a[u].x, a[u].y, a[u].z, a[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sb[j] += av[j];
#pragma unroll
          for (int k = 0; k < KP; ++k) sw[j][k] = fmaf(av[j], xr[k], sw[j][k]);
        }
      }
    }
  }
  float4* mine = reinterpret_cast<float4*>(wr_red) + static_cast<int64_t>(wv) * NV * 64 + lane;
  mine[0] = make_float4(sb[0], sb[1], sb[2], sb[3]);
#pragma unroll
  for (int k = 0; k < KP; ++k) mine[(1 + k) * 64] = make_float4(sw[0][k], sw[1][k], sw[2][k], sw[3][k]);
  __syncthreads();
  // record [NV][256 columns] of this (row range, column group), waves added in order
  constexpr int nrec4 = NV * 64;
  const float4* img = reinterpret_cast<const float4*>(wr_red);
  float4* rec = reinterpret_cast<float4*>(partials) +
                (static_cast<int64_t>(blockIdx.x) * gridDim.y + cg) * nrec4;
  for (int i = threadIdx.x; i < nrec4; i += 64 * kWrWaves) {
    float4 t = img[i];
#pragma unroll
    for (int q = 1; q < kWrWaves; ++q) {
      const float4 b = img[q * nrec4 + i];
      t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
    }
    rec[i] = t;
  }
}

// Adds the G records of every column group with a fixed-shape tree: a block owns 32 record
// entries x 8 record groups; group gi takes records gi, gi + 8, ... in batches of 32 loads in
// flight, each batch summed pairwise, then the 8 group sums pairwise through LDS.
// Output o = (column group, value v, column): v = 0 the bias gradient, 1..K the weight columns.
constexpr int kWfOut = 32, kWfGroups = 8, kWfBatch = 32;
// everything the finish needs, fixed at the rows launch (ocppo_relu_bias_wgrad_rows hands it to
// the caller as an ocppo_deferred_finish_t so it can ride in a later launch)
struct WgFinish {
  const float* partials;
  int G, NV, K, blocks;
  int64_t npw, N;
  float *dw, *db;
};
__device__ __forceinline__ void wg_finish_block(const WgFinish& f, int blk) {
  __shared__ float red[kWfGroups][kWfOut + 1];
  const int o = threadIdx.x % kWfOut, gi = threadIdx.x / kWfOut;
  const int64_t idx = static_cast<int64_t>(blk) * kWfOut + o;
  const float* __restrict__ partials = f.partials;
  const int G = f.G;
  const int64_t npw = f.npw;
  float s = 0.f;
  if (idx < npw) {
    for (int g0 = gi; g0 < G; g0 += kWfGroups * kWfBatch) {
      float v[kWfBatch];
#pragma unroll
      for (int u = 0; u < kWfBatch; ++u) {
        const int gg = g0 + u * kWfGroups;
        v[u] = gg < G ? partials[static_cast<int64_t>(gg) * npw + idx] : 0.f;
      }
#pragma unroll
      for (int wdt = kWfBatch / 2; wdt >= 1; wdt /= 2)
#pragma unroll
        for (int u = 0; u < wdt; ++u) v[u] += v[u + wdt];
      s += v[0];
    }
  }
  red[gi][o] = s;
  __syncthreads();
  for (int wdt = kWfGroups / 2; wdt >= 1; wdt /= 2) {
    if (gi < wdt) red[gi][o] += red[gi + wdt][o];
    __syncthreads();
  }
  if (gi != 0 || idx >= npw) return;
  const float t = red[0][o];
  const int64_t per = static_cast<int64_t>(kWrCols) * f.NV;
  const int64_t cgi = idx / per, rem = idx - cgi * per;
  const int v = static_cast<int>(rem / kWrCols);
  const int64_t col = cgi * kWrCols + (rem - static_cast<int64_t>(v) * kWrCols);
  if (col >= f.N) return;
  if (v == 0) f.db[col] = t;
  else if (v - 1 < f.K) f.dw[col * f.K + (v - 1)] = t;
}

__global__ __launch_bounds__(256) void relu_bias_wgrad_finish_kernel(WgFinish f) {
  wg_finish_block(f, blockIdx.x);
}

// the finish folded into a later split-K combine of the same backward (the second encoder
// layer's weight gradient, which runs after the first layer's rows when the trainer defers it):
// workgroups [0, f.blocks) finish, the rest are sum_splits_db's
template <int S>
__global__ __launch_bounds__(256) void sum_splits_db_wgfin_kernel(
    const float4* __restrict__ part, int64_t n4, float4* __restrict__ out, int nsb,
    const float* __restrict__ dbp, int chunks, int64_t N, float* __restrict__ db, WgFinish f) {
  if (static_cast<int>(blockIdx.x) < f.blocks) {
    wg_finish_block(f, blockIdx.x);
    return;
  }
  sum_splits_db_block<S>(part, n4, out, nsb, dbp, chunks, N, db, blockIdx.x - f.blocks);
}

template <bool RELU>
static WgFinish launch_wgrad_rows(hipStream_t s, int K, const float* g, const float* out,
                                  const float* x, int64_t ldx, float* dw, float* db, int64_t R,
                                  int64_t N, float* partials) {
  const int64_t rpw = wr_rows_per_wg(R);
  const int G = static_cast<int>((R + rpw - 1) / rpw);
  const int ncg = static_cast<int>((N + kWrCols - 1) / kWrCols);
  const dim3 grid(G, ncg), block(64 * kWrWaves);
  int KP = K <= 4 ? 4 : K <= 8 ? 8 : K <= 12 ? 12 : 16;
  const size_t lds = sizeof(float) * kWrWaves * kWrCols * (KP + 1);
#define OCPPO_WR(KP_)                                                                            \
  hipLaunchKernelGGL((relu_bias_wgrad_rows_kernel<RELU, KP_>), grid, block, lds, s, g, out, x,   \
                     ldx, R, N, K, rpw, partials)
  if (KP == 4) OCPPO_WR(4);
  else if (KP == 8) OCPPO_WR(8);
  else if (KP == 12) OCPPO_WR(12);
  else OCPPO_WR(16);
#undef OCPPO_WR
  const int64_t npw = static_cast<int64_t>(ncg) * kWrCols * (KP + 1);
  return WgFinish{partials, G, KP + 1, K, static_cast<int>((npw + kWfOut - 1) / kWfOut), npw, N,
                  dw, db};
}


}  // namespace ocppo

extern "C" size_t ocppo_relu_bias_wgrad_workspace_bytes(int64_t R, int64_t N, int64_t K) {
  if (R < 1 || N < 1 || K < 1) return 256;
  const int64_t rpw = ocppo::wr_rows_per_wg(R);
  const int64_t G = (R + rpw - 1) / rpw;
  const int64_t ncg = (N + ocppo::kWrCols - 1) / ocppo::kWrCols;
  return static_cast<size_t>(G * ncg * ocppo::kWrCols * (ocppo::wg_kp(K) + 1)) * sizeof(float);
}

static int relu_bias_wgrad_impl(ocppo_stream_t stream, const float* g, const float* out,
                                const float* x, int64_t ldx, float* dw, float* db, int64_t R,
                                int64_t N, int64_t K, void* workspace, size_t workspace_bytes,
                                WgFinish* fin_out) {
  OCPPO_REQUIRE(R >= 0 && N >= 4 && N % 4 == 0 && N <= 16384 && K >= 1 && K <= 16 && ldx >= K,
                "ocppo_relu_bias_wgrad: bad sizes R=%lld N=%lld K=%lld ldx=%lld (N %% 4 == 0, "
                "N <= 16384, 1 <= K <= 16, ldx >= K)", (long long)R, (long long)N, (long long)K,
                (long long)ldx);
  OCPPO_REQUIRE(dw && db && workspace, "ocppo_relu_bias_wgrad: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (R == 0) {  // empty batch: zero gradients (g / out / x may be NULL)
    (void)hipMemsetAsync(db, 0, N * sizeof(float), s);
    (void)hipMemsetAsync(dw, 0, N * K * sizeof(float), s);
    return check_launch("ocppo_relu_bias_wgrad");
  }
  OCPPO_REQUIRE(g && x, "ocppo_relu_bias_wgrad: null pointer");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(g) % 16 == 0 &&
                    (!out || reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                    reinterpret_cast<uintptr_t>(workspace) % 16 == 0,
                "ocppo_relu_bias_wgrad: g/out/workspace must be 16-B aligned");
  OCPPO_REQUIRE(workspace_bytes >= ocppo_relu_bias_wgrad_workspace_bytes(R, N, K),
                "ocppo_relu_bias_wgrad: workspace too small (%zu < %zu)", workspace_bytes,
                ocppo_relu_bias_wgrad_workspace_bytes(R, N, K));
  float* partials = static_cast<float*>(workspace);
  const WgFinish f = out ? launch_wgrad_rows<true>(s, (int)K, g, out, x, ldx, dw, db, R, N, partials)
                         : launch_wgrad_rows<false>(s, (int)K, g, out, x, ldx, dw, db, R, N, partials);
  if (int rc = check_launch("ocppo_relu_bias_wgrad")) return rc;
  if (fin_out) {
    *fin_out = f;
    return OCPPO_OK;
  }
  hipLaunchKernelGGL(relu_bias_wgrad_finish_kernel, dim3(f.blocks), dim3(256), 0, s, f);
  return check_launch("ocppo_relu_bias_wgrad/finish");
}

extern "C" int ocppo_relu_bias_wgrad(ocppo_stream_t stream, const float* g, const float* out,
                                     const float* x, int64_t ldx, float* dw, float* db, int64_t R,
                                     int64_t N, int64_t K, void* workspace,
                                     size_t workspace_bytes) {
  return relu_bias_wgrad_impl(stream, g, out, x, ldx, dw, db, R, N, K, workspace,
                              workspace_bytes, nullptr);
}

// the deferred-finish record behind the C-ABI's opaque ocppo_deferred_finish_t (heads-loss
// records carry another tag, ocppo_loss.hip)
constexpr uint64_t kDeferWgrad = 0x6f63707077676631ull;
struct DeferredWgrad {
  uint64_t tag;
  WgFinish f;
};
static_assert(sizeof(DeferredWgrad) <= sizeof(ocppo_deferred_finish_t),
              "ocppo_deferred_finish_t too small");

extern "C" int ocppo_relu_bias_wgrad_rows(ocppo_stream_t stream, const float* g, const float* out,
                                          const float* x, int64_t ldx, float* dw, float* db,
                                          int64_t R, int64_t N, int64_t K, void* workspace,
                                          size_t workspace_bytes,
                                          ocppo_deferred_finish_t* finish) {
  OCPPO_REQUIRE(finish && R >= 1, "ocppo_relu_bias_wgrad_rows: null finish record or R == 0");
  DeferredWgrad d;
  d.tag = kDeferWgrad;
  if (int rc = relu_bias_wgrad_impl(stream, g, out, x, ldx, dw, db, R, N, K, workspace,
                                    workspace_bytes, &d.f))
    return rc;
  memset(finish, 0, sizeof(*finish));
  memcpy(finish, &d, sizeof(d));
  return OCPPO_OK;
}

namespace ocppo {
// a relu_bias_wgrad finish record over G row-range records written by another kernel (gemm_x6's
// wgrad epilogue) in the same layout
void wgrad_record(ocppo_deferred_finish_t* out, const float* partials, int G, int64_t N, int K,
                  float* dw, float* db) {
  const int KP = wg_kp(K);
  const int64_t ncg = (N + kWrCols - 1) / kWrCols;
  const int64_t npw = ncg * kWrCols * (KP + 1);
  DeferredWgrad d;
  d.tag = kDeferWgrad;
  d.f = WgFinish{partials, G, KP + 1, K, static_cast<int>((npw + kWfOut - 1) / kWfOut), npw, N,
                 dw, db};
  memset(out, 0, sizeof(*out));
  memcpy(out, &d, sizeof(d));
}

// ocppo_deferred_finish_run for a relu_bias_wgrad record (1: done; 0: not such a record)
int wgrad_finish_run(hipStream_t s, const ocppo_deferred_finish_t* finish) {
  DeferredWgrad d;
  memcpy(&d, finish, sizeof(d));
  if (d.tag != kDeferWgrad) return 0;
  hipLaunchKernelGGL(relu_bias_wgrad_finish_kernel, dim3(d.f.blocks), dim3(256), 0, s, d.f);
  return 1;
}
}  // namespace ocppo

extern "C" int ocppo_sum_splits_db_finish(ocppo_stream_t stream, const float* part, int64_t S,
                                          int64_t n, float* out, const float* db_partials,
                                          int64_t chunks, int64_t N, float* db,
                                          const ocppo_deferred_finish_t* finish) {
  OCPPO_REQUIRE(n >= 4 && n % 4 == 0 && (S == 1 || S == 2 || S == 4 || S == 8 || S == 16) &&
                    N >= 4 && N % 4 == 0 && chunks >= 1,
                "ocppo_sum_splits_db_finish: bad sizes S=%lld n=%lld N=%lld chunks=%lld",
                (long long)S, (long long)n, (long long)N, (long long)chunks);
  OCPPO_REQUIRE(part && out && db_partials && db && finish,
                "ocppo_sum_splits_db_finish: null pointer");
  OCPPO_REQUIRE((reinterpret_cast<uintptr_t>(part) | reinterpret_cast<uintptr_t>(out) |
                 reinterpret_cast<uintptr_t>(db_partials) | reinterpret_cast<uintptr_t>(db)) % 16 == 0,
                "ocppo_sum_splits_db_finish: pointers must be 16-B aligned");
  DeferredWgrad d;
  memcpy(&d, finish, sizeof(d));
  OCPPO_REQUIRE(d.tag == kDeferWgrad,
                "ocppo_sum_splits_db_finish: not a finish record of ocppo_relu_bias_wgrad_rows");
  clear_stale_error();
  const int64_t n4 = n / 4;
  const int nsb = grid_for(n4, 256);
  const int ndb = static_cast<int>((N + 4 * kDbQuads - 1) / (4 * kDbQuads));
  const dim3 grid(d.f.blocks + nsb + ndb), block(256);
  hipStream_t s = as_stream(stream);
  const float4* p4 = reinterpret_cast<const float4*>(part);
  float4* o4 = reinterpret_cast<float4*>(out);
  const int c = static_cast<int>(chunks);
  switch (S) {
    case 1: hipLaunchKernelGGL(sum_splits_db_wgfin_kernel<1>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db, d.f); break;
    case 2: hipLaunchKernelGGL(sum_splits_db_wgfin_kernel<2>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db, d.f); break;
    case 4: hipLaunchKernelGGL(sum_splits_db_wgfin_kernel<4>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db, d.f); break;
    case 8: hipLaunchKernelGGL(sum_splits_db_wgfin_kernel<8>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db, d.f); break;
    default: hipLaunchKernelGGL(sum_splits_db_wgfin_kernel<16>, grid, block, 0, s, p4, n4, o4, nsb, db_partials, c, N, db, d.f); break;
  }
  return check_launch("ocppo_sum_splits_db_finish");
}

// ---- policy heads + decoder ReLU backward in ONE pass ---------------------------------------------
// The actor / critic heads (architectures/ppo.py:81-84: Linear(H, A), Linear(H, 1) on the decoder
// output h = relu(z)) get d loss / d logits [M, A] and d loss / d value [M] from the fused loss
// (ppo_atari_oc.py:581-605). Autograd then runs per head a dX GEMM (K = A), a split-K dW GEMM and
// a bias sum, adds the two dX, and the decoder's ReLU-backward + bias-grad pass: ~9 launches, dh
// written and read back. Here, with c[m] = (dlogits[m, 0..A), dv[m]) and W = [Wa; Wc] ([A+1, H]):
//   dh[m, j]  = sum_k c[m, k] W[k, j]                   (k order, fmaf)
//   gp[m, j]  = relu ? (h[m, j] <= 0 ? 0 : dh[m, j]) : dh[m, j]      (written once)
//   db_h[j]   = sum_m gp[m, j]                          (the decoder bias grad; optional)
//   dW[k, j]  = sum_m c[m, k] h[m, j]                   (dWa rows k < A, dWc row A)
//   dbk[k]    = sum_m c[m, k]                           (dba, dbc)
// Same launch structure as relu_bias_wgrad (32-column stripes x row chunks, fixed-order LDS
// combine, chunk-order tail by the stripe's last arriver); stripe 0 also carries dbk.
// Roofline: HBM stream, 8 B per element of h (h in, gp out) + 4(A+1) B per row.
namespace ocppo {

constexpr int kHbKP = 8;  // A + 1 <= 8

inline size_t hb_partials_per_chunk(int64_t H, int K) { return H * (K + 1) + K; }

template <bool RELU>
__global__ __launch_bounds__(256) void heads_bwd_kernel(
    const float* __restrict__ h, const float* __restrict__ dl, const float* __restrict__ dv,
    const float* __restrict__ wa, const float* __restrict__ wc, float* __restrict__ gp,
    float* __restrict__ dbh, float* __restrict__ dwa, float* __restrict__ dwc,
    float* __restrict__ dba, float* __restrict__ dbc, int64_t M, int64_t H, int A, int K, int chunks,
    unsigned* __restrict__ tickets, float* __restrict__ partials) {
  constexpr int L = kWgL, RP = 64 / L, SW = 4 * L, KP = kHbKP, NV = KP + 1;
  __shared__ float red[4 * RP][SW][NV + 1];
  __shared__ float redc[4 * RP][KP];
  __shared__ int s_last;
  // K = A + 1 with a critic row (dv, wc), K = A without (a single head, e.g. the DQN Q head)
  const int nstripes = static_cast<int>((H + SW - 1) / SW);
  const int stripe = blockIdx.x % nstripes;
  const int chunk = blockIdx.x / nstripes;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int lrow = lane / L, lcol = lane - lrow * L;
  const int64_t c0 = static_cast<int64_t>(stripe) * SW + 4 * lcol;
  const bool live = c0 < H;
  const int64_t rows_per = (M + chunks - 1) / chunks;
  const int64_t r0 = chunk * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  const int64_t step = 4 * RP;
  const int64_t ppc = static_cast<int64_t>(H) * (K + 1) + K;  // partials per chunk

  // this lane's 4 columns of W = [Wa; Wc]
  float wk[KP][4];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const float* wr = k < A ? wa + static_cast<int64_t>(k) * H : wc;
#pragma unroll
    for (int j = 0; j < 4; ++j) wk[k][j] = (live && k < K) ? wr[c0 + j] : 0.f;
  }
  float sb[4] = {0.f, 0.f, 0.f, 0.f};
  float sw[4][KP];
  float sc[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    sc[k] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) sw[j][k] = 0.f;
  }
  if (live) {
    constexpr int U = 3;
    for (int64_t rb = r0 + wv * RP + lrow; rb < r1; rb += U * step) {
      float4 hv[U];
      float cv[U][KP];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = rb + u * step;
        ok[u] = r < r1;
        const int64_t rr = ok[u] ? r : r0;
        hv[u] = *reinterpret_cast<const float4*>(h + rr * H + c0);
#pragma unroll
        for (int k = 0; k < KP; ++k)
          cv[u][k] = !ok[u] || k >= K ? 0.f : (k < A ? dl[rr * A + k] : dv[rr]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float hj[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w};
        float g4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float d = 0.f;
#pragma unroll
          for (int k = 0; k < KP; ++k) d = fmaf(cv[u][k], wk[k][j], d);
          g4[j] = (RELU && hj[j] <= 0.f) ? 0.f : d;
          sb[j] += g4[j];
#pragma unroll
          for (int k = 0; k < KP; ++k) sw[j][k] = fmaf(cv[u][k], hj[j], sw[j][k]);
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) sc[k] += cv[u][k];
        if (ok[u])
          *reinterpret_cast<float4*>(gp + (rb + u * step) * H + c0) =
              make_float4(g4[0], g4[1], g4[2], g4[3]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[wv * RP + lrow][4 * lcol + j][0] = sb[j];
#pragma unroll
    for (int k = 0; k < KP; ++k) red[wv * RP + lrow][4 * lcol + j][1 + k] = sw[j][k];
  }
  if (lcol == 0) {
#pragma unroll
    for (int k = 0; k < KP; ++k) redc[wv * RP + lrow][k] = live ? sc[k] : 0.f;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < SW * NV; q += 256) {
    const int j = q / NV, v = q - j * NV;
    const int64_t col = static_cast<int64_t>(stripe) * SW + j;
    if (col < H && v < K + 1) {
      float s = 0.f;
#pragma unroll 8
      for (int w = 0; w < 4 * RP; ++w) s += red[w][j][v];
      __hip_atomic_store(&partials[chunk * ppc + col * (K + 1) + v], s, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (stripe == 0 && threadIdx.x < K) {
    float s = 0.f;
    for (int w = 0; w < 4 * RP; ++w) s += redc[w][threadIdx.x];
    __hip_atomic_store(&partials[chunk * ppc + H * (K + 1) + threadIdx.x], s, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ticket = tickets + stripe * 32;
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == static_cast<unsigned>(chunks - 1);
  }
  __syncthreads();
  if (!s_last) return;
  const int nq = SW * (K + 1) + (stripe == 0 ? K : 0);
  for (int q = threadIdx.x; q < nq; q += 256) {
    int64_t idx;
    int j = 0, v = 0;
    const bool colv = q < SW * (K + 1);
    if (colv) {
      j = q / (K + 1);
      v = q - j * (K + 1);
      const int64_t col = static_cast<int64_t>(stripe) * SW + j;
      if (col >= H) continue;
      idx = col * (K + 1) + v;
    } else {
      idx = static_cast<int64_t>(H) * (K + 1) + (q - SW * (K + 1));
    }
    float s = 0.f;
    for (int c = 0; c < chunks; c += 32) {
      float t[32];
#pragma unroll
      for (int u = 0; u < 32; ++u)
        t[u] = c + u < chunks ? __hip_atomic_load(&partials[(c + u) * ppc + idx], __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : 0.f;
#pragma unroll
      for (int u = 0; u < 32; ++u) s += t[u];
    }
    if (colv) {
      const int64_t col = static_cast<int64_t>(stripe) * SW + j;
      if (v == 0) {
        if (dbh) dbh[col] = s;
      } else if (v - 1 < A) {
        dwa[static_cast<int64_t>(v - 1) * H + col] = s;
      } else {
        dwc[col] = s;
      }
    } else {
      const int k = q - SW * (K + 1);
      if (k < A) dba[k] = s;
      else dbc[0] = s;
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ocppo

extern "C" size_t ocppo_heads_bwd_workspace_bytes(int64_t M, int64_t H, int64_t A) {
  if (M < 1 || H < 1 || A < 1) return kWgTicketBytes;
  return kWgTicketBytes +
         static_cast<size_t>(wg_chunks(M, H)) * hb_partials_per_chunk(H, (int)A + 1) * sizeof(float);
}

extern "C" int ocppo_heads_bwd(ocppo_stream_t stream, const float* h, const float* dlogits,
                               const float* dvalue, const float* wa, const float* wc, float* gp,
                               float* db_h, float* dwa, float* dwc, float* dba, float* dbc,
                               int64_t M, int64_t H, int64_t A, int relu, void* workspace,
                               size_t workspace_bytes) {
  OCPPO_REQUIRE(M >= 1 && H >= 4 && H % 4 == 0 && H <= kWgMaxStripes * 4 * kWgL && A >= 1 &&
                    A + 1 <= kHbKP,
                "ocppo_heads_bwd: bad sizes M=%lld H=%lld A=%lld (M >= 1, H %% 4 == 0, "
                "H <= 16384, 1 <= A <= 7)", (long long)M, (long long)H, (long long)A);
  OCPPO_REQUIRE(h && dlogits && wa && gp && dwa && dba && workspace &&
                    (wc ? (dvalue && dwc && dbc) : (!dvalue && !dwc && !dbc)),
                "ocppo_heads_bwd: null pointer (wc, dvalue, dwc, dbc: all set or all NULL)");
  OCPPO_REQUIRE(reinterpret_cast<uintptr_t>(h) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(gp) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(workspace) % 256 == 0,
                "ocppo_heads_bwd: h/gp must be 16-B aligned, workspace 256-B aligned");
  OCPPO_REQUIRE(workspace_bytes >= ocppo_heads_bwd_workspace_bytes(M, H, A),
                "ocppo_heads_bwd: workspace too small (%zu < %zu)", workspace_bytes,
                ocppo_heads_bwd_workspace_bytes(M, H, A));
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const int chunks = wg_chunks(M, H);
  const int K = static_cast<int>(A) + (wc ? 1 : 0);
  const int64_t stripes = (H + 4 * kWgL - 1) / (4 * kWgL);
  unsigned* tickets = static_cast<unsigned*>(workspace);
  float* partials = reinterpret_cast<float*>(static_cast<char*>(workspace) + kWgTicketBytes);
  const dim3 grid(static_cast<unsigned>(stripes * chunks)), block(256);
  if (relu)
    hipLaunchKernelGGL(heads_bwd_kernel<true>, grid, block, 0, s, h, dlogits, dvalue, wa, wc, gp,
                       db_h, dwa, dwc, dba, dbc, M, H, (int)A, K, chunks, tickets, partials);
  else
    hipLaunchKernelGGL(heads_bwd_kernel<false>, grid, block, 0, s, h, dlogits, dvalue, wa, wc, gp,
                       db_h, dwa, dwc, dba, dbc, M, H, (int)A, K, chunks, tickets, partials);
  return check_launch("ocppo_heads_bwd");
}
