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
// ranges; workgroup (stripe, chunk) owns 256 columns x one row range (4 waves split the rows,
// each lane 4 adjacent columns, 16-B accesses), sums its rows in a fixed order, combines the 4
// waves through LDS in wave order and publishes its 256 partial sums with write-through (sc1)
// stores; the last workgroup of a stripe to arrive on the stripe's ticket (one 128-B line per
// stripe) sums the `chunks` partials of each column in chunk order. Hand-off per
// MI355X_MICROARCH.md "Valid forms" row 1 (sc1 stores, every storing wave's vmcnt(0), barrier,
// one agent-scope atomic add; the last arriver reads with sc1 loads). Tickets re-arm themselves.
// Roofline: HBM / Infinity-Cache stream, 12 B per element (relu) or 4 B (no relu) + 4 B per
// partial; no flops to speak of.
#include "ocppo_common.h"

namespace ocppo {

constexpr int kRbStripeCols = 256;  // columns per workgroup (64 lanes x 4)
constexpr int kRbMaxStripes = 64;   // N <= 16384
constexpr int kRbMaxChunks = 128;
constexpr size_t kRbTicketBytes = kRbMaxStripes * 128;

inline int rb_chunks(int64_t R, int64_t stripes) {
  // >= ~512 workgroups when the rows allow it, >= 32 rows per chunk, <= kRbMaxChunks
  int64_t c = 512 / stripes;
  if (c > kRbMaxChunks) c = kRbMaxChunks;
  const int64_t by_rows = (R + 31) / 32;
  if (c > by_rows) c = by_rows;
  return static_cast<int>(c < 1 ? 1 : c);
}

template <bool RELU>
__global__ __launch_bounds__(256) void relu_bias_grad_kernel(const float* __restrict__ g,
                                                             const float* __restrict__ out,
                                                             float* __restrict__ gp,
                                                             float* __restrict__ db, int64_t R,
                                                             int64_t N, int chunks,
                                                             unsigned* __restrict__ tickets,
                                                             float* __restrict__ partials) {
  __shared__ float red[4][kRbStripeCols];
  __shared__ int s_last;
  const int stripe = blockIdx.x % (static_cast<int>((N + kRbStripeCols - 1) / kRbStripeCols));
  const int chunk = blockIdx.x / (static_cast<int>((N + kRbStripeCols - 1) / kRbStripeCols));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c0 = static_cast<int64_t>(stripe) * kRbStripeCols + 4 * lane;
  const bool live = c0 < N;  // N % 4 == 0: a lane's 4 columns are all live or all dead
  const int64_t rows_per = (R + chunks - 1) / chunks;
  const int64_t r0 = chunk * rows_per;
  const int64_t r1 = r0 + rows_per < R ? r0 + rows_per : R;

  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    int64_t r = r0 + wv;
    // two rows in flight per wave iteration
    for (; r + 4 < r1; r += 8) {
      float4 a = *reinterpret_cast<const float4*>(g + r * N + c0);
      float4 b = *reinterpret_cast<const float4*>(g + (r + 4) * N + c0);
      if (RELU) {
        const float4 oa = *reinterpret_cast<const float4*>(out + r * N + c0);
        const float4 ob = *reinterpret_cast<const float4*>(out + (r + 4) * N + c0);
        a.x = oa.x <= 0.f ? 0.f : a.x; a.y = oa.y <= 0.f ? 0.f : a.y;
        a.z = oa.z <= 0.f ? 0.f : a.z; a.w = oa.w <= 0.f ? 0.f : a.w;
        b.x = ob.x <= 0.f ? 0.f : b.x; b.y = ob.y <= 0.f ? 0.f : b.y;
        b.z = ob.z <= 0.f ? 0.f : b.z; b.w = ob.w <= 0.f ? 0.f : b.w;
        *reinterpret_cast<float4*>(gp + r * N + c0) = a;
        *reinterpret_cast<float4*>(gp + (r + 4) * N + c0) = b;
      }
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
      acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
    }
    for (; r < r1; r += 4) {
      float4 a = *reinterpret_cast<const float4*>(g + r * N + c0);
      if (RELU) {
        const float4 oa = *reinterpret_cast<const float4*>(out + r * N + c0);
        a.x = oa.x <= 0.f ? 0.f : a.x; a.y = oa.y <= 0.f ? 0.f : a.y;
        a.z = oa.z <= 0.f ? 0.f : a.z; a.w = oa.w <= 0.f ? 0.f : a.w;
        *reinterpret_cast<float4*>(gp + r * N + c0) = a;
      }
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
  }
  red[wv][4 * lane + 0] = acc.x;
  red[wv][4 * lane + 1] = acc.y;
  red[wv][4 * lane + 2] = acc.z;
  red[wv][4 * lane + 3] = acc.w;
  __syncthreads();
  const int j = threadIdx.x;  // one column of the stripe per thread
  const int64_t col = static_cast<int64_t>(stripe) * kRbStripeCols + j;
  if (col < N) {
    const float s = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
    __hip_atomic_store(&partials[static_cast<int64_t>(chunk) * N + col], s, __ATOMIC_RELAXED,
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
  if (col < N) {
    float s = 0.f;
#pragma unroll 16
    for (int c = 0; c < chunks; ++c)
      s += __hip_atomic_load(&partials[static_cast<int64_t>(c) * N + col], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    db[col] = s;
  }
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ocppo

using namespace ocppo;

extern "C" size_t ocppo_relu_bias_grad_workspace_bytes(int64_t R, int64_t N) {
  if (R < 1 || N < 1) return kRbTicketBytes;
  const int64_t stripes = (N + kRbStripeCols - 1) / kRbStripeCols;
  return kRbTicketBytes + static_cast<size_t>(rb_chunks(R, stripes)) * N * sizeof(float);
}

extern "C" int ocppo_relu_bias_grad(ocppo_stream_t stream, const float* g, const float* out,
                                    float* gp, float* db, int64_t R, int64_t N, void* workspace,
                                    size_t workspace_bytes) {
  OCPPO_REQUIRE(R >= 0 && N >= 4 && N % 4 == 0 && N <= kRbMaxStripes * kRbStripeCols,
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
  const int64_t stripes = (N + kRbStripeCols - 1) / kRbStripeCols;
  const int chunks = rb_chunks(R, stripes);
  unsigned* tickets = static_cast<unsigned*>(workspace);
  float* partials = reinterpret_cast<float*>(static_cast<char*>(workspace) + kRbTicketBytes);
  const dim3 grid(static_cast<unsigned>(stripes * chunks)), block(256);
  if (out)
    hipLaunchKernelGGL(relu_bias_grad_kernel<true>, grid, block, 0, s, g, out, gp, db, R, N,
                       chunks, tickets, partials);
  else
    hipLaunchKernelGGL(relu_bias_grad_kernel<false>, grid, block, 0, s, g, out, gp, db, R, N,
                       chunks, tickets, partials);
  return check_launch("ocppo_relu_bias_grad");
}
