// Backward of y = relu(x W^T + b) up to the two GEMMs, in ONE HBM pass:
//   gp = threshold_backward(g, y, 0) = (y > 0) ? g : 0       (written, feeds dX = gp W, dW = gp^T x)
//   db = sum over rows of gp                                  (the bias gradient)
// replacing ATen's threshold_backward + sum(0) kernels of the PPObj update (the backward of the
// Linear/ReLU layers of architectures/ppo.py:60-84, reached from ppo_atari_oc.py:607).
// With relu = 0 it is just the column sum (bias gradient of the actor/critic heads), gp unused.
//
// Grid = column tiles (256 columns = 64 lanes x float4) x row chunks; each thread accumulates its
// 4 columns over the chunk's rows (rows strided by the 4 waves), the 4 waves combine in LDS in
// wave order, the chunk partial goes out write-through (sc1), and per column tile the last
// arriving chunk (one agent-scope ticket per tile, MI355X_MICROARCH "Valid forms" row 1) sums the
// chunk partials in chunk order: deterministic. HBM: read g (+ y), write gp, 12 B per element.
#include "ocppo_common.h"

namespace ocppo {

constexpr int kBwdThreads = 256;
constexpr int kBwdCols = 256;  // columns per tile (float4 per lane)

template <bool RELU, bool VEC>
__global__ __launch_bounds__(kBwdThreads) void relu_bias_grad_kernel(
    const float* __restrict__ g, const float* __restrict__ y, int64_t R, int64_t C,
    int64_t rows_per_chunk, float* __restrict__ gp, float* __restrict__ db,
    float* __restrict__ partials, unsigned* __restrict__ tickets) {
  __shared__ float4 red[kBwdThreads / kWave][kWave];
  __shared__ int s_last;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int64_t tile = blockIdx.x, chunk = blockIdx.y, nchunks = gridDim.y;
  const int64_t c0 = tile * kBwdCols + 4 * lane;
  const int64_t r0 = chunk * rows_per_chunk;
  const int64_t r1 = (r0 + rows_per_chunk) < R ? (r0 + rows_per_chunk) : R;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < C) {
    for (int64_t r = r0 + wid; r < r1; r += kBwdThreads / kWave) {
      const int64_t o = r * C + c0;
      float v[4];
      if (VEC) {
        const float4 gg = *reinterpret_cast<const float4*>(g + o);
        v[0] = gg.x; v[1] = gg.y; v[2] = gg.z; v[3] = gg.w;
        if (RELU) {
          const float4 yy = *reinterpret_cast<const float4*>(y + o);
          v[0] = yy.x <= 0.f ? 0.f : v[0];
          v[1] = yy.y <= 0.f ? 0.f : v[1];
          v[2] = yy.z <= 0.f ? 0.f : v[2];
          v[3] = yy.w <= 0.f ? 0.f : v[3];
          *reinterpret_cast<float4*>(gp + o) = make_float4(v[0], v[1], v[2], v[3]);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = 0.f;
          if (c0 + q < C) {
            v[q] = g[o + q];
            if (RELU) {
              v[q] = y[o + q] <= 0.f ? 0.f : v[q];
              gp[o + q] = v[q];
            }
          }
        }
      }
      acc.x += v[0];
      acc.y += v[1];
      acc.z += v[2];
      acc.w += v[3];
    }
  }
  red[wid][lane] = acc;
  __syncthreads();
  if (wid == 0) {
    float4 s = red[0][lane];
#pragma unroll
    for (int w = 1; w < kBwdThreads / kWave; ++w) {
      s.x += red[w][lane].x;
      s.y += red[w][lane].y;
      s.z += red[w][lane].z;
      s.w += red[w][lane].w;
    }
    float* pp = partials + chunk * C;
    const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (c0 + q < C) __hip_atomic_store(pp + c0 + q, sv[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's partial stores drained
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(&tickets[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == nchunks - 1;
  }
  __syncthreads();
  if (!s_last) return;
  // last chunk of this column tile: db[c] = sum over chunks (in order) of the partials
  for (int64_t c = tile * kBwdCols + threadIdx.x; c < C && c < (tile + 1) * kBwdCols;
       c += kBwdThreads) {
    float s = 0.f;
    for (int64_t k = 0; k < nchunks; ++k)
      s += __hip_atomic_load(partials + k * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    db[c] = s;
  }
  if (threadIdx.x == 0) __hip_atomic_store(&tickets[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int64_t bwd_chunks(int64_t R, int64_t C) {
  const int64_t tiles = ceil_div(C, kBwdCols);
  int64_t n = 512 / tiles;                  // ~2 workgroups per CU in total
  const int64_t max_by_rows = ceil_div(R, 32);  // at least 32 rows per chunk
  n = n < max_by_rows ? n : max_by_rows;
  return n > 0 ? n : 1;
}

}  // namespace ocppo

using namespace ocppo;

extern "C" size_t ocppo_relu_bias_grad_workspace_bytes(int64_t R, int64_t C) {
  if (R <= 0 || C <= 0) return 256;
  const int64_t tiles = ceil_div(C, kBwdCols);
  const size_t tick = ((tiles * sizeof(unsigned) + 255) / 256) * 256;
  return tick + static_cast<size_t>(bwd_chunks(R, C)) * C * sizeof(float);
}

extern "C" int ocppo_relu_bias_grad(ocppo_stream_t stream, const float* g, const float* y,
                                    int64_t R, int64_t C, int relu, float* gp, float* db,
                                    void* workspace, size_t workspace_bytes) {
  OCPPO_REQUIRE(R > 0 && C > 0 && ceil_div(C, kBwdCols) <= 65535,
                "ocppo_relu_bias_grad: bad sizes R=%lld C=%lld", (long long)R, (long long)C);
  OCPPO_REQUIRE(g && db && (!relu || (y && gp)), "ocppo_relu_bias_grad: null pointer");
  if (!workspace || workspace_bytes < ocppo_relu_bias_grad_workspace_bytes(R, C))
    return fail(OCPPO_E_WORKSPACE, "ocppo_relu_bias_grad: workspace needs %zu bytes, got %zu",
                ocppo_relu_bias_grad_workspace_bytes(R, C), workspace_bytes);
  const int64_t tiles = ceil_div(C, kBwdCols), chunks = bwd_chunks(R, C);
  const size_t tick = ((tiles * sizeof(unsigned) + 255) / 256) * 256;
  unsigned* tickets = static_cast<unsigned*>(workspace);
  float* partials = reinterpret_cast<float*>(static_cast<char*>(workspace) + tick);
  const int64_t rpc = ceil_div(R, chunks);
  const bool vec = (C % 4 == 0) && ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(y) |
                                      reinterpret_cast<uintptr_t>(gp)) % 16 == 0);
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(chunks)), block(kBwdThreads);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (relu) {
    if (vec)
      hipLaunchKernelGGL((relu_bias_grad_kernel<true, true>), grid, block, 0, s, g, y, R, C, rpc, gp,
                         db, partials, tickets);
    else
      hipLaunchKernelGGL((relu_bias_grad_kernel<true, false>), grid, block, 0, s, g, y, R, C, rpc,
                         gp, db, partials, tickets);
  } else {
    if (vec)
      hipLaunchKernelGGL((relu_bias_grad_kernel<false, true>), grid, block, 0, s, g, y, R, C, rpc,
                         gp, db, partials, tickets);
    else
      hipLaunchKernelGGL((relu_bias_grad_kernel<false, false>), grid, block, 0, s, g, y, R, C, rpc,
                         gp, db, partials, tickets);
  }
  return check_launch("ocppo_relu_bias_grad");
}
