// GAE reverse scan (replaces the Python loop of cleanrl/ppo_atari_oc.py:533-547; the same block is
// ppo.py:218-231 and ppo_atari_multigpu.py:288-301).
//
// Layout: rewards/values/dones/advantages/returns are [T, N] f32, step-major, so one time row of
// an env tile is contiguous. A workgroup owns ENV_TILE envs and walks the rollout from t = T-1
// down in chunks of TC rows:
//   1. all 256 threads stage the chunk's r, v, d rows into LDS with 16-B loads (coalesced);
//   2. one lane per env runs the sequential recurrence out of LDS and overwrites r with A;
//   3. all threads stream A and R = A + v back out with 16-B stores.
// The recurrence is carried in registers across chunks. The arithmetic is the reference's, op by
// op, in f32 without contraction (build flag -ffp-contract=off):
//   nnt = 1 - d';  delta = (r + (f32(gamma) * v') * nnt) - v;  A = delta + (f32(gamma*lambda) * nnt) * A'
// so advantages and returns are bit-identical to the PyTorch loop.
// Roofline: HBM-bound, 20 B per (t, n) element + 8 B per env (next_value, next_done).
#include "ocppo_common.h"

namespace ocppo {

template <int ENV_TILE>
__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rew,
                                                  const float* __restrict__ val,
                                                  const float* __restrict__ don,
                                                  const float* __restrict__ next_val,
                                                  const float* __restrict__ next_done, int T,
                                                  int64_t N, int TC, float g, float gl,
                                                  float* __restrict__ adv, float* __restrict__ ret) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sr = smem;                  // [TC][ENV_TILE]  rewards in, advantages out
  float* sv = smem + TC * ENV_TILE;  // [TC][ENV_TILE]  values
  float* sd = sv + TC * ENV_TILE;    // [TC][ENV_TILE]  dones

  const int64_t n0 = static_cast<int64_t>(blockIdx.x) * ENV_TILE;
  const int tid = threadIdx.x;
  const bool vec = (N & 3) == 0;  // every row start is 16-B aligned
  const bool active = tid < ENV_TILE && n0 + tid < N;

  float last = 0.f, carry_v = 0.f, carry_d = 0.f;
  if (active) {
    carry_v = next_val[n0 + tid];
    carry_d = next_done[n0 + tid];
  }

  for (int t_hi = T; t_hi > 0; t_hi -= TC) {
    const int t_lo = t_hi > TC ? t_hi - TC : 0;
    const int rows = t_hi - t_lo;

    // 1. stage
    if (vec) {
      constexpr int C4 = ENV_TILE / 4;
      for (int e = tid; e < rows * C4; e += blockDim.x) {
        const int row = e / C4, c4 = e - row * C4;
        const int64_t col = n0 + 4 * c4;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          const int li = row * ENV_TILE + 4 * c4;
          *reinterpret_cast<float4*>(sr + li) = *reinterpret_cast<const float4*>(rew + gi);
          *reinterpret_cast<float4*>(sv + li) = *reinterpret_cast<const float4*>(val + gi);
          *reinterpret_cast<float4*>(sd + li) = *reinterpret_cast<const float4*>(don + gi);
        }
      }
    } else {
      for (int e = tid; e < rows * ENV_TILE; e += blockDim.x) {
        const int row = e / ENV_TILE, c = e - row * ENV_TILE;
        const int64_t col = n0 + c;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          sr[e] = rew[gi];
          sv[e] = val[gi];
          sd[e] = don[gi];
        }
      }
    }
    __syncthreads();

    // 2. sequential recurrence, one lane per env
    if (active) {
      for (int row = rows - 1; row >= 0; --row) {
        const int li = row * ENV_TILE + tid;
        const float r = sr[li], v = sv[li], d = sd[li];
        const float nnt = 1.0f - carry_d;
        float delta = r + (g * carry_v) * nnt;
        delta = delta - v;
        last = delta + (gl * nnt) * last;
        sr[li] = last;
        carry_v = v;
        carry_d = d;
      }
    }
    __syncthreads();

    // 3. write back advantages and returns
    if (vec) {
      constexpr int C4 = ENV_TILE / 4;
      for (int e = tid; e < rows * C4; e += blockDim.x) {
        const int row = e / C4, c4 = e - row * C4;
        const int64_t col = n0 + 4 * c4;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          const int li = row * ENV_TILE + 4 * c4;
          const float4 a = *reinterpret_cast<const float4*>(sr + li);
          const float4 v = *reinterpret_cast<const float4*>(sv + li);
          *reinterpret_cast<float4*>(adv + gi) = a;
          *reinterpret_cast<float4*>(ret + gi) = make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
        }
      }
    } else {
      for (int e = tid; e < rows * ENV_TILE; e += blockDim.x) {
        const int row = e / ENV_TILE, c = e - row * ENV_TILE;
        const int64_t col = n0 + c;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          adv[gi] = sr[e];
          ret[gi] = sr[e] + sv[e];
        }
      }
    }
    __syncthreads();  // the next chunk overwrites the LDS tile
  }
}

// Streaming form for wide rollouts (N >= 64K envs): one thread per env walks t = T-1 .. 0 with
// the rows in registers, U rows of r/v/d loaded per batch before the U dependent steps run
// (256 B per wave instruction: consecutive lanes = consecutive envs of a time row), advantages
// and returns stored per batch. No LDS and no barriers, so every wave streams independently and
// the occupancy (16 waves per CU at N = 262144) hides the latency; same arithmetic as gae_kernel,
// op by op. T=128, N=262144 on MI355X: U = 1/2/4/8/16/32 -> 121/120/123/128/133/146 us, the LDS
// form 143 us (tools/kernel_bench.py gae scaled).
template <int U>
__global__ __launch_bounds__(256) void gae_stream_kernel(const float* __restrict__ rew,
                                                         const float* __restrict__ val,
                                                         const float* __restrict__ don,
                                                         const float* __restrict__ next_val,
                                                         const float* __restrict__ next_done,
                                                         int T, int64_t N, float g, float gl,
                                                         float* __restrict__ adv,
                                                         float* __restrict__ ret) {
  const int64_t n = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float last = 0.f, carry_v = next_val[n], carry_d = next_done[n];
  for (int t_hi = T; t_hi > 0; t_hi -= U) {
    const int rows = t_hi < U ? t_hi : U;
    float r[U], v[U], d[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (k < rows) {
        const size_t gi = static_cast<size_t>(t_hi - 1 - k) * N + n;
        r[k] = rew[gi];
        v[k] = val[gi];
        d[k] = don[gi];
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (k < rows) {
        const float nnt = 1.0f - carry_d;
        float delta = r[k] + (g * carry_v) * nnt;
        delta = delta - v[k];
        last = delta + (gl * nnt) * last;
        r[k] = last;
        carry_v = v[k];
        carry_d = d[k];
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (k < rows) {
        const size_t gi = static_cast<size_t>(t_hi - 1 - k) * N + n;
        adv[gi] = r[k];
        ret[gi] = r[k] + v[k];
      }
    }
  }
}

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_gae(ocppo_stream_t stream, const float* rewards, const float* values,
                         const float* dones, const float* next_value, const float* next_done,
                         int64_t T, int64_t N, double gamma, double gae_lambda, float* advantages,
                         float* returns) {
  OCPPO_REQUIRE(T >= 0 && N >= 0 && T <= INT32_MAX, "ocppo_gae: bad sizes T=%lld N=%lld",
                (long long)T, (long long)N);
  if (T == 0 || N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(rewards && values && dones && next_value && next_done && advantages && returns,
                "ocppo_gae: null pointer");
  // PyTorch rounds `gamma * tensor` to f32(gamma) and `gamma * gae_lambda * tensor` to
  // f32(gamma * gae_lambda) with the product taken in double (Python floats).
  const float g = static_cast<float>(gamma);
  const float gl = static_cast<float>(gamma * gae_lambda);
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (N >= 64 * 1024) {
    hipLaunchKernelGGL(gae_stream_kernel<2>, dim3(ceil_div(N, 256)), dim3(256), 0, s, rewards,
                       values, dones, next_value, next_done, (int)T, N, g, gl, advantages,
                       returns);
  } else {
    constexpr int TILE = 64;
    const int TC = 64;
    const size_t lds = 3 * sizeof(float) * TC * TILE;
    hipLaunchKernelGGL(gae_kernel<TILE>, dim3(ceil_div(N, TILE)), dim3(256), lds, s, rewards,
                       values, dones, next_value, next_done, (int)T, N, TC, g, gl, advantages,
                       returns);
  }
  return check_launch("ocppo_gae");
}
