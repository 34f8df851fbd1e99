// GAE reverse scan (replaces the Python loop of cleanrl/ppo_atari_oc.py:533-547; the same block is
// ppo.py:218-231 and ppo_atari_multigpu.py:288-301).
//
// Layout: rewards/values/dones/advantages/returns are [T, N] f32, step-major, so one time row of
// an env tile is contiguous.
//
// The recurrence A_t = delta_t + c_t * A_{t+1} is the only serial part, and it is two dependent
// f32 ops per step; everything else is parallel over (t, n). gae_tile_kernel therefore spreads a
// rollout over many small workgroups (E envs each, E chosen so that the grid has >= 64
// workgroups) and splits the work into phases:
//   1. all 256 threads stage the chunk's r, v, d rows into LDS (16-B loads when E % 4 == 0);
//   2. all threads form, per (t, n), delta = (r + (f32(gamma) * v') * nnt) - v and
//      c = f32(gamma*lambda) * nnt with nnt = 1 - d' (v', d' = the next row, or next_value /
//      next_done / the later chunk's first row at the chunk boundary);
//   3. one lane per env runs A = delta + c * A over the chunk (16 rows of operands per LDS batch);
//   4. all threads store A and R = A + v.
// Every value is the reference's op for op, in f32 without contraction (-ffp-contract=off), so
// advantages and returns are bit-identical to the PyTorch loop (ppo_atari_oc.py:533-547): only
// WHERE each op runs changed, not the ops or their order along the recurrence.
// Roofline: HBM-bound, 20 B per (t, n) element + 8 B per env (next_value, next_done); at config
// sizes (128 x 128, 328 KB) it is latency-bound, hence the small tiles.
#include "ocppo_common.h"

namespace ocppo {

// The per-sample record ocppo_minibatch_prepare_records gathers (ocppo.h OcppoSampleRecord): one
// 16-B load per sample instead of five scattered 4-8 B values. The return is not stored: it is
// advantage + value, recomputed by the gather with the same f32 add (bitwise the same).
__device__ __forceinline__ void gae_put_record(float4* __restrict__ rec, size_t gi, float lp,
                                               float a, float v, int64_t act) {
  rec[gi] = make_float4(lp, a, v, __int_as_float(static_cast<int>(act)));
}

// The recurrence over rows rows-1 .. 0 of env column `tid` of an E-wide LDS tile (delta in sa,
// c in sc; A written over delta): whole groups of 16 rows with no per-step branch (a uniform
// branch per step costs more than the two dependent ops it guards), then the remainder.
template <int E>
__device__ __forceinline__ void gae_chain(float* sa, const float* sc, int rows, int tid,
                                          float& last) {
  int r0 = rows - 1;
  for (int grp = rows / 16; grp > 0; --grp, r0 -= 16) {
    float d[16], c[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      d[k] = sa[(r0 - k) * E + tid];
      c[k] = sc[(r0 - k) * E + tid];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      last = d[k] + c[k] * last;
      d[k] = last;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) sa[(r0 - k) * E + tid] = d[k];
  }
  for (; r0 >= 0; --r0) {
    last = sa[r0 * E + tid] + sc[r0 * E + tid] * last;
    sa[r0 * E + tid] = last;
  }
}

template <int E>
__global__ __launch_bounds__(256) void gae_tile_kernel(const float* __restrict__ rew,
                                                       const float* __restrict__ val,
                                                       const float* __restrict__ don,
                                                       const float* __restrict__ next_val,
                                                       const float* __restrict__ next_done, int T,
                                                       int64_t N, int TC, float g, float gl,
                                                       float* __restrict__ adv,
                                                       float* __restrict__ ret,
                                                       const float* __restrict__ lp,
                                                       const int64_t* __restrict__ act,
                                                       float4* __restrict__ rec) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sa = smem;           // [TC][E]  rewards in -> delta -> advantages
  float* sv = sa + TC * E;    // [TC][E]  values
  float* sd = sv + TC * E;    // [TC][E]  dones
  float* sc = sd + TC * E;    // [TC][E]  c = f32(gamma * lambda) * nnt
  __shared__ float s_cv[E], s_cd[E];  // per env: the value / done of the row after the chunk

  const int64_t n0 = static_cast<int64_t>(blockIdx.x) * E;
  const int tid = threadIdx.x;
  const bool vec = (E % 4) == 0 && (N & 3) == 0;  // every tile row is 16-B aligned
  const bool chain = tid < E && n0 + tid < N;
  if (tid < E) {
    s_cv[tid] = n0 + tid < N ? next_val[n0 + tid] : 0.f;
    s_cd[tid] = n0 + tid < N ? next_done[n0 + tid] : 0.f;
  }
  float last = 0.f;

  for (int t_hi = T; t_hi > 0; t_hi -= TC) {
    const int t_lo = t_hi > TC ? t_hi - TC : 0;
    const int rows = t_hi - t_lo;
    // 1. stage
    if (vec) {
      constexpr int C4 = E / 4;
      for (int e = tid; e < rows * C4; e += 256) {
        const int row = e / C4, c4 = e - row * C4;
        const int64_t col = n0 + 4 * c4;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          const int li = row * E + 4 * c4;
          *reinterpret_cast<float4*>(sa + li) = *reinterpret_cast<const float4*>(rew + gi);
          *reinterpret_cast<float4*>(sv + li) = *reinterpret_cast<const float4*>(val + gi);
          *reinterpret_cast<float4*>(sd + li) = *reinterpret_cast<const float4*>(don + gi);
        }
      }
    } else {
      for (int e = tid; e < rows * E; e += 256) {
        const int row = e / E, c = e - row * E;
        const int64_t col = n0 + c;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          sa[e] = rew[gi];
          sv[e] = val[gi];
          sd[e] = don[gi];
        }
      }
    }
    __syncthreads();
    // 2. delta and c of every (t, n) of the chunk
    for (int e = tid; e < rows * E; e += 256) {
      const int row = e / E, c = e - row * E;
      const float nv = row + 1 < rows ? sv[e + E] : s_cv[c];
      const float nd = row + 1 < rows ? sd[e + E] : s_cd[c];
      const float nnt = 1.0f - nd;
      float delta = sa[e] + (g * nv) * nnt;
      sa[e] = delta - sv[e];
      sc[e] = gl * nnt;
    }
    __syncthreads();
    if (tid < E) {  // the next (earlier) chunk's boundary row
      s_cv[tid] = sv[tid];
      s_cd[tid] = sd[tid];
    }
    // 3. the recurrence, one lane per env
#ifndef OCPPO_GAE_NOCHAIN  // probe variant (tools/): every phase but the recurrence
    if (chain) {
#else
    if (chain && T < 0) {
#endif
      gae_chain<E>(sa, sc, rows, tid, last);
    }
    __syncthreads();
    // 4. advantages and returns
    if (vec) {
      constexpr int C4 = E / 4;
      for (int e = tid; e < rows * C4; e += 256) {
        const int row = e / C4, c4 = e - row * C4;
        const int64_t col = n0 + 4 * c4;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          const int li = row * E + 4 * c4;
          const float4 a = *reinterpret_cast<const float4*>(sa + li);
          const float4 v = *reinterpret_cast<const float4*>(sv + li);
          const float4 r = make_float4(a.x + v.x, a.y + v.y, a.z + v.z, a.w + v.w);
          *reinterpret_cast<float4*>(adv + gi) = a;
          *reinterpret_cast<float4*>(ret + gi) = r;
          if (rec) {
            const float4 l = *reinterpret_cast<const float4*>(lp + gi);
            gae_put_record(rec, gi, l.x, a.x, v.x, act[gi]);
            gae_put_record(rec, gi + 1, l.y, a.y, v.y, act[gi + 1]);
            gae_put_record(rec, gi + 2, l.z, a.z, v.z, act[gi + 2]);
            gae_put_record(rec, gi + 3, l.w, a.w, v.w, act[gi + 3]);
          }
        }
      }
    } else {
      for (int e = tid; e < rows * E; e += 256) {
        const int row = e / E, c = e - row * E;
        const int64_t col = n0 + c;
        if (col < N) {
          const size_t gi = static_cast<size_t>(t_lo + row) * N + col;
          adv[gi] = sa[e];
          ret[gi] = sa[e] + sv[e];
          if (rec) gae_put_record(rec, gi, lp[gi], sa[e], sv[e], act[gi]);
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
// the occupancy (16 waves per CU at N = 262144) hides the latency; same arithmetic as gae_tile_kernel,
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
                                                         float* __restrict__ ret,
                                                         const float* __restrict__ lp,
                                                         const int64_t* __restrict__ act,
                                                         float4* __restrict__ rec) {
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
        if (rec) gae_put_record(rec, gi, lp[gi], r[k], v[k], act[gi]);
      }
    }
  }
}

}  // namespace ocppo

using namespace ocppo;

static int gae_launch(ocppo_stream_t stream, const float* rewards, const float* values,
                      const float* dones, const float* next_value, const float* next_done,
                      int64_t T, int64_t N, double gamma, double gae_lambda, float* advantages,
                      float* returns, const float* logprobs, const int64_t* actions,
                      void* records) {
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
                       returns, logprobs, actions, static_cast<float4*>(records));
  } else {
    // >= 64 workgroups where N allows it: E = 4 envs per workgroup up to N = 256, then wider
    const int TC = T < 128 ? (int)T : 128;
#define OCPPO_GAE_TILE(E)                                                                          \
  hipLaunchKernelGGL(gae_tile_kernel<E>, dim3(ceil_div(N, E)), dim3(256),                         \
                     4 * sizeof(float) * TC * (E), s, rewards, values, dones, next_value,          \
                     next_done, (int)T, N, TC, g, gl, advantages, returns, logprobs, actions,      \
                     static_cast<float4*>(records))
#ifdef OCPPO_GAE_E  // tile-width variants (tools/)
    if (N <= 1024) OCPPO_GAE_TILE(OCPPO_GAE_E);
    else
#endif
    if (N <= 256) OCPPO_GAE_TILE(4);
    else if (N <= 1024) OCPPO_GAE_TILE(16);
    else OCPPO_GAE_TILE(64);
#undef OCPPO_GAE_TILE
  }
  return check_launch("ocppo_gae");
}

extern "C" int ocppo_gae(ocppo_stream_t stream, const float* rewards, const float* values,
                         const float* dones, const float* next_value, const float* next_done,
                         int64_t T, int64_t N, double gamma, double gae_lambda, float* advantages,
                         float* returns) {
  return gae_launch(stream, rewards, values, dones, next_value, next_done, T, N, gamma,
                    gae_lambda, advantages, returns, nullptr, nullptr, nullptr);
}

extern "C" int ocppo_gae_records(ocppo_stream_t stream, const float* rewards, const float* values,
                                 const float* dones, const float* next_value,
                                 const float* next_done, int64_t T, int64_t N, double gamma,
                                 double gae_lambda, float* advantages, float* returns,
                                 const float* logprobs, const int64_t* actions, void* records) {
  OCPPO_REQUIRE(logprobs && actions && records && reinterpret_cast<uintptr_t>(records) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(logprobs) % 16 == 0,
                "ocppo_gae_records: logprobs (16-B aligned), actions and 16-B aligned records");
  return gae_launch(stream, rewards, values, dones, next_value, next_done, T, N, gamma,
                    gae_lambda, advantages, returns, logprobs, actions, records);
}
