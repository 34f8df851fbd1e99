// Rollout-side kernels: the per-step store with device frame stacking (replaces
// cleanrl/ppo_atari_oc.py:502-503 and :512-514), the minibatch obs gather (replaces
// `b_obs[mb_inds]` at :566-567), VecNormalize reward normalisation (the SB3 wrapper of :414) and
// the synthetic device env used by the benchmark and tests.
//
// All kernels are HBM streams: one 4-element group per thread, 8-16 B per lane per access,
// consecutive lanes on consecutive addresses.
#include <cstdlib>
#include "ocppo_common.h"
#include "ocppo_store.h"
#include "ocppo_synth_env.h"

namespace ocppo {

template <int FDT, int ODT, int VEC, bool CL>
__global__ __launch_bounds__(256) void rollout_store_kernel(
    const void* __restrict__ frame, const float* __restrict__ reward,
    const float* __restrict__ done, int64_t N, int W, int64_t D, const void* __restrict__ prev,
    void* __restrict__ out, float* __restrict__ net, float* __restrict__ reward_out,
    float* __restrict__ done_out, float net_scale, const void* __restrict__ reset_prev) {
  if (CL)
    store_groups_cl<FDT, ODT, VEC>(blockIdx.x, gridDim.x, frame, reward, done, N, W, D, prev, out,
                                   net, reward_out, done_out, net_scale, reset_prev);
  else
    store_groups<FDT, ODT, VEC>(blockIdx.x, gridDim.x, frame, reward, done, N, W, D, prev, out,
                                net, reward_out, done_out, net_scale, reset_prev);
}

template <int FDT, int ODT, int VEC, bool CL>
__global__ __launch_bounds__(256) void obs_reset_kernel(const void* __restrict__ frame, int64_t N,
                                                        int W, int64_t D, void* __restrict__ out,
                                                        float* __restrict__ net, float net_scale) {
  const int64_t DG = D / VEC;
  const int64_t groups = N * W * DG;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < groups;
       g += stride) {
    const int64_t n = g / (W * DG);
    const int64_t rem = g - n * W * DG;
    const int w = static_cast<int>(rem / DG);
    const int64_t k = (rem - static_cast<int64_t>(w) * DG) * VEC;
    float v[VEC];
    VecIO<FDT, VEC>::load(frame, n * D + k, v);
    const int64_t o = (n * W + w) * D + k;
    VecIO<ODT, VEC>::store(out, o, v);
    if (net) {
      float back[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) back[q] = Elem<ODT>::roundtrip(v[q]) * net_scale;
      if (CL) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) net[(n * D + k + q) * W + w] = back[q];
      } else {
        VecIO<OCPPO_F32, VEC>::store(net, o, back);
      }
    }
  }
}

// ---- minibatch gather: dst[i, :] = f32(src[idx[i], :]) -------------------------------------------
template <int SDT, int VEC>
__global__ __launch_bounds__(256) void gather_rows_kernel(const void* __restrict__ src,
                                                          const int64_t* __restrict__ idx,
                                                          int64_t M, int64_t R,
                                                          float* __restrict__ dst) {
  const int64_t RG = R / VEC;
  const int64_t groups = M * RG;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < groups;
       g += stride) {
    const int64_t i = g / RG;
    const int64_t k = (g - i * RG) * VEC;
    const int64_t row = idx[i];
    float v[VEC];
    VecIO<SDT, VEC>::load(src, row * R + k, v);
    VecIO<OCPPO_F32, VEC>::store(dst, i * R + k, v);
  }
}

// ---- minibatch gather into channels-last order: dst[i, p, c] = f32(src[idx[i], c, p]) ------------
// src rows [C, P] (C stacked frames of P elements), dst rows [P, C]: the NHWC network input of a
// channels_last NatureCNN. One thread per (row, VEC consecutive elements): C loads of VEC, then
// VEC x C contiguous f32 (C == 4: one 16-B store per element).
template <int SDT, int VEC>
__global__ __launch_bounds__(256) void gather_rows_cl_kernel(const void* __restrict__ src,
                                                             const int64_t* __restrict__ idx,
                                                             int64_t M, int C, int64_t P,
                                                             float* __restrict__ dst,
                                                             float scale) {
  const int64_t PG = P / VEC;
  const int64_t groups = M * PG;
  const int64_t R = C * P;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < groups;
       g += stride) {
    const int64_t i = g / PG;
    const int64_t k = (g - i * PG) * VEC;
    const int64_t row = idx[i];
    float* out = dst + i * R + k * C;
    if (C == 4) {
      float v[4][VEC];
#pragma unroll
      for (int c = 0; c < 4; ++c) VecIO<SDT, VEC>::load(src, row * R + c * P + k, v[c]);
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        float px[4] = {v[0][q] * scale, v[1][q] * scale, v[2][q] * scale, v[3][q] * scale};
        VecIO<OCPPO_F32, 4>::store(out, 4 * q, px);  // dst is 16-B aligned (host check)
      }
    } else {
      for (int c = 0; c < C; ++c) {
        float v[VEC];
        VecIO<SDT, VEC>::load(src, row * R + c * P + k, v);
#pragma unroll
        for (int q = 0; q < VEC; ++q) out[q * C + c] = v[q] * scale;
      }
    }
  }
}

__global__ __launch_bounds__(1024) void vecnorm_reward_kernel(
    const float* reward, const float* __restrict__ done, int64_t N, double gamma, double eps,
    double clip, double* __restrict__ ret, double* __restrict__ rms, float* out) {
  vecnorm_block(reward, done, N, gamma, eps, clip, ret, rms, out);
}

// Store + VecNormalize in ONE launch: workgroup 0 normalises the rewards of all N envs (f64
// reduction), workgroups 1.. do the frame-stack store. Both halves only read the env outputs, so
// they need no ordering between them.
template <int FDT, int ODT, int VEC, bool CL>
__global__ __launch_bounds__(256) void store_vecnorm_kernel(
    const void* __restrict__ frame, const float* __restrict__ reward,
    const float* __restrict__ done, int64_t N, int W, int64_t D, const void* __restrict__ prev,
    void* __restrict__ out, float* __restrict__ net, float* __restrict__ done_out, double gamma,
    double eps, double clip, double* __restrict__ ret, double* __restrict__ rms,
    float* __restrict__ reward_out, float net_scale, const void* __restrict__ reset_prev) {
  if (blockIdx.x == 0) {
    vecnorm_block(reward, done, N, gamma, eps, clip, ret, rms, reward_out);
    return;
  }
  if (CL)
    store_groups_cl<FDT, ODT, VEC>(blockIdx.x - 1, gridDim.x - 1, frame, reward, done, N, W, D,
                                   prev, out, net, nullptr, done_out, net_scale, reset_prev);
  else
    store_groups<FDT, ODT, VEC>(blockIdx.x - 1, gridDim.x - 1, frame, reward, done, N, W, D, prev,
                                out, net, nullptr, done_out, net_scale, reset_prev);
}

// ---- synthetic env (per-element step: ocppo_synth_env.h) --------------------------------------
template <bool PIXELS>
__global__ __launch_bounds__(256) void synth_env_kernel(uint64_t seed,
                                                        const int64_t* __restrict__ step_base,
                                                        int64_t step_offset,
                                                        const int64_t* __restrict__ actions,
                                                        int64_t N, int64_t D, void* frame_out,
                                                        float* __restrict__ reward_out,
                                                        float* __restrict__ done_out,
                                                        float* __restrict__ ep) {
  const uint64_t step = static_cast<uint64_t>(step_base[0] + step_offset);
  const int64_t total = N * D;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
       g += stride) {
    const int64_t n = g / D;
    const int64_t k = g - n * D;
    const uint64_t key = synth_env_key(seed, step, n);
    const int64_t a = actions ? actions[n] : 0;
    if (PIXELS) static_cast<uint8_t*>(frame_out)[g] = synth_env_pixel(key, k, a);
    else static_cast<float*>(frame_out)[g] = synth_env_obj(key, k, a);
    if (k == 0) synth_env_outcome(key, n, reward_out, done_out, ep);
  }
}

// Grid of a store launch: one group per (env, slot, VEC elements), or per (env, VEC elements)
// when the network copy is channels-last (the thread then writes every slot).
inline int64_t store_groups_count(int64_t N, int64_t W, int64_t D, int vec, bool cl) {
  return cl ? N * (D / vec) : N * W * (D / vec);
}

template <int FDT, int ODT, bool CL>
int launch_store(hipStream_t s, const void* frame, const float* reward, const float* done,
                 int64_t N, int64_t W, int64_t D, const void* prev, void* out, float* net,
                 float* rout, float* dout, float sc, const void* rp) {
  if (D % 4 == 0)
    hipLaunchKernelGGL((rollout_store_kernel<FDT, ODT, 4, CL>),
                       dim3(grid_for(store_groups_count(N, W, D, 4, CL), 256)), dim3(256), 0, s,
                       frame, reward, done, N, (int)W, D, prev, out, net, rout, dout, sc, rp);
  else
    hipLaunchKernelGGL((rollout_store_kernel<FDT, ODT, 1, CL>),
                       dim3(grid_for(store_groups_count(N, W, D, 1, CL), 256)), dim3(256), 0, s,
                       frame, reward, done, N, (int)W, D, prev, out, net, rout, dout, sc, rp);
  return check_launch("ocppo_rollout_store");
}

struct VecNormArgs {
  double gamma, eps, clip;
  double* ret;
  double* rms;
  float* reward_out;
  float net_scale;
  const void* reset_prev;
};

template <int FDT, int ODT, bool CL>
int launch_store_vecnorm(hipStream_t s, const void* frame, const float* reward, const float* done,
                         int64_t N, int64_t W, int64_t D, const void* prev, void* out, float* net,
                         float* dout, const VecNormArgs& vn) {
  if (D % 4 == 0)
    hipLaunchKernelGGL((store_vecnorm_kernel<FDT, ODT, 4, CL>),
                       dim3(1 + grid_for(store_groups_count(N, W, D, 4, CL), 256)), dim3(256), 0,
                       s, frame, reward, done, N, (int)W, D, prev, out, net, dout, vn.gamma,
                       vn.eps, vn.clip, vn.ret, vn.rms, vn.reward_out, vn.net_scale,
                       vn.reset_prev);
  else
    hipLaunchKernelGGL((store_vecnorm_kernel<FDT, ODT, 1, CL>),
                       dim3(1 + grid_for(store_groups_count(N, W, D, 1, CL), 256)), dim3(256), 0,
                       s, frame, reward, done, N, (int)W, D, prev, out, net, dout, vn.gamma,
                       vn.eps, vn.clip, vn.ret, vn.rms, vn.reward_out, vn.net_scale,
                       vn.reset_prev);
  return check_launch("ocppo_rollout_store_vecnorm");
}

template <int FDT, int ODT, bool CL>
int launch_reset(hipStream_t s, const void* frame, int64_t N, int64_t W, int64_t D, void* out,
                 float* net, float sc) {
  if (D % 4 == 0) {
    const int64_t groups = N * W * (D / 4);
    hipLaunchKernelGGL((obs_reset_kernel<FDT, ODT, 4, CL>), dim3(grid_for(groups, 256)), dim3(256),
                       0, s, frame, N, (int)W, D, out, net, sc);
  } else {
    const int64_t groups = N * W * D;
    hipLaunchKernelGGL((obs_reset_kernel<FDT, ODT, 1, CL>), dim3(grid_for(groups, 256)), dim3(256),
                       0, s, frame, N, (int)W, D, out, net, sc);
  }
  return check_launch("ocppo_obs_reset");
}

template <int SDT>
int launch_gather(hipStream_t s, const void* src, const int64_t* idx, int64_t M, int64_t R,
                  float* dst) {
  if (R % 4 == 0) {
    const int64_t groups = M * (R / 4);
    hipLaunchKernelGGL((gather_rows_kernel<SDT, 4>), dim3(grid_for(groups, 256)), dim3(256), 0, s,
                       src, idx, M, R, dst);
  } else {
    const int64_t groups = M * R;
    hipLaunchKernelGGL((gather_rows_kernel<SDT, 1>), dim3(grid_for(groups, 256)), dim3(256), 0, s,
                       src, idx, M, R, dst);
  }
  return check_launch("ocppo_gather_rows");
}

// The pixel case (u8 stacks of C = 4 frames, NatureCNN input): a workgroup owns 1024 pixels of
// one row. Load phase: thread t reads pixels [4t, 4t+4) of each frame plane (one dword, 256 B per
// wave instruction) into LDS; store phase: thread t writes pixel j = t + 256 i as ONE float4
// (its 4 channels), so consecutive lanes write consecutive 16 B: every wave store instruction is
// a contiguous 1 KB run (the direct form's lanes wrote 16 B pieces 64 B apart). The stores are
// nontemporal: a config-3 minibatch is 925 MB of f32, past the 256 MB Infinity Cache, so caching
// it only evicts; measured 222 -> 176 us per 8192-row launch (tools/kernel_bench.py gather_pixels).
constexpr int kClTile = 1024;  // pixels per workgroup

template <bool NT>
__global__ __launch_bounds__(256) void gather_rows_cl4_u8_kernel(const uint8_t* __restrict__ src,
                                                                 const int64_t* __restrict__ idx,
                                                                 int64_t M, int64_t P,
                                                                 float* __restrict__ dst,
                                                                 float scale, int tiles) {
  __shared__ uint32_t s[4][kClTile / 4];
  const int64_t i = blockIdx.x / tiles;
  const int tile = blockIdx.x - static_cast<int>(i * tiles);
  const int64_t p0 = static_cast<int64_t>(tile) * kClTile;
  const int64_t row = idx[i];
  const uint8_t* sr = src + row * 4 * P;
  const int t = threadIdx.x;
  const int64_t pl = p0 + 4 * t;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    s[c][t] = pl + 3 < P ? *reinterpret_cast<const uint32_t*>(sr + c * P + pl) : 0u;
  __syncthreads();
  float* out = dst + (i * P + p0) * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = t + 256 * k;
    if (p0 + j < P) {
      const int w = j >> 2, sh = 8 * (j & 3);
      const float4 v = make_float4(static_cast<float>((s[0][w] >> sh) & 0xFFu) * scale,
                                   static_cast<float>((s[1][w] >> sh) & 0xFFu) * scale,
                                   static_cast<float>((s[2][w] >> sh) & 0xFFu) * scale,
                                   static_cast<float>((s[3][w] >> sh) & 0xFFu) * scale);
      if constexpr (NT) {
        float* o = out + 4 * j;
        __builtin_nontemporal_store(v.x, o);
        __builtin_nontemporal_store(v.y, o + 1);
        __builtin_nontemporal_store(v.z, o + 2);
        __builtin_nontemporal_store(v.w, o + 3);
      } else {
        *reinterpret_cast<float4*>(out + 4 * j) = v;
      }
    }
  }
}

template <int SDT>
int launch_gather_cl(hipStream_t s, const void* src, const int64_t* idx, int64_t M, int64_t C,
                     int64_t P, float* dst, float sc) {
  if (SDT == OCPPO_U8 && C == 4 && P % 4 == 0 &&
      reinterpret_cast<uintptr_t>(src) % 4 == 0) {
    const int tiles = static_cast<int>((P + kClTile - 1) / kClTile);
    hipLaunchKernelGGL(gather_rows_cl4_u8_kernel<true>, dim3(static_cast<unsigned>(M * tiles)),
                       dim3(256), 0, s, static_cast<const uint8_t*>(src), idx, M, P, dst, sc,
                       tiles);
    return check_launch("ocppo_gather_rows_cl");
  }
  if (P % 4 == 0)
    hipLaunchKernelGGL((gather_rows_cl_kernel<SDT, 4>), dim3(grid_for(M * (P / 4), 256)), dim3(256),
                       0, s, src, idx, M, (int)C, P, dst, sc);
  else
    hipLaunchKernelGGL((gather_rows_cl_kernel<SDT, 1>), dim3(grid_for(M * P, 256)), dim3(256), 0,
                       s, src, idx, M, (int)C, P, dst, sc);
  return check_launch("ocppo_gather_rows_cl");
}

static bool aligned16(const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; }

// x / 255 as ATen computes it for a float tensor and a CPU scalar: x * (1.0f / 255.0f)
// (div_true_kernel_cuda multiplies by the scalar's reciprocal); 1.0f leaves values untouched
inline float net_scale_of(int flags) { return (flags & OCPPO_NET_SCALE_255) ? 1.0f / 255.0f : 1.0f; }

// ---- frame-encoding cache of the rollout (PPObj: the encoder acts on each frame alone) ---------
// enc[n, w, :] = done[n] != 0 || w == W-1 ? fresh[n, :] : enc[n, w+1, :]   (in place)
// The same shift + reset fill as store_groups applies to the stacked frames, applied to their
// encoder outputs: at rollout step t only the newest frame is encoded (N rows instead of N*W).
// One thread owns one (n, VEC-column group) and walks w upward, so every slot w+1 is read before
// it is overwritten.
template <int VEC>
__global__ __launch_bounds__(256) void frame_cache_shift_kernel(float* __restrict__ enc,
                                                                const float* __restrict__ fresh,
                                                                int64_t ld_fresh,
                                                                const float* __restrict__ done,
                                                                int64_t N, int W, int64_t E) {
  const int64_t EG = E / VEC;
  const int64_t groups = N * EG;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < groups;
       g += stride) {
    const int64_t n = g / EG;
    const int64_t k = (g - n * EG) * VEC;
    float nv[VEC];
    VecIO<OCPPO_F32, VEC>::load(fresh, n * ld_fresh + k, nv);
    float* row = enc + n * W * E + k;
    if (done != nullptr && done[n] != 0.f) {
      for (int w = 0; w < W; ++w) VecIO<OCPPO_F32, VEC>::store(row, w * E, nv);
    } else {
      for (int w = 0; w + 1 < W; ++w) {
        float v[VEC];
        VecIO<OCPPO_F32, VEC>::load(row, (w + 1) * E, v);
        VecIO<OCPPO_F32, VEC>::store(row, w * E, v);
      }
      VecIO<OCPPO_F32, VEC>::store(row, (W - 1) * E, nv);
    }
  }
}

static bool valid_dtype(int dt) { return dt == OCPPO_F32 || dt == OCPPO_BF16 || dt == OCPPO_U8; }

}  // namespace ocppo

using namespace ocppo;

extern "C" int ocppo_rollout_store(ocppo_stream_t stream, const void* frame, int frame_dtype,
                                   const float* reward, const float* done, int64_t N, int64_t W,
                                   int64_t D, const void* prev_obs, void* obs_out, int obs_dtype,
                                   float* net_obs, float* reward_out, float* done_out,
                                   int net_flags, const void* reset_prev) {
  OCPPO_REQUIRE(N >= 0 && W >= 1 && D >= 1 && W <= 64, "ocppo_rollout_store: bad sizes");
  OCPPO_REQUIRE((net_flags & ~3) == 0 &&
                    (!(net_flags & OCPPO_NET_CHANNELS_LAST) || (net_obs && aligned16(net_obs))),
                "ocppo_rollout_store: bad net_flags %d (channels-last needs a 16-B aligned net_obs)",
                net_flags);
  const bool net_layout = net_flags & OCPPO_NET_CHANNELS_LAST;
  const float sc = net_scale_of(net_flags);
  OCPPO_REQUIRE(frame_dtype == OCPPO_F32 || frame_dtype == OCPPO_U8,
                "ocppo_rollout_store: frame dtype must be OCPPO_F32 or OCPPO_U8");
  OCPPO_REQUIRE(valid_dtype(obs_dtype), "ocppo_rollout_store: bad obs dtype %d", obs_dtype);
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(frame && reward && done && prev_obs && obs_out, "ocppo_rollout_store: null pointer");
  OCPPO_REQUIRE(prev_obs != obs_out, "ocppo_rollout_store: prev_obs must not alias obs_out");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
#define OCPPO_STORE(F, O)                                                                     \
  if (frame_dtype == F && obs_dtype == O)                                                     \
    return net_layout                                                                        \
               ? launch_store<F, O, true>(s, frame, reward, done, N, W, D, prev_obs, obs_out,  \
                                          net_obs, reward_out, done_out, sc, reset_prev)       \
               : launch_store<F, O, false>(s, frame, reward, done, N, W, D, prev_obs, obs_out, \
                                           net_obs, reward_out, done_out, sc, reset_prev);
  OCPPO_STORE(OCPPO_F32, OCPPO_F32)
  OCPPO_STORE(OCPPO_F32, OCPPO_BF16)
  OCPPO_STORE(OCPPO_F32, OCPPO_U8)
  OCPPO_STORE(OCPPO_U8, OCPPO_F32)
  OCPPO_STORE(OCPPO_U8, OCPPO_BF16)
  OCPPO_STORE(OCPPO_U8, OCPPO_U8)
#undef OCPPO_STORE
  return fail(OCPPO_E_INVALID, "ocppo_rollout_store: unsupported dtype pair");
}

extern "C" int ocppo_obs_reset(ocppo_stream_t stream, const void* frame, int frame_dtype, int64_t N,
                               int64_t W, int64_t D, void* obs_out, int obs_dtype, float* net_obs,
                               int net_flags) {
  OCPPO_REQUIRE(N >= 0 && W >= 1 && D >= 1 && W <= 64, "ocppo_obs_reset: bad sizes");
  OCPPO_REQUIRE((net_flags & ~3) == 0, "ocppo_obs_reset: bad net_flags %d", net_flags);
  const bool net_layout = net_flags & OCPPO_NET_CHANNELS_LAST;
  const float sc = net_scale_of(net_flags);
  OCPPO_REQUIRE(frame_dtype == OCPPO_F32 || frame_dtype == OCPPO_U8,
                "ocppo_obs_reset: frame dtype must be OCPPO_F32 or OCPPO_U8");
  OCPPO_REQUIRE(valid_dtype(obs_dtype), "ocppo_obs_reset: bad obs dtype %d", obs_dtype);
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(frame && obs_out, "ocppo_obs_reset: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
#define OCPPO_RESET(F, O)                                                                 \
  if (frame_dtype == F && obs_dtype == O)                                                 \
    return net_layout ? launch_reset<F, O, true>(s, frame, N, W, D, obs_out, net_obs, sc)  \
                      : launch_reset<F, O, false>(s, frame, N, W, D, obs_out, net_obs, sc);
  OCPPO_RESET(OCPPO_F32, OCPPO_F32)
  OCPPO_RESET(OCPPO_F32, OCPPO_BF16)
  OCPPO_RESET(OCPPO_F32, OCPPO_U8)
  OCPPO_RESET(OCPPO_U8, OCPPO_F32)
  OCPPO_RESET(OCPPO_U8, OCPPO_BF16)
  OCPPO_RESET(OCPPO_U8, OCPPO_U8)
#undef OCPPO_RESET
  return fail(OCPPO_E_INVALID, "ocppo_obs_reset: unsupported dtype pair");
}

extern "C" int ocppo_gather_rows(ocppo_stream_t stream, const void* src, int src_dtype,
                                 const int64_t* idx, int64_t M, int64_t R, float* dst) {
  OCPPO_REQUIRE(M >= 0 && R >= 1, "ocppo_gather_rows: bad sizes");
  OCPPO_REQUIRE(valid_dtype(src_dtype), "ocppo_gather_rows: bad dtype %d", src_dtype);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(src && idx && dst, "ocppo_gather_rows: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (src_dtype == OCPPO_F32) return launch_gather<OCPPO_F32>(s, src, idx, M, R, dst);
  if (src_dtype == OCPPO_BF16) return launch_gather<OCPPO_BF16>(s, src, idx, M, R, dst);
  return launch_gather<OCPPO_U8>(s, src, idx, M, R, dst);
}

extern "C" int ocppo_gather_rows_cl(ocppo_stream_t stream, const void* src, int src_dtype,
                                    const int64_t* idx, int64_t M, int64_t C, int64_t P,
                                    float* dst, int net_flags) {
  OCPPO_REQUIRE((net_flags & ~3) == 0, "ocppo_gather_rows_cl: bad net_flags %d", net_flags);
  const float sc = net_scale_of(net_flags);
  OCPPO_REQUIRE(M >= 0 && C >= 1 && C <= 64 && P >= 1, "ocppo_gather_rows_cl: bad sizes");
  OCPPO_REQUIRE(valid_dtype(src_dtype), "ocppo_gather_rows_cl: bad dtype %d", src_dtype);
  if (M == 0) return OCPPO_OK;
  OCPPO_REQUIRE(src && idx && dst, "ocppo_gather_rows_cl: null pointer");
  OCPPO_REQUIRE(aligned16(dst), "ocppo_gather_rows_cl: dst must be 16-B aligned");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  if (src_dtype == OCPPO_F32) return launch_gather_cl<OCPPO_F32>(s, src, idx, M, C, P, dst, sc);
  if (src_dtype == OCPPO_BF16) return launch_gather_cl<OCPPO_BF16>(s, src, idx, M, C, P, dst, sc);
  return launch_gather_cl<OCPPO_U8>(s, src, idx, M, C, P, dst, sc);
}

extern "C" int ocppo_vecnorm_reward(ocppo_stream_t stream, const float* reward, const float* done,
                                    int64_t N, double gamma, double epsilon, double clip_reward,
                                    double* ret_state, double* rms_state, float* reward_out) {
  OCPPO_REQUIRE(N >= 1, "ocppo_vecnorm_reward: bad size N=%lld", (long long)N);
  OCPPO_REQUIRE(reward && done && ret_state && rms_state && reward_out,
                "ocppo_vecnorm_reward: null pointer");
  clear_stale_error();
  hipLaunchKernelGGL(vecnorm_reward_kernel, dim3(1), dim3(1024), 0, as_stream(stream), reward, done,
                     N, gamma, epsilon, clip_reward, ret_state, rms_state, reward_out);
  return check_launch("ocppo_vecnorm_reward");
}

extern "C" int ocppo_synth_env_step(ocppo_stream_t stream, uint64_t seed, const int64_t* step_base,
                                    int64_t step_offset, const int64_t* actions, int64_t N,
                                    int64_t D, int pixel_mode, void* frame_out, float* reward_out,
                                    float* done_out, float* ep_state) {
  OCPPO_REQUIRE(N >= 0 && D >= 1, "ocppo_synth_env_step: bad sizes");
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(step_base && frame_out && reward_out && done_out,
                "ocppo_synth_env_step: null pointer");
  const dim3 grid(grid_for(N * D, 256));
  clear_stale_error();
  if (pixel_mode)
    hipLaunchKernelGGL(synth_env_kernel<true>, grid, dim3(256), 0, as_stream(stream), seed,
                       step_base, step_offset, actions, N, D, frame_out, reward_out, done_out,
                       ep_state);
  else
    hipLaunchKernelGGL(synth_env_kernel<false>, grid, dim3(256), 0, as_stream(stream), seed,
                       step_base, step_offset, actions, N, D, frame_out, reward_out, done_out,
                       ep_state);
  return check_launch("ocppo_synth_env_step");
}

extern "C" int ocppo_rollout_store_vecnorm(ocppo_stream_t stream, const void* frame,
                                           int frame_dtype, const float* reward, const float* done,
                                           int64_t N, int64_t W, int64_t D, const void* prev_obs,
                                           void* obs_out, int obs_dtype, float* net_obs,
                                           float* done_out, double gamma, double epsilon,
                                           double clip_reward, double* ret_state,
                                           double* rms_state, float* reward_out, int net_flags,
                                           const void* reset_prev) {
  OCPPO_REQUIRE(N >= 1 && W >= 1 && D >= 1 && W <= 64, "ocppo_rollout_store_vecnorm: bad sizes");
  OCPPO_REQUIRE((net_flags & ~3) == 0 &&
                    (!(net_flags & OCPPO_NET_CHANNELS_LAST) || (net_obs && aligned16(net_obs))),
                "ocppo_rollout_store_vecnorm: bad net_flags %d (channels-last needs a 16-B aligned "
                "net_obs)", net_flags);
  const bool net_layout = net_flags & OCPPO_NET_CHANNELS_LAST;
  OCPPO_REQUIRE(frame_dtype == OCPPO_F32 || frame_dtype == OCPPO_U8,
                "ocppo_rollout_store_vecnorm: frame dtype must be OCPPO_F32 or OCPPO_U8");
  OCPPO_REQUIRE(valid_dtype(obs_dtype), "ocppo_rollout_store_vecnorm: bad obs dtype %d", obs_dtype);
  OCPPO_REQUIRE(frame && reward && done && prev_obs && obs_out && ret_state && rms_state &&
                    reward_out,
                "ocppo_rollout_store_vecnorm: null pointer");
  OCPPO_REQUIRE(prev_obs != obs_out, "ocppo_rollout_store_vecnorm: prev_obs must not alias obs_out");
  OCPPO_REQUIRE(reward_out != reward, "ocppo_rollout_store_vecnorm: reward_out must not alias reward");
  const VecNormArgs vn{gamma,     epsilon,    clip_reward,
                       ret_state, rms_state,  reward_out, net_scale_of(net_flags),
                       reset_prev};
  clear_stale_error();
  hipStream_t s = as_stream(stream);
#define OCPPO_SV(F, O)                                                                        \
  if (frame_dtype == F && obs_dtype == O)                                                     \
    return net_layout ? launch_store_vecnorm<F, O, true>(s, frame, reward, done, N, W, D,     \
                                                         prev_obs, obs_out, net_obs,          \
                                                         done_out, vn)                        \
                      : launch_store_vecnorm<F, O, false>(s, frame, reward, done, N, W, D,    \
                                                          prev_obs, obs_out, net_obs,         \
                                                          done_out, vn);
  OCPPO_SV(OCPPO_F32, OCPPO_F32)
  OCPPO_SV(OCPPO_F32, OCPPO_BF16)
  OCPPO_SV(OCPPO_F32, OCPPO_U8)
  OCPPO_SV(OCPPO_U8, OCPPO_F32)
  OCPPO_SV(OCPPO_U8, OCPPO_BF16)
  OCPPO_SV(OCPPO_U8, OCPPO_U8)
#undef OCPPO_SV
  return fail(OCPPO_E_INVALID, "ocppo_rollout_store_vecnorm: unsupported dtype pair");
}

extern "C" int ocppo_frame_cache_shift(ocppo_stream_t stream, float* enc, const float* fresh,
                                       int64_t ld_fresh, const float* done, int64_t N, int64_t W,
                                       int64_t E) {
  OCPPO_REQUIRE(N >= 0 && W >= 1 && W <= 64 && E >= 1 && ld_fresh >= E,
                "ocppo_frame_cache_shift: bad sizes");
  if (N == 0) return OCPPO_OK;
  OCPPO_REQUIRE(enc && fresh, "ocppo_frame_cache_shift: null pointer");
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  const bool vec = E % 4 == 0 && ld_fresh % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(enc) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(fresh) % 16 == 0;
  if (vec)
    hipLaunchKernelGGL(frame_cache_shift_kernel<4>, dim3(grid_for(N * (E / 4), 256)), dim3(256), 0,
                       s, enc, fresh, ld_fresh, done, N, (int)W, E);
  else
    hipLaunchKernelGGL(frame_cache_shift_kernel<1>, dim3(grid_for(N * E, 256)), dim3(256), 0, s,
                       enc, fresh, ld_fresh, done, N, (int)W, E);
  return check_launch("ocppo_frame_cache_shift");
}
