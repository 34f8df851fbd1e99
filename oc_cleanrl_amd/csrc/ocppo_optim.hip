// Gradient-norm clipping + Adam over ONE flat parameter / gradient / moment buffer
// (replaces `nn.utils.clip_grad_norm_(agent.parameters(), max_grad_norm); optimizer.step()` of
// cleanrl/ppo_atari_oc.py:608-610 with torch.optim.Adam(eps=1e-5), and the `/ world_size` of the
// DP all-reduce, ppo_atari_multigpu.py:369-374).
//
//   norm kernel : grid-strided partial sums of (g * grad_scale)^2 per workgroup (16-B loads),
//                 one plain store per workgroup; workgroup 0 also advances the step counter
//                 (the only writer of it; the adam kernel, next on the stream, only reads it)
//   adam kernel : every workgroup first combines the <= 1024 partials itself, in a fixed order
//                 (the same fixed-order sum in every workgroup, so every one derives the same
//                 total_norm, clip = min(max_norm / (total_norm + 1e-6), 1), step_size =
//                 lr / (1 - beta1^step), bc2_sqrt = sqrt(1 - beta2^step)), then
//                 g = (g * grad_scale) * clip;  m = beta1*m + (1-beta1)*g;
//                 v = beta2*v + (1-beta2)*g*g;  p -= step_size * m / (sqrt(v)/bc2_sqrt + eps)
//                 (the formula of ATen's fused Adam), 16-B vectors, 28 B of HBM per parameter.
// No ticket and no last-arriver hand-off: the kernel boundary orders the partials (round 3's
// ticketed form spent ~7 us of its 11 per minibatch in the 256-way fan-in and the dependent
// combine at config 2).
#include "ocppo_common.h"
#include "ocppo_x6split.h"

namespace ocppo {

// Weight planes written by the step (ocppo_clip_adam_step's plane jobs): the new values of a
// row-major [R, C] weight at flat offset off (float4 units) as the three exact bf16 pieces
// ocppo_split_planes writes for it -- plane p at dst + p R C (bf16 units), [R, C] or, trans,
// [C, R] -- so the next minibatch's GEMMs read them without a split launch
constexpr int kAdamPlaneJobs = 8;
struct AdamPlanes {
  int n;
  int64_t off4[kAdamPlaneJobs];
  int64_t len4[kAdamPlaneJobs];
  int rows[kAdamPlaneJobs];
  int cols[kAdamPlaneJobs];
  int trans[kAdamPlaneJobs];
  uint16_t* dst[kAdamPlaneJobs];
};

__device__ __forceinline__ void adam_planes_store(const AdamPlanes& pl, int64_t i, float4 v) {
  for (int j = 0; j < pl.n; ++j) {
    const int64_t q = i - pl.off4[j];
    if (q >= 0 && q < pl.len4[j]) {
      uint32_t a0, a1, a2, b0, b1, b2;
      x6_split2(x6f2{v.x, v.y}, a0, a1, a2);
      x6_split2(x6f2{v.z, v.w}, b0, b1, b2);
      const int64_t ps = 4 * pl.len4[j];  // elements per plane
      if (!pl.trans[j]) {
        uint2* d = reinterpret_cast<uint2*>(pl.dst[j]);
        d[q] = uint2{a0, b0};
        d[ps / 4 + q] = uint2{a1, b1};
        d[ps / 2 + q] = uint2{a2, b2};
      } else {  // element (r, c .. c + 3) -> plane rows c .. c + 3, column r
        const int64_t e = 4 * q;
        const int64_t r = e / pl.cols[j], c = e - r * pl.cols[j];
        const int64_t R = pl.rows[j];
        uint16_t* d = pl.dst[j] + c * R + r;
        const uint32_t w[3][2] = {{a0, b0}, {a1, b1}, {a2, b2}};
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          uint16_t* dp = d + p * ps;
          dp[0] = static_cast<uint16_t>(w[p][0]);
          dp[R] = static_cast<uint16_t>(w[p][0] >> 16);
          dp[2 * R] = static_cast<uint16_t>(w[p][1]);
          dp[3 * R] = static_cast<uint16_t>(w[p][1] >> 16);
        }
      }
      return;
    }
  }
}

constexpr int kOptThreads = 256;
constexpr int kOptBlocks = 1024;  // grid-stride cap for the norm pass (4 workgroups per CU), at
                                  // most 1024 partials for every adam workgroup to combine

// scalars layout (f32): see include/ocppo.h OCPPO_OPT_*
enum { S_STEP = 0, S_TOTAL_NORM = 1, S_CLIP = 2, S_STEP_SIZE = 3, S_BC2_SQRT = 4 };

__global__ __launch_bounds__(kOptThreads) void grad_norm_kernel(
    const float* __restrict__ g, int64_t P, float grad_scale, float* __restrict__ scalars,
    float* __restrict__ partials) {
  __shared__ float red[kOptThreads / kWave];
  float acc = 0.f;
  const int64_t P4 = P / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kOptThreads;
  // kNormU grid-strided float4 loads in flight per thread, then accumulated in index order
  constexpr int kNormU = 4;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * kOptThreads + threadIdx.x; i0 < P4;
       i0 += kNormU * stride) {
    float4 x[kNormU];
#pragma unroll
    for (int u = 0; u < kNormU; ++u) {
      const int64_t i = i0 + u * stride;
      x[u] = i < P4 ? reinterpret_cast<const float4*>(g)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kNormU; ++u) {
      const float a = x[u].x * grad_scale, b = x[u].y * grad_scale, c = x[u].z * grad_scale,
                  d = x[u].w * grad_scale;
      acc += a * a + b * b + c * c + d * d;
    }
  }
  if (blockIdx.x == 0)
    for (int64_t i = 4 * P4 + threadIdx.x; i < P; i += kOptThreads) {
      const float a = g[i] * grad_scale;
      acc += a * a;
    }
  const float w = wave_sum(acc);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) red[wid] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = red[0];
    for (int k = 1; k < kOptThreads / kWave; ++k) s += red[k];
    partials[blockIdx.x] = s;
    if (blockIdx.x == 0) scalars[S_STEP] = scalars[S_STEP] + 1.f;
  }
}

// The step scalars from the norm kernel's partials, in every workgroup alike (fixed order: the
// partial of workgroup t in thread t, the wave sums, then the 4 waves in order)
struct AdamScalars {
  float clip, step_size, bc2_sqrt, total;
};
__device__ __forceinline__ AdamScalars adam_scalars(const float* __restrict__ partials, int nb,
                                                    float max_norm, const float* __restrict__ lr,
                                                    float beta1, float beta2,
                                                    const float* __restrict__ scalars) {
  __shared__ float red[kOptThreads / kWave];
  __shared__ AdamScalars sc;
  float t = 0.f;
  for (int b = threadIdx.x; b < nb; b += kOptThreads) t += partials[b];
  const float tw = wave_sum(t);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) red[wid] = tw;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = red[0];
    for (int k = 1; k < kOptThreads / kWave; ++k) s += red[k];
    const float total = sqrtf(s);
    float clip = 1.f;
    if (max_norm > 0.f) {
      clip = max_norm / (total + 1e-6f);
      clip = clip < 1.f ? clip : 1.f;
    }
    const float step = scalars[S_STEP];
    sc = AdamScalars{clip, lr[0] / (1.f - powf(beta1, step)), sqrtf(1.f - powf(beta2, step)),
                     total};
  }
  __syncthreads();
  return sc;
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1, float b2,
                                          float step_size, float bc2_sqrt, float eps) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p - step_size * m / denom;
}

__global__ __launch_bounds__(kOptThreads) void adam_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, int64_t P, float grad_scale, float b1, float b2, float eps,
    float max_norm, const float* __restrict__ lr, const float* __restrict__ partials, int nb,
    float* __restrict__ scalars, AdamPlanes planes) {
  // the first element group's loads are issued before the scalars are combined: their latency
  // hides the partials' combine (at config 2 every thread has about one group)
  const int64_t P4 = P / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kOptThreads;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kOptThreads + threadIdx.x;
  float4 pp{}, gg{}, mm{}, vv{};
  if (i < P4) {
    pp = reinterpret_cast<float4*>(p)[i];
    gg = reinterpret_cast<const float4*>(g)[i];
    mm = reinterpret_cast<float4*>(m)[i];
    vv = reinterpret_cast<float4*>(v)[i];
  }
  const AdamScalars sc = adam_scalars(partials, nb, max_norm, lr, b1, b2, scalars);
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the reported figures (read after the step)
    scalars[S_TOTAL_NORM] = sc.total;
    scalars[S_CLIP] = sc.clip;
    scalars[S_STEP_SIZE] = sc.step_size;
    scalars[S_BC2_SQRT] = sc.bc2_sqrt;
  }
  const float clip = sc.clip, step_size = sc.step_size, bc2_sqrt = sc.bc2_sqrt;
  for (; i < P4; i += stride) {
    adam_elem(pp.x, (gg.x * grad_scale) * clip, mm.x, vv.x, b1, b2, step_size, bc2_sqrt, eps);
    adam_elem(pp.y, (gg.y * grad_scale) * clip, mm.y, vv.y, b1, b2, step_size, bc2_sqrt, eps);
    adam_elem(pp.z, (gg.z * grad_scale) * clip, mm.z, vv.z, b1, b2, step_size, bc2_sqrt, eps);
    adam_elem(pp.w, (gg.w * grad_scale) * clip, mm.w, vv.w, b1, b2, step_size, bc2_sqrt, eps);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (planes.n) adam_planes_store(planes, i, pp);
    if (i + stride < P4) {
      pp = reinterpret_cast<float4*>(p)[i + stride];
      gg = reinterpret_cast<const float4*>(g)[i + stride];
      mm = reinterpret_cast<float4*>(m)[i + stride];
      vv = reinterpret_cast<float4*>(v)[i + stride];
    }
  }
  if (blockIdx.x == 0)
    for (int64_t i = 4 * P4 + threadIdx.x; i < P; i += kOptThreads)
      adam_elem(p[i], (g[i] * grad_scale) * clip, m[i], v[i], b1, b2, step_size, bc2_sqrt, eps);
}

}  // namespace ocppo

using namespace ocppo;

extern "C" size_t ocppo_clip_adam_workspace_bytes(int64_t P) {
  (void)P;
  return 256 + kOptBlocks * sizeof(float);
}

extern "C" int ocppo_clip_adam_step(ocppo_stream_t stream, float* params, const float* grads,
                                    float* exp_avg, float* exp_avg_sq, int64_t P, const float* lr,
                                    double beta1, double beta2, double eps, double grad_scale,
                                    double max_norm, float* scalars, void* workspace,
                                    size_t workspace_bytes, int n_planes,
                                    const int64_t* plane_offset, const int64_t* plane_rows,
                                    const int64_t* plane_cols, const int* plane_trans,
                                    void* const* plane_dst) {
  OCPPO_REQUIRE(P > 0, "ocppo_clip_adam_step: bad size P=%lld", (long long)P);
  AdamPlanes planes{};
  OCPPO_REQUIRE(n_planes >= 0 && n_planes <= kAdamPlaneJobs &&
                    (n_planes == 0 ||
                     (plane_offset && plane_rows && plane_cols && plane_trans && plane_dst)),
                "ocppo_clip_adam_step: n_planes=%d (0..%d) and its arrays", n_planes,
                kAdamPlaneJobs);
  planes.n = n_planes;
  for (int j = 0; j < n_planes; ++j) {
    const int64_t R = plane_rows[j], C = plane_cols[j];
    OCPPO_REQUIRE(plane_offset[j] >= 0 && plane_offset[j] % 4 == 0 && R >= 1 && C >= 4 &&
                      C % 4 == 0 && R <= INT32_MAX && C <= INT32_MAX &&
                      (plane_trans[j] ? R : C) % 8 == 0 && plane_offset[j] + R * C <= P &&
                      plane_dst[j] && reinterpret_cast<uintptr_t>(plane_dst[j]) % 16 == 0,
                  "ocppo_clip_adam_step: plane job %d (offset %lld, %lld x %lld, trans %d): "
                  "offset %% 4, cols %% 4, plane rows %% 8, inside P, 16-B aligned planes", j,
                  (long long)plane_offset[j], (long long)R, (long long)C, plane_trans[j]);
    planes.off4[j] = plane_offset[j] / 4;
    planes.len4[j] = R * C / 4;
    planes.rows[j] = static_cast<int>(R);
    planes.cols[j] = static_cast<int>(C);
    planes.trans[j] = plane_trans[j] ? 1 : 0;
    planes.dst[j] = static_cast<uint16_t*>(plane_dst[j]);
  }
  OCPPO_REQUIRE(params && grads && exp_avg && exp_avg_sq && lr && scalars,
                "ocppo_clip_adam_step: null pointer");
  OCPPO_REQUIRE((reinterpret_cast<uintptr_t>(params) | reinterpret_cast<uintptr_t>(grads) |
                 reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) %
                        16 == 0,
                "ocppo_clip_adam_step: buffers must be 16-byte aligned");
  if (!workspace || workspace_bytes < ocppo_clip_adam_workspace_bytes(P))
    return fail(OCPPO_E_WORKSPACE, "ocppo_clip_adam_step: workspace needs %zu bytes, got %zu",
                ocppo_clip_adam_workspace_bytes(P), workspace_bytes);
  char* ws = static_cast<char*>(workspace);
  float* partials = reinterpret_cast<float*>(ws + 256);
  int64_t nb = ceil_div(P / 4 > 0 ? P / 4 : 1, kOptThreads);
  nb = nb < kOptBlocks ? nb : kOptBlocks;
  clear_stale_error();
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(grad_norm_kernel, dim3(static_cast<unsigned>(nb)), dim3(kOptThreads), 0, s,
                     grads, P, static_cast<float>(grad_scale), scalars, partials);
  if (int rc = check_launch("ocppo_clip_adam_step/norm")) return rc;
  int64_t na = ceil_div(P / 4 > 0 ? P / 4 : 1, kOptThreads);
  na = na < 256 * 8 ? na : 256 * 8;
  hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(na)), dim3(kOptThreads), 0, s, params,
                     grads, exp_avg, exp_avg_sq, P, static_cast<float>(grad_scale),
                     static_cast<float>(beta1), static_cast<float>(beta2),
                     static_cast<float>(eps), static_cast<float>(max_norm), lr, partials,
                     static_cast<int>(nb), scalars, planes);
  return check_launch("ocppo_clip_adam_step/adam");
}
