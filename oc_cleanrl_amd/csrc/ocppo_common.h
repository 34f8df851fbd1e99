// Shared helpers of libocppo_hip.so (gfx950 only): error reporting across the C-ABI, element
// conversions, wave/block reductions with a fixed combination order (determinism), and launch
// checks. Every kernel in this library is compiled with -ffp-contract=off so that f32 arithmetic
// keeps PyTorch's per-op rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/ocppo.h"

namespace ocppo {

// ---- error state (thread-local, read through ocppo_last_error) -------------------------------
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define OCPPO_REQUIRE(cond, ...)                                   \
  do {                                                             \
    if (!(cond)) return ::ocppo::fail(OCPPO_E_INVALID, __VA_ARGS__); \
  } while (0)

// hipGetLastError() reports the last error of ANY runtime call on this thread (e.g. a benign
// failed query inside torch). Clear it before our launches so check_launch sees only ours.
inline void clear_stale_error() { (void)hipGetLastError(); }

// Check the launch that was just issued (also valid while the stream is being captured).
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(OCPPO_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
  return OCPPO_OK;
}

inline hipStream_t as_stream(ocppo_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr int kWave = 64;  // CDNA wavefront width
// The first-layer weight-gradient record layout (relu_bias_wgrad's rows kernel and gemm_x6's
// wgrad epilogue write it, relu_bias_wgrad's finish reads it): per row range, for each group of
// kWgRecCols columns, [value v][column] with v = 0 the bias gradient and v = 1..K the weight
// columns, K padded to wg_kp(K)
constexpr int kWgRecCols = 256;
__host__ __device__ inline int wg_kp(int64_t K) { return K <= 4 ? 4 : K <= 8 ? 8 : K <= 12 ? 12 : 16; }

// ReLU as torch computes it (clamp_min: NaN propagates). v_max_f32 alone returns the non-NaN
// operand, which would clamp a diverging layer's NaNs to 0 instead of surfacing them in the loss;
// for every non-NaN input the result is fmaxf's, bit for bit.
__device__ __forceinline__ float relu_f(float v) { return v != v ? v : fmaxf(v, 0.f); }
__device__ __forceinline__ float4 relu_f4(float4 v) {
  return make_float4(relu_f(v.x), relu_f(v.y), relu_f(v.z), relu_f(v.w));
}

// ---- element conversions ----------------------------------------------------------------------
// f32 -> bf16 round-to-nearest-even through the hardware converter (NaN stays NaN).
__device__ __forceinline__ uint16_t f32_to_bf16(float x) {
  __bf16 h = static_cast<__bf16>(x);
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t u) {
  return __uint_as_float(static_cast<uint32_t>(u) << 16);
}

template <int DT> struct Elem;
template <> struct Elem<OCPPO_F32> {
  using T = float;
  __device__ static float load(const T* p, int64_t i) { return p[i]; }
  __device__ static void store(T* p, int64_t i, float v) { p[i] = v; }
  __device__ static float roundtrip(float v) { return v; }
};
template <> struct Elem<OCPPO_BF16> {
  using T = uint16_t;
  __device__ static float load(const T* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ static void store(T* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
  __device__ static float roundtrip(float v) { return bf16_to_f32(f32_to_bf16(v)); }
};
template <> struct Elem<OCPPO_U8> {
  using T = uint8_t;
  __device__ static float load(const T* p, int64_t i) { return static_cast<float>(p[i]); }
  // values are integers in [0, 255] on this path; saturate anything else
  __device__ static void store(T* p, int64_t i, float v) {
    v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
    p[i] = static_cast<uint8_t>(__float2int_rn(v));
  }
  __device__ static float roundtrip(float v) {
    v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
    return static_cast<float>(__float2int_rn(v));
  }
};

// ---- vector element I/O: VEC elements of dtype DT as one aligned access -----------------------
template <int DT, int VEC> struct VecIO {
  // generic fallback (VEC == 1 or unaligned sizes)
  __device__ static void load(const void* p, int64_t i, float (&v)[VEC]) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) v[k] = Elem<DT>::load(static_cast<const typename Elem<DT>::T*>(p), i + k);
  }
  __device__ static void store(void* p, int64_t i, const float (&v)[VEC]) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) Elem<DT>::store(static_cast<typename Elem<DT>::T*>(p), i + k, v[k]);
  }
};
template <> struct VecIO<OCPPO_F32, 4> {
  __device__ static void load(const void* p, int64_t i, float (&v)[4]) {
    const float4 x = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  __device__ static void store(void* p, int64_t i, const float (&v)[4]) {
    *reinterpret_cast<float4*>(static_cast<float*>(p) + i) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct VecIO<OCPPO_BF16, 4> {
  __device__ static void load(const void* p, int64_t i, float (&v)[4]) {
    const uint2 x = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xFFFF0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xFFFF0000u);
  }
  __device__ static void store(void* p, int64_t i, const float (&v)[4]) {
    uint2 x;
    x.x = static_cast<uint32_t>(f32_to_bf16(v[0])) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
    x.y = static_cast<uint32_t>(f32_to_bf16(v[2])) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p) + i) = x;
  }
};
template <> struct VecIO<OCPPO_U8, 4> {
  __device__ static void load(const void* p, int64_t i, float (&v)[4]) {
    const uint32_t x = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(p) + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = static_cast<float>((x >> (8 * k)) & 0xFFu);
  }
  __device__ static void store(void* p, int64_t i, const float (&v)[4]) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float f = v[k] < 0.f ? 0.f : (v[k] > 255.f ? 255.f : v[k]);
      x |= static_cast<uint32_t>(__float2int_rn(f)) << (8 * k);
    }
    *reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(p) + i) = x;
  }
};

inline int grid_for(int64_t work, int block) {
  int64_t g = ceil_div(work, block);
  const int64_t cap = 256 * 16;  // 256 CUs x 16 blocks: grid-stride beyond that
  return static_cast<int>(g < cap ? (g > 0 ? g : 1) : cap);
}

// ---- deterministic reductions -----------------------------------------------------------------
// Butterfly over the 64 lanes: every lane ends with the same value, combined in a fixed order.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Block-wide sum of one value per thread (blockDim.x a multiple of 64, <= 1024). `scratch` holds
// at least blockDim.x/64 elements. Result valid in every thread. Fixed order: lanes by butterfly,
// then waves 0..nw-1 sequentially.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  const int nw = blockDim.x / kWave;
  v = wave_sum(v);
  __syncthreads();  // scratch may still be read by a previous call
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T r = scratch[0];
  for (int w = 1; w < nw; ++w) r += scratch[w];
  return r;
}

// ---- two-level last-block hand-off -------------------------------------------------------------
// A grid-wide reduction of NP per-block partials without a second launch. Blocks arrive on one of
// G = ceil(nb / 32) group tickets (one 128-B line each, so arrivals on any one address stay <= 32
// instead of nb); the last block of a group combines its group's partials and arrives on the
// global ticket; the last group's combiner produces the total. Every hand-off follows
// MI355X_MICROARCH.md "Valid forms" row 1: write-through (sc1) stores, drained with
// s_waitcnt vmcnt(0), then ONE agent-scope relaxed atomic; the receiver reads with sc1 loads.
// No release/acquire fence, so the block's other dirty lines are not written back here.
// Tickets re-arm themselves (graph replay). Sums run over lanes by a fixed butterfly, so the
// result is deterministic for a given grid.
constexpr int kHandoffGroup = 32;
constexpr int kHandoffMaxGroups = 256;  // nb <= 8192
constexpr int kHandoffMaxBlocks = kHandoffGroup * kHandoffMaxGroups;
constexpr int kTicketStride = 32;      // unsigned per 128-B line
constexpr size_t kHandoffTicketBytes = (1 + kHandoffMaxGroups) * kTicketStride * sizeof(unsigned);

// Call from every thread of the block; `mine` must be valid in thread 0. Returns true (in every
// thread) only in the final block, where `total` is valid in threads 0..63.
template <int NP>
__device__ __forceinline__ bool handoff_combine(const float (&mine)[NP], unsigned* tickets,
                                                float* partials, float* gpartials,
                                                float (&total)[NP], int* s_flag) {
  const unsigned nb = gridDim.x, b = blockIdx.x;
  const unsigned g = b / kHandoffGroup, G = (nb + kHandoffGroup - 1) / kHandoffGroup;
  const unsigned gsize = (nb - g * kHandoffGroup) < kHandoffGroup ? (nb - g * kHandoffGroup)
                                                                   : kHandoffGroup;
  unsigned* gt = tickets + (1 + g) * kTicketStride;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NP; ++k)
      __hip_atomic_store(&partials[b * NP + k], mine[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = prev == gsize - 1;
  }
  __syncthreads();
  if (!*s_flag) return false;
  __syncthreads();  // everyone has read the flag before thread 0 reuses it
  if (threadIdx.x < kWave) {
    const unsigned lane = threadIdx.x;
    float v[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k)
      v[k] = lane < gsize ? __hip_atomic_load(&partials[(g * kHandoffGroup + lane) * NP + k],
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : 0.f;
#pragma unroll
    for (int k = 0; k < NP; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
      __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm group
#pragma unroll
      for (int k = 0; k < NP; ++k)
        __hip_atomic_store(&gpartials[g * NP + k], v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev =
          __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = prev == G - 1;
    }
  }
  __syncthreads();
  if (!*s_flag) return false;
  if (threadIdx.x < kWave) {
    const unsigned lane = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      float v = 0.f;  // group partials lane, lane + 64, ... in a fixed order
      for (unsigned q = lane; q < G; q += kWave)
        v += __hip_atomic_load(&gpartials[q * NP + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      total[k] = wave_sum(v);
    }
    if (lane == 0) __hip_atomic_store(tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

}  // namespace ocppo
