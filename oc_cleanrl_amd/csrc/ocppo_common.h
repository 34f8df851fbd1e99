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

}  // namespace ocppo
