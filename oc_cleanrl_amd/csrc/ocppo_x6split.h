// The exact three-way bf16 split of f32 values the update GEMMs (ocppo_gemm.hip) stage their
// operands with, shared with the optimizer's plane writes (ocppo_optim.hip: the weights' planes
// written by the Adam step that produced them).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ocppo {

// The three bf16 pieces of an f32 pair (exact: x == x0 + x1 + x2 for finite normal x), packed:
// p_i = (x_i of a) | (x_i of b) << 16 (5 v_cvt_pk_bf16_f32, 4 scalar f32 subtractions and 2
// v_perm_b32 per pair).
typedef float x6f2 __attribute__((ext_vector_type(2)));
typedef __bf16 x6h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t x6_pk(x6f2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, x6h2));
}
__device__ __forceinline__ x6f2 x6_unpk(uint32_t p) {
  return x6f2{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}
// PROBE (probe builds only, tools/build_variant.py -DOCPPO_X6_PROBE_NOSPLIT[_B]): the same LDS
// traffic with 2 VALU per pair instead of 9 -- wrong products, the main loop's cost without the
// split (of both operands, or of B only)
template <bool PROBE = false>
__device__ __forceinline__ void x6_split2(x6f2 v, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  if constexpr (PROBE) {
    const uint32_t ua = __float_as_uint(v.x), ub = __float_as_uint(v.y);
    p0 = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
    p1 = __builtin_amdgcn_perm(ub, ua, 0x05040100u);
    p2 = p1;
    return;
  }
  // the residuals as scalar subtractions (build.py: -fno-slp-vectorize keeps them apart): a
  // packed f32 VALU op issued beside MFMAs costs more than two scalar ones (MI355X_MICROARCH.md,
  // filler prices) -- config-2 shapes 730 -> 704 us, bench +2.4 % (profiles/r04/exp_x6_scalar_sub)
  // each lead piece as an f32 straight from the converter (bf16(0) in the low half: the register
  // IS the rounded value) instead of unpacked from the packed pair by a shift and a mask; the
  // packed planes words by one byte permute (GEMM set 676 -> 673 us, profiles/r04/exp_x6_split)
  const float h0x = __uint_as_float(x6_pk(x6f2{0.f, v.x}));
  const float h0y = __uint_as_float(x6_pk(x6f2{0.f, v.y}));
  const float r1x = v.x - h0x, r1y = v.y - h0y;
  const float h1x = __uint_as_float(x6_pk(x6f2{0.f, r1x}));
  const float h1y = __uint_as_float(x6_pk(x6f2{0.f, r1y}));
  p0 = __builtin_amdgcn_perm(__float_as_uint(h0y), __float_as_uint(h0x), 0x07060302u);
  p1 = __builtin_amdgcn_perm(__float_as_uint(h1y), __float_as_uint(h1x), 0x07060302u);
  p2 = x6_pk(x6f2{r1x - h1x, r1y - h1y});
}

}  // namespace ocppo
