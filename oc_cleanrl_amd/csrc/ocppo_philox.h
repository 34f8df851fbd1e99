// The Exp(1) draws of the reference's Categorical.sample, reproduced element by element inside
// the kernel that consumes them (no noise tensor, no generator launch per rollout step).
//
// The reference samples with Categorical(logits).sample() (cleanrl/architectures/ppo.py:92-94,
// called per step at cleanrl/ppo_atari_oc.py:505-506). In torch that is multinomial(probs, 1),
// whose one-sample path is argmax(probs / q) with q = empty_like(probs).exponential_(1, gen) on
// the default CUDA generator. On ROCm exponential_ runs ATen's
// distribution_elementwise_grid_stride_kernel (ATen/native/cuda/DistributionTemplates.h):
// 256-thread blocks, grid = min(ceil(numel / 256), CUs * (max threads per CU / 256)), thread idx
// seeds a Philox4x32-10 stream with (seed, subsequence = idx, offset = the generator's philox
// offset), draws float4 uniforms (hiprand_uniform4 = rocrand's philox4x32_10 + 2^-32 + v * 2^-32,
// in (0, 1]) and element li = idx + S * (4 r + i) (S = 256 * grid) takes component i of draw r;
// the transform (ATen/core/TransformationHelper.h, exponential, device branch) is
// -1 / lambda * (u >= 1 - eps/2 ? -eps/2 : __logf(u)). The generator's offset then advances by
// ((numel - 1) / (4 S) + 1) * 4 per call.
//
// torch_exponential() below restates exactly that per element, from (seed, offset, li, S): the
// Philox rounds (Salmon et al. 2011, the constants and counter/key layout of rocrand's
// philox4x32_10_engine: counter = (offset / 4 + r, subsequence), key = seed, 10 rounds),
// the uniform conversion and the transform, with the same f32 operations in the same order
// (tests/test_kernels_gpu.py: bitwise against torch's own exponential_ on the box).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace ocppo {

// Where a kernel's Exp(1) draws come from when it generates them itself: the rollout's (seed,
// offset) in device memory (so a captured graph reads the generator state of each replay), the
// offset of this launch's draws relative to it, and torch's grid stride S for a [numel] draw.
struct PhiloxNoise {
  const int64_t* state;  // device [seed, offset at the first draw of the rollout]; null: off
  int64_t step_offset;   // philox offset of this launch's draw relative to state[1]
  int64_t stride;        // S = 256 * grid of torch's launch for this draw's numel
};

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c.x;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c.z;
    c = make_uint4(static_cast<uint32_t>(p1 >> 32) ^ c.y ^ k.x, static_cast<uint32_t>(p1),
                   static_cast<uint32_t>(p0 >> 32) ^ c.w ^ k.y, static_cast<uint32_t>(p0));
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Philox block `blk` of subsequence `sub`: counter = (blk, sub) as two 64-bit halves (the low
// half never wraps at any offset a generator reaches, so no carry into the subsequence)
__device__ __forceinline__ uint4 philox_block(uint64_t seed, uint64_t sub, uint64_t blk) {
  const uint4 c = make_uint4(static_cast<uint32_t>(blk), static_cast<uint32_t>(blk >> 32),
                             static_cast<uint32_t>(sub), static_cast<uint32_t>(sub >> 32));
  return philox4x32_10(c, make_uint2(static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32)));
}

__device__ __forceinline__ float philox_uniform(uint32_t v) {
  constexpr float kInv32 = 2.3283064365386963e-10f;  // 2^-32 (rocrand's ROCRAND_2POW32_INV)
  return kInv32 + static_cast<float>(v) * kInv32;      // the product is exact: no rounding order
}

// Element li of torch.empty(numel).exponential_() drawn at generator (seed, offset) with grid
// stride S (numel enters only through S).
__device__ __forceinline__ float torch_exponential(uint64_t seed, uint64_t offset, int64_t li,
                                                   int64_t S) {
  // 32-bit quotient whenever the operands fit (a 64-bit division is a ~100-instruction routine
  // on the critical path of the sampling head): the same q either way
  const int64_t q = (li >> 31) == 0 && (S >> 31) == 0
                        ? static_cast<int64_t>(static_cast<uint32_t>(li) / static_cast<uint32_t>(S))
                        : li / S;
  const uint64_t idx = static_cast<uint64_t>(li - q * S);
  const uint64_t r = static_cast<uint64_t>(q >> 2);
  const int comp = static_cast<int>(q & 3);
  const uint64_t base = (offset >> 2) + r;
  const int sub = static_cast<int>(offset & 3);  // 0 for torch's own offsets (multiples of 4)
  const uint4 a = philox_block(seed, idx, base);
  uint32_t w[8] = {a.x, a.y, a.z, a.w, 0u, 0u, 0u, 0u};
  if (sub != 0) {  // rocrand4 with a partial first block: the next block's words follow
    const uint4 b = philox_block(seed, idx, base + 1);
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
  }
  const float u = philox_uniform(w[sub + comp]);
  constexpr float kHalfEps = 5.9604644775390625e-08f;  // numeric_limits<float>::epsilon() / 2
  const float lg = u >= 1.f - kHalfEps ? -kHalfEps : __logf(u);
  return -1.f * lg;  // static_cast<float>(-1.0) / lambda * log with lambda = 1
}

__device__ __forceinline__ float philox_noise(const PhiloxNoise& pn, int64_t li) {
  const uint64_t seed = static_cast<uint64_t>(pn.state[0]);
  const uint64_t off = static_cast<uint64_t>(pn.state[1] + pn.step_offset);
  return torch_exponential(seed, off, li, pn.stride);
}

}  // namespace ocppo
