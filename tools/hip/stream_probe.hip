// Bandwidth probe: how fast can gfx950 stream S read arrays and W write arrays of float4 per lane
// (grid-stride, 256-thread blocks)? Calibrates the achievable ceiling for the multi-stream
// kernels of libocppo_hip.so (the fused loss reads 7 arrays and writes 2).
//   hipcc -O3 --offload-arch=gfx950 tools/hip/stream_probe.hip -o tools/hip/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <int S, int W>
__global__ __launch_bounds__(256) void probe(const float4* const* __restrict__ in, float4* const* __restrict__ out,
                                             const int* __restrict__ in_len, const int* __restrict__ out_len,
                                             long n_units) {
  // one "unit" = one float4 of every stream scaled by its relative length (len in float4 per unit)
  const long stride = (long)gridDim.x * blockDim.x;
  for (long u = (long)blockIdx.x * blockDim.x + threadIdx.x; u < n_units; u += stride) {
    float4 acc = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < S; ++s)
      for (int k = 0; k < in_len[s]; ++k) {
        float4 v = in[s][(long)k * n_units + u];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
#pragma unroll
    for (int w = 0; w < W; ++w)
      for (int k = 0; k < out_len[w]; ++k) out[w][(long)k * n_units + u] = acc;
  }
}

template <int S, int W>
void run(const char* name, std::vector<int> il, std::vector<int> ol, long units, int grid) {
  std::vector<float4*> ins(S), outs(W);
  long bytes = 0;
  for (int s = 0; s < S; ++s) { CK(hipMalloc(&ins[s], 16L * il[s] * units)); CK(hipMemset(ins[s], 0, 16L * il[s] * units)); bytes += 16L * il[s] * units; }
  for (int w = 0; w < W; ++w) { CK(hipMalloc(&outs[w], 16L * ol[w] * units)); bytes += 16L * ol[w] * units; }
  float4 **din, **dout; int *dil, *dol;
  CK(hipMalloc(&din, sizeof(void*) * S)); CK(hipMalloc(&dout, sizeof(void*) * W));
  CK(hipMalloc(&dil, 4 * S)); CK(hipMalloc(&dol, 4 * W));
  CK(hipMemcpy(din, ins.data(), sizeof(void*) * S, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, outs.data(), sizeof(void*) * W, hipMemcpyHostToDevice));
  CK(hipMemcpy(dil, il.data(), 4 * S, hipMemcpyHostToDevice));
  CK(hipMemcpy(dol, ol.data(), 4 * W, hipMemcpyHostToDevice));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((probe<S, W>), dim3(grid), dim3(256), 0, 0, din, dout, dil, dol, units);
  const int reps = 20;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((probe<S, W>), dim3(grid), dim3(256), 0, 0, din, dout, dil, dol, units);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  const double us = 1e3 * ms / reps;
  printf("{\"probe\": \"%s\", \"grid\": %d, \"MB\": %.1f, \"us\": %.2f, \"GBps\": %.1f}\n", name, grid, bytes / 1e6, us, bytes / us / 1e3);
  for (auto p : ins) CK(hipFree(p));
  for (auto p : outs) CK(hipFree(p));
  CK(hipFree(din)); CK(hipFree(dout)); CK(hipFree(dil)); CK(hipFree(dol));
}

int main() {
  // fused-loss shape at A=6 with M=4M elements: per 4 elements (one float4 "unit" = 4 elements):
  // reads actions 2 units, logits 6, lp/adv/ret/val/newv 1 each; writes dlogits 6, dv 1
  const long units = 1L << 20;  // 4M elements
  for (int grid : {1024, 2048, 4096}) {
    run<1, 1>("copy 1r1w (13:7 bytes as one stream each)", {13}, {7}, units, grid);
    run<7, 2>("loss-shaped 7r2w", {2, 6, 1, 1, 1, 1, 1}, {6, 1}, units, grid);
    run<2, 2>("records AoS 2r(+logits) 2w", {7, 6}, {6, 1}, units, grid);
    run<3, 2>("gae-shaped 3r2w", {1, 1, 1}, {1, 1}, units * 4, grid);
  }
  return 0;
}
