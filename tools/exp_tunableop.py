"""Experiment: the fp32 GEMMs of one PPO iteration (config 2) under the default hipBLASLt
heuristic vs PyTorch TunableOp (which times every hipBLASLt/rocBLAS solution per shape).

    python tools/exp_tunableop.py            # default heuristic
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
        PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop.csv python tools/exp_tunableop.py
"""
import os

import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


tag = "tunable" if os.environ.get("PYTORCH_TUNABLEOP_ENABLED") == "1" else "default"
if os.environ.get("OCPPO_BLAS"):  # "cublas" = rocBLAS, "cublaslt" = hipBLASLt on ROCm
    torch.backends.cuda.preferred_blas_library(os.environ["OCPPO_BLAS"])
    tag = os.environ["OCPPO_BLAS"]
total = 0.0
# rollout (M = 128 envs): fwd only, 128 steps per iteration
for M, K, N, per_iter in [(128, 512, 1024, 128), (128, 1024, 512, 129), (128, 2048, 512, 129)]:
    x, w, b = (torch.randn(M, K, device=dev), torch.randn(N, K, device=dev),
               torch.randn(N, device=dev))
    t = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    total += t * per_iter
    print(f"[{tag}] rollout M={M} K={K} N={N} fwd {t:7.2f} us", flush=True)
# update: 16 minibatches; encoder rows 11520 (dedup capacity), decoder rows 4096
for M, K, N in [(11520, 256, 512), (11520, 512, 1024), (11520, 1024, 512), (4096, 2048, 512)]:
    x, w, b = (torch.randn(M, K, device=dev), torch.randn(N, K, device=dev),
               torch.randn(N, device=dev))
    gp = torch.randn(M, N, device=dev)
    dw = torch.empty(N, K, device=dev)
    s = 8 if M >= 8192 else 1
    tf = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    tx = timeit(lambda: gp.mm(w))
    if s > 1:
        tw = timeit(lambda: torch.sum(torch.bmm(gp.view(s, M // s, N).transpose(1, 2),
                                                x.view(s, M // s, K)), 0, out=dw))
    else:
        tw = timeit(lambda: torch.mm(gp.t(), x, out=dw))
    total += 16 * (tf + tx + tw)
    print(f"[{tag}] update M={M} K={K} N={N} fwd {tf:7.2f}  dX {tx:7.2f}  dW {tw:7.2f} us",
          flush=True)
print(f"[{tag}] total GEMM time per iteration (these shapes): {total / 1e3:.2f} ms", flush=True)
