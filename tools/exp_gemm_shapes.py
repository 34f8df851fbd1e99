"""Experiment: backward GEMM formulations for the PPObj update shapes (M = 4096 x 4 frames)."""
import os
import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
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


shapes = [(16384, 12, 256), (16384, 256, 512), (16384, 512, 1024), (16384, 1024, 512),
          (4096, 2048, 512), (4096, 512, 6), (4096, 512, 1)]
print("tunableop", os.environ.get("PYTORCH_TUNABLEOP_ENABLED"))
for M, K, N in shapes:  # x [M, K], W [N, K], gp [M, N]
    x = torch.randn(M, K, device=dev)
    gp = torch.randn(M, N, device=dev)
    w = torch.randn(N, K, device=dev)
    ones = torch.ones(M, device=dev)
    dw = torch.empty(N, K, device=dev)
    r = {}
    r["dW=gp^T x"] = timeit(lambda: gp.t().mm(x))
    r["dW=(x^T gp)^T"] = timeit(lambda: x.t().mm(gp).t())
    for s in (4, 8, 16):
        if M % s == 0:
            r[f"splitK{s}"] = timeit(lambda s=s: torch.bmm(gp.view(s, M // s, N).transpose(1, 2),
                                                           x.view(s, M // s, K)).sum(0))
    r["dX=gp W"] = timeit(lambda: gp.mm(w))
    r["fwd x W^T"] = timeit(lambda: x.mm(w.t()))
    r["db=sum0"] = timeit(lambda: gp.sum(0))
    r["db=mv"] = timeit(lambda: gp.t().mv(ones))
    fl = 2 * M * K * N / 1e12
    print(f"M={M} K={K} N={N}: " + "  ".join(f"{k} {v:.1f}us({fl/(v*1e-6):.0f}TF)" if 'db' not in k else f"{k} {v:.1f}us" for k, v in r.items()), flush=True)
