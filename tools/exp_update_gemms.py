"""Experiment: every GEMM-shaped op of the PPObj update at the dedup shapes (encoder rows = 12288
capacity, decoder rows = M = 4096), each formulation timed in a hipGraph of back-to-back launches.

    python tools/exp_update_gemms.py [rows_enc] [rows_dec]
"""
import sys

import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)
R_ENC = int(sys.argv[1]) if len(sys.argv) > 1 else 12288
R_DEC = int(sys.argv[2]) if len(sys.argv) > 2 else 4096


def timeit(fn, reps=20):
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


shapes = [(R_ENC, 12, 256), (R_ENC, 256, 512), (R_ENC, 512, 1024), (R_ENC, 1024, 512),
          (R_DEC, 2048, 512)]
total_best = 0.0
for M, K, N in shapes:  # x [M, K], W [N, K], y/gp [M, N]
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev)
    b = torch.randn(N, device=dev)
    gp = torch.randn(M, N, device=dev)
    out = torch.relu(torch.randn(M, N, device=dev))
    ones = torch.ones(M, device=dev)
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    r = {}
    r["fwd addmm_relu"] = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    r["fwd mm"] = timeit(lambda: torch.mm(x, w.t()))
    r["thr_bwd"] = timeit(lambda: torch.ops.aten.threshold_backward(gp, out, 0))
    if K > 16:
        r["dX gp@W"] = timeit(lambda: gp.mm(w))
        r["dX (W^T gp^T)^T"] = timeit(lambda: w.t().mm(gp.t()).t())
    r["dW gp^T x"] = timeit(lambda: torch.mm(gp.t(), x, out=dw))
    r["dW (x^T gp)^T"] = timeit(lambda: torch.mm(x.t(), gp, out=dw.t()))
    for s in (2, 4, 8, 16, 32):
        if M % s == 0:
            r[f"dW splitK{s}"] = timeit(lambda s=s: torch.sum(torch.bmm(
                gp.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K)), 0, out=dw))
            r[f"dW splitK{s} bmm only"] = timeit(lambda s=s: torch.bmm(
                gp.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K)))
    r["db sum0"] = timeit(lambda: torch.sum(gp, 0, out=db))
    r["db mv"] = timeit(lambda: torch.mv(gp.t(), ones, out=db))
    fl = 2 * M * K * N / 1e12
    print(f"\nM={M} K={K} N={N} ({fl * 1e3:.2f} GFLOP per GEMM)")
    for k, v in r.items():
        tf = "" if k.startswith(("db", "thr")) or "bmm only" in k else f" {fl / (v * 1e-6):6.1f} TF"
        print(f"  {k:24s} {v:8.1f} us{tf}", flush=True)
