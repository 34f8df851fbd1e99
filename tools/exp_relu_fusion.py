"""Experiment: does torch._addmm_activation (GEMM + bias + ReLU epilogue) fuse on ROCm/gfx950,
is it differentiable, and what does it save on PPObj shapes (fwd and fwd+bwd, graph-timed)?"""
import torch
import torch.nn.functional as F

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


dims = [(12, 256), (256, 512), (512, 1024), (1024, 512)]
Ws = [(torch.randn(o, i, device=dev) * 0.05).requires_grad_() for i, o in dims]
Bs = [torch.zeros(o, device=dev).requires_grad_() for i, o in dims]
Wd = (torch.randn(512, 2048, device=dev) * 0.02).requires_grad_()
Bd = torch.zeros(512, device=dev).requires_grad_()
for B in (128, 4096):
    x = torch.randint(0, 160, (B * 4, 12), device=dev).float()

    def plain(grad):
        h = x
        for w, b in zip(Ws, Bs):
            h = F.relu(F.linear(h, w, b))
        h = F.relu(F.linear(h.reshape(B, 2048), Wd, Bd))
        if grad:
            h.sum().backward()
        return h

    def fused(grad):
        h = x
        for w, b in zip(Ws, Bs):
            h = torch._addmm_activation(b, h, w.t(), use_gelu=False)
        h = torch._addmm_activation(Bd, h.reshape(B, 2048), Wd.t(), use_gelu=False)
        if grad:
            h.sum().backward()
        return h

    with torch.no_grad():
        d = (plain(False) - fused(False)).abs().max().item()
    print(f"B={B} max|plain-fused| = {d:.3e}")
    for grad in (False, True):
        ctx = torch.enable_grad() if grad else torch.no_grad()
        with ctx:
            tp = timeit(lambda: plain(grad))
            tf = timeit(lambda: fused(grad))
        print(f"B={B} grad={grad}: plain {tp:8.1f} us  fused {tf:8.1f} us")
