import torch, json
dev = torch.device("cuda:0")
def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s): fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); g.replay(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3
for rows, k, n in [(128, 256, 512), (128, 512, 1024), (128, 1024, 512), (32, 2048, 512)]:
    x = torch.randn(rows, k, device=dev); g = torch.randn(rows, n, device=dev); w = torch.randn(n, k, device=dev)
    dw = torch.empty(n, k, device=dev); b = torch.randn(n, device=dev)
    r = {"fwd": timeit(lambda: torch._addmm_activation(b, x, w.t())),
         "dX": timeit(lambda: g.mm(w)),
         "dW mm": timeit(lambda: torch.mm(g.t(), x, out=dw)),
         "dW (x^T g)^T": timeit(lambda: torch.mm(x.t(), g, out=dw.t())),
         "dW bmm4": timeit(lambda: torch.bmm(g.view(4, rows // 4, n).transpose(1, 2), x.view(4, rows // 4, k)))}
    print(json.dumps({"rows": rows, "k": k, "n": n, **{a: round(v, 2) for a, v in r.items()}}), flush=True)

import sys
sys.path.insert(0, ".")
from oc_cleanrl_amd import ops  # noqa: E402
for rows, k, n in [(128, 256, 512), (128, 512, 1024), (128, 1024, 512), (32, 2048, 512)]:
    g = torch.randn(rows, n, device=dev); w = torch.randn(n, k, device=dev)
    wt = w.t().contiguous()
    r = {"dX": timeit(lambda: g.mm(w)),
         "dX^T^T": timeit(lambda: torch.mm(w.t(), g.t()).t().contiguous()),
         "wT copy": timeit(lambda: wt.copy_(w.t())),
         "dX hip linear(g, W^T)": timeit(lambda: ops.linear_act(g, wt)),
         "dX matmul(g, wt.t())": timeit(lambda: torch.mm(g, wt.t()))}
    print(json.dumps({"rows": rows, "k": k, "n": n, **{a: round(v, 2) for a, v in r.items()}}), flush=True)
