"""Experiment: ocppo_gemm (hand-written f32 MFMA) vs torch/hipBLASLt at every GEMM of the PPObj
update (frame-dedup rows R = 11520, decoder rows D = 4096), each timed in a hipGraph of
back-to-back launches; correctness vs an f64 product.

    python tools/exp_gemm_update.py [--quick]
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from oc_cleanrl_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
R, D = 11520, 4096
QUICK = "--quick" in sys.argv


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
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3


def rel(a, ref):
    return float((a.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))


def emit(**kw):
    print(json.dumps(kw), flush=True)


TILES = (44, 42, 24, 22)
total_torch = total_best = 0.0
# forward: y = relu(x W^T + b)
for M, K, N in [(8192, 2048, 8192), (R, 256, 512), (R, 512, 1024), (R, 1024, 512), (D, 2048, 512)]:
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    ref = torch.relu(x.double() @ w.double().t() + b.double())
    t_torch = timeit(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    res = {}
    for tile in TILES:
        if M % (32 * (tile // 10)) or N % (32 * (tile % 10)):
            continue
        y = ops.linear_fwd(x, w, b, relu=True, tile=tile)
        err = rel(y, ref)
        res[tile] = (timeit(lambda: ops.linear_fwd(x, w, b, relu=True, out=y, tile=tile)), err)
    best = min(v[0] for v in res.values())
    fl = 2 * M * N * K
    if M != 8192:
        total_torch += t_torch
        total_best += best
    emit(kind="fwd", M=M, N=N, K=K, torch_us=round(t_torch, 2), torch_tf=round(fl / t_torch / 1e6, 1),
         ours={k: [round(v[0], 2), round(fl / v[0] / 1e6, 1), f"{v[1]:.1e}"] for k, v in res.items()},
         auto=ops.gemm_tile(M, N))
    del x, w, y, ref

# dX: dx = g W (and the masked form with the bias-gradient partials)
for M, N, K in [(D, 512, 2048), (R, 512, 1024), (R, 1024, 512), (R, 512, 256)]:
    g = torch.randn(M, N, device=dev)
    w = torch.randn(N, K, device=dev) / N ** 0.5
    mask = torch.relu(torch.randn(M, K, device=dev))
    ref = g.double() @ w.double()
    t_torch = timeit(lambda: g.mm(w))
    t_thr = timeit(lambda: torch.ops.aten.threshold_backward(ref.float(), mask, 0))
    res = {}
    for tile in TILES:
        if M % (32 * (tile // 10)) or K % (32 * (tile % 10)):
            continue
        y = ops.linear_dx(g, w, tile=tile)
        err = rel(y, ref)
        bm = 32 * (tile // 10)
        dbp = torch.empty(M // bm, K, device=dev)
        ym = ops.linear_dx(g, w, mask=mask, dbp=dbp, tile=tile)
        refm = torch.where(mask.double() > 0, ref, torch.zeros_like(ref))
        errm = max(rel(ym, refm), rel(dbp.sum(0), refm.sum(0)))
        res[tile] = (timeit(lambda: ops.linear_dx(g, w, out=y, tile=tile)),
                     timeit(lambda: ops.linear_dx(g, w, out=ym, mask=mask, dbp=dbp, tile=tile)),
                     err, errm)
    best = min(v[0] for v in res.values())
    fl = 2 * M * N * K
    total_torch += t_torch
    total_best += best
    emit(kind="dx", M=M, N=K, K=N, torch_us=round(t_torch, 2), torch_tf=round(fl / t_torch / 1e6, 1),
         threshold_bwd_us=round(t_thr, 2),
         ours={k: [round(v[0], 2), round(fl / v[0] / 1e6, 1), round(v[1], 2), f"{v[2]:.1e}",
                   f"{v[3]:.1e}"] for k, v in res.items()})
    del g, w, mask, ref

# dW: split-K partials of g^T x, summed
for rows, N, K, s_torch in [(D, 512, 2048, 8), (R, 512, 1024, 8), (R, 1024, 512, 8),
                            (R, 512, 256, 4)]:
    g = torch.randn(rows, N, device=dev)
    x = torch.relu(torch.randn(rows, K, device=dev))
    ref = g.double().t() @ x.double()
    t_torch = timeit(lambda: torch.bmm(g.view(s_torch, rows // s_torch, N).transpose(1, 2),
                                       x.view(s_torch, rows // s_torch, K)))
    t_sum = timeit(lambda: ops.sum_splits(torch.empty(s_torch, N, K, device=dev)))
    res = {}
    for S in (1, 2, 4, 8, 16):
        if rows % (32 * S):
            continue
        for tile in TILES:
            if N % (32 * (tile // 10)) or K % (32 * (tile % 10)):
                continue
            part = ops.linear_dw(g, x, S, tile=tile)
            err = rel(part.sum(0), ref)
            res[f"{S}/{tile}"] = (timeit(lambda: ops.linear_dw(g, x, S, out=part, tile=tile)), err)
    best = min(v[0] for v in res.values())
    fl = 2 * rows * N * K
    total_torch += t_torch
    total_best += best
    emit(kind="dw", rows=rows, N=N, K=K, torch_bmm_us=round(t_torch, 2), torch_splits=s_torch,
         sum_splits_us=round(t_sum, 2), torch_tf=round(fl / t_torch / 1e6, 1),
         ours={k: [round(v[0], 2), round(fl / v[0] / 1e6, 1), f"{v[1]:.1e}"]
               for k, v in sorted(res.items(), key=lambda kv: kv[1][0])[:6]})
    del g, x, ref
emit(kind="total", torch_us=round(total_torch, 1), ours_best_us=round(total_best, 1))
