"""ocppo_gemm_x6 (f32 GEMM as six bf16 piece products) vs hipBLASLt's f32 GEMM at the config-2
update shapes: error against an f64 product and device time per call, every tile config.

    python tools/exp_gemm_x6.py [--reps 20] [--out gpurun_out/exp_gemm_x6.jsonl]

Error = max over the output of |C - C64| / (|A| |B|)[m, n] (the f64 product of the absolute
operands: the scale an f32 dot product's rounding error is bounded by).
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import ops  # noqa: E402

# (kind, M, N, K): fwd y[M,N] = x[M,K] W[N,K]^T; dx dX[M,K] = g[M,N] W[N,K]; dw dW[N,K] = g[R,N]^T x[R,K]
SHAPES = [
    ("fwd", 11520, 512, 256), ("fwd", 11520, 1024, 512), ("fwd", 11520, 512, 1024), ("fwd", 4096, 512, 2048),
    ("dx", 4096, 512, 2048), ("dx", 11520, 512, 1024), ("dx", 11520, 1024, 512), ("dx", 11520, 512, 256),
    ("dw", 4096, 512, 2048), ("dw", 11520, 512, 1024), ("dw", 11520, 1024, 512), ("dw", 11520, 512, 256),
]


def dev_time_us(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000 / reps)
    return best


def err(c, ref, scale):
    d = (c.double() - ref).abs() / scale.clamp_min(1e-300)
    return float(d.max()), float(d.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="kind,M,N,K: one shape (profiling)")
    ap.add_argument("--tiles", default=None, help="comma-separated variants (default: all built)")
    ap.add_argument("--stream-k", action="store_true",
                    help="fwd / dx on tiles 57 / 58: the persistent stream-K launch")
    ap.add_argument("--planes", action="store_true",
                    help="fwd / dx: B as pre-split bf16 planes (ops.WeightPlanes' operand)")
    ap.add_argument("--mbig", type=int, default=None,
                    help="rows in 128 x 128 tiles for the mixed variant (ocppo_gemm_x6's mbig)")
    a = ap.parse_args()
    if a.mbig is not None:
        # every mixed-variant ops.gemm_x6 call of this run with the given split
        _gemm_x6 = ops.gemm_x6

        def _with_mbig(*args, **kw):
            if kw.get("tile") == ops.X6_MIXED:
                kw["mbig"] = a.mbig
            return _gemm_x6(*args, **kw)
        ops.gemm_x6 = _with_mbig
    shapes = SHAPES
    if a.only:
        k, *dims = a.only.split(",")
        shapes = [(k, *map(int, dims))]
    tiles = [int(t) for t in a.tiles.split(",")] if a.tiles else list(ops.X6_BUILT)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    lines = []
    tot_torch, tot_best = 0.0, 0.0
    for kind, M, N, K in shapes:
        flops = 2.0 * M * N * K
        if kind == "fwd":
            x = torch.rand(M, K, device=dev, generator=g) * 2 - 1
            w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5
            ref = x.double() @ w.double().t()
            scale = x.double().abs() @ w.double().abs().t()
            tfn = lambda: torch.mm(x, w.t())  # noqa: E731
            out = torch.empty(M, N, device=dev)
            pl = ops.split_planes_ref(w).contiguous() if a.planes else None
            ofn = lambda t: (lambda: ops.gemm_x6(x, K, 1, w, K, 1, out, N, M, N, K, tile=t,  # noqa: E731
                                                 b_planes=pl, stream_k=a.stream_k and t in (57, 58)))
            shape_ok = lambda t: ops.x6_tile(M, N, 1, t) is not None  # noqa: E731
        elif kind == "dx":
            gg = torch.rand(M, N, device=dev, generator=g) * 2 - 1
            w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5
            ref = gg.double() @ w.double()
            scale = gg.double().abs() @ w.double().abs()
            tfn = lambda: torch.mm(gg, w)  # noqa: E731
            out = torch.empty(M, K, device=dev)
            plt = ops.split_planes_ref(w.t().contiguous()).contiguous() if a.planes else None
            ofn = lambda t: (lambda: ops.gemm_x6(gg, N, 1, w, 1, K, out, K, M, K, N, tile=t,  # noqa: E731
                                                 b_planes=plt, stream_k=a.stream_k and t in (57, 58)))
            shape_ok = lambda t: ops.x6_tile(M, K, 1, t) is not None  # noqa: E731
        else:
            R = M
            gg = torch.rand(R, N, device=dev, generator=g) * 2 - 1
            x = torch.rand(R, K, device=dev, generator=g) * 2 - 1
            ref = gg.double().t() @ x.double()
            scale = gg.double().abs().t() @ x.double().abs()
            S = 16
            tfn = lambda: torch.bmm(gg.view(S, R // S, N).transpose(1, 2), x.view(S, R // S, K)).sum(0)  # noqa: E731
            part = torch.empty(S, N, K, device=dev)
            out = torch.empty(N, K, device=dev)

            def ofn(t, S=S, part=part, out=out, gg=gg, x=x, R=R, N=N, K=K):
                def f():
                    ops.gemm_x6(gg, 1, N, x, 1, K, part, K, N, K, R, splits=S, split_c=N * K,
                                tile=t)
                    ops.sum_splits(part, out)
                return f
            shape_ok = lambda t: ops.x6_tile(N, K, S, t) is not None  # noqa: E731
        if a.mbig is not None:  # the mixed split must fit the output [rows, cols]
            rows, cols = (M, N) if kind == "fwd" else (M, K)
            if (not shape_ok(ops.X6_MIXED) or a.mbig > rows
                    or (a.mbig // 128) * (cols // 128) % 8):
                continue
        ct = tfn()
        torch.cuda.synchronize()
        t_err = err(ct, ref, scale)
        t_us = dev_time_us(tfn, a.reps)
        # the library's own bf16 GEMM of the same shape (one product, bf16 out): the efficiency
        # a plain bf16 GEMM reaches here, x6 issues six of them
        xa = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        xb = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        b16_us = dev_time_us(lambda: torch.mm(xa, xb.t()), a.reps)
        rec = {"kind": kind, "M": M, "N": N, "K": K, "torch_us": round(t_us, 2),
               "torch_tf": round(flops / t_us / 1e6, 1), "torch_err": t_err,
               "bf16_lib_us": round(b16_us, 2), "bf16_lib_tf": round(flops / b16_us / 1e6, 1),
               "ours": {}}
        best = None
        for t in tiles:
            if not shape_ok(t):
                continue
            f = ofn(t)
            f()
            torch.cuda.synchronize()
            e = err(out, ref, scale)
            us = dev_time_us(f, a.reps)
            rec["ours"][str(t)] = [round(us, 2), round(flops / us / 1e6, 1), e]
            if best is None or us < best:
                best = us
        rec["best_us"] = round(best, 2)
        tot_torch += t_us
        tot_best += best
        print(json.dumps(rec), flush=True)
        lines.append(rec)
    tot = {"kind": "total", "torch_us": round(tot_torch, 1), "ours_best_us": round(tot_best, 1)}
    print(json.dumps(tot), flush=True)
    lines.append(tot)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        with open(a.out, "w") as fh:
            for r in lines:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
