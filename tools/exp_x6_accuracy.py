"""Accuracy of the update GEMMs on gradient-like operands (experiment, not a test).

The config-2 golden's f64 twin showed the x6 chain's encoder gradients 1e-5..1e-4 of their largest
element off f64, against the f32 reference's own 1e-7..2e-6. Random [-1, 1) operands (the GEMM
tests) hide what matters for gradients: heavy cancellation, where an error that scales with
sum |a b| (not with the running partial sums) or a biased rounding dominates. Here, per variant:
  err_max  = max |C - C64| / max |C64|        (what the golden measures)
  err_sab  = max |C - C64| / (|A| |B|)        (the GEMM tests' yardstick)
  bias     = mean(sign(C64) (C - C64)) / mean |C - C64|   (0: unbiased; -1: always toward zero)

    python tools/exp_x6_accuracy.py > gpurun_out/x6_acc.jsonl
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import ops  # noqa: E402

DEV = torch.device("cuda:0")


def stats(c, ref, sab):
    d = c.double() - ref
    return {"err_max": float(d.abs().max() / ref.abs().max()),
            "err_sab": float((d.abs() / sab.clamp_min(1e-300)).max()),
            "bias": float((torch.sign(ref) * d).mean() / d.abs().mean().clamp_min(1e-300))}


def case_dw(g, x, S, variants):
    R, N = g.shape
    K = x.shape[1]
    ref = g.double().t() @ x.double()
    sab = g.double().abs().t() @ x.double().abs()
    out = {"hipblaslt_mm": stats(g.t() @ x, ref, sab)}
    part = torch.empty(S, N, K, device=DEV)
    c = torch.empty(N, K, device=DEV)
    for t in variants:
        if ops.x6_tile(N, K, S, t) is None:
            continue
        ops.gemm_x6(g, 1, N, x, 1, K, part, K, N, K, R, splits=S, split_c=N * K, tile=t)
        ops.sum_splits(part, c)
        out[f"x6_{t}"] = stats(c, ref, sab)
    return out


def case_dx(g, w, variants):
    M, N = g.shape
    K = w.shape[1]
    ref = g.double() @ w.double()
    sab = g.double().abs() @ w.double().abs()
    out = {"hipblaslt_mm": stats(g @ w, ref, sab)}
    c = torch.empty(M, K, device=DEV)
    for t in variants:
        if ops.x6_tile(M, K, 1, t) is None:
            continue
        ops.gemm_x6(g, N, 1, w, 1, K, c, K, M, K, N, tile=t)
        out[f"x6_{t}"] = stats(c, ref, sab)
    return out


def main():
    gen = torch.Generator(device=DEV).manual_seed(0)
    variants = [0, 24, 56]
    R = 11520
    # dW of a 512 -> 1024 layer: g' = upstream gradient masked by the layer's ReLU (zero mean),
    # x = the layer's input (a ReLU output: nonnegative)
    g = torch.randn(R, 1024, device=DEV, generator=gen) * 1e-3
    g *= torch.rand(R, 1024, device=DEV, generator=gen) < 0.5
    x = torch.relu(torch.randn(R, 512, device=DEV, generator=gen))
    print(json.dumps({"case": "dW [1024 x 512] over 11520 rows, zero-mean g', x >= 0",
                      **case_dw(g, x, 16, variants)}), flush=True)
    # the same with random-sign x (no structure)
    xs = torch.randn(R, 512, device=DEV, generator=gen)
    print(json.dumps({"case": "dW, random-sign x", **case_dw(g, xs, 16, variants)}), flush=True)
    # dX of a 1024 -> 512 layer (K = 512): g [R, 512] x W [512, 1024]
    g2 = torch.randn(R, 512, device=DEV, generator=gen) * 1e-3
    w = torch.randn(512, 1024, device=DEV, generator=gen) / 32
    print(json.dumps({"case": "dX [11520 x 1024] from K = 512", **case_dx(g2, w, variants)}),
          flush=True)
    # a sum with a large positive running total and small terms: the bias of the accumulation
    a = torch.ones(R, 256, device=DEV) + torch.rand(R, 256, device=DEV, generator=gen) * 1e-3
    b = torch.rand(R, 256, device=DEV, generator=gen)
    print(json.dumps({"case": "dW, all-positive operands (running sum grows)",
                      **case_dw(a, b, 16, variants)}), flush=True)


if __name__ == "__main__":
    main()
