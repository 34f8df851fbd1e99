"""Experiment (GPU): ocppo_conv_x6 tile and split choices at config 3's update sizes (minibatch
8192): each layer's forward / weight gradient / data gradient timed with HIP events over 20
launches per choice.

    python tools/exp_conv_tiles.py
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import ops  # noqa: E402

DEV = torch.device("cuda:0")
CL = torch.channels_last


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n


def main():
    B = 8192
    out = []
    layers = {"conv2": (32, 20, 64, 4, 2), "conv3": (64, 9, 64, 3, 1)}
    for name, (C, H, Cout, K, s) in layers.items():
        x = torch.rand(B, C, H, H, device=DEV).contiguous(memory_format=CL)
        w = (torch.rand(Cout, C, K, K, device=DEV) - 0.5).contiguous(memory_format=CL)
        b = torch.rand(Cout, device=DEV)
        OH = (H - K) // s + 1
        gp = torch.rand(B, Cout, OH, OH, device=DEV).contiguous(memory_format=CL)
        rows = gp.permute(0, 2, 3, 1).reshape(-1, Cout)
        orig_f, orig_w = ops._conv_fwd_tile, ops._conv_wgrad_tile
        for t in (2, 3, 6):
            ops._conv_fwd_tile = lambda M, N, t=t: t
            try:
                out.append({"layer": name, "op": "fwd", "tile": t,
                            "us": round(timeit(lambda: ops.conv_x6(x, w, b, s, True)), 1)})
            except Exception as e:  # noqa: BLE001
                out.append({"layer": name, "op": "fwd", "tile": t, "err": str(e)[:80]})
        ops._conv_fwd_tile = orig_f
        for t in (2, 3, 5, 6):
            if t == 5 and (s * s * C) % 128:
                continue
            ops._conv_fwd_tile = lambda M, N, t=t: t
            try:
                out.append({"layer": name, "op": "dgrad", "tile": t,
                            "us": round(timeit(lambda: ops.conv_x6_dgrad(gp, w, s, (H, H))), 1)})
            except Exception as e:  # noqa: BLE001
                out.append({"layer": name, "op": "dgrad", "tile": t, "err": str(e)[:80]})
        ops._conv_fwd_tile = orig_f
        for t in (3, 4):
            ops._conv_wgrad_tile = lambda M, N, t=t: t
            try:
                out.append({"layer": name, "op": "wgrad", "tile": t,
                            "us": round(timeit(lambda: ops.conv_x6_wgrad(rows, x, (K, K), s)), 1)})
            except Exception as e:  # noqa: BLE001
                out.append({"layer": name, "op": "wgrad", "tile": t, "err": str(e)[:80]})
        ops._conv_wgrad_tile = orig_w
        print(json.dumps(out[-9:]), flush=True)
    # the first convolution: f32 NHWC vs u8 frame stacks
    src = torch.randint(0, 256, (32768, 4, 84, 84), device=DEV, dtype=torch.uint8)
    idx = torch.randperm(32768, device=DEV)[:B]
    w1 = (torch.rand(32, 4, 8, 8, device=DEV) - 0.5).contiguous(memory_format=CL)
    b1 = torch.rand(32, device=DEV)
    x1 = (src[idx].float() / 255).contiguous(memory_format=CL)
    gp1 = torch.rand(B * 400, 32, device=DEV)
    out.append({"layer": "conv1", "op": "fwd_f32", "us": round(timeit(lambda: ops.conv_x6(x1, w1, b1, 4, True)), 1)})
    out.append({"layer": "conv1", "op": "fwd_u8", "us": round(timeit(lambda: ops.conv_x6_u8(src, idx, w1, b1, 4, True)), 1)})
    out.append({"layer": "conv1", "op": "wgrad_f32", "us": round(timeit(lambda: ops.conv_x6_wgrad(gp1, x1, (8, 8), 4)), 1)})
    out.append({"layer": "conv1", "op": "wgrad_u8", "us": round(timeit(lambda: ops.conv_x6_u8_wgrad(gp1, src, idx, (8, 8), 4)), 1)})
    out.append({"layer": "conv1", "op": "gather", "us": round(timeit(lambda: ops.gather_rows(src, idx, x1, scale255=True)), 1)})
    print(json.dumps(out[-5:]), flush=True)


if __name__ == "__main__":
    main()
