"""Rollout-sized convolution forwards (NatureCNN's second / third layer at 256 envs) on
ocppo_conv_x6 tile 7 against the tile loop: mean us per launch over a hipGraph-free loop of
back-to-back launches. Run once per library build (OCPPO_LIB=variant .so):
    python tools/exp_conv_rows.py [--envs 256]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oc_cleanrl_amd import ops  # noqa: E402


def bench(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    opt = ap.parse_args()
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    out = {}
    for name, (C, H, Cout, K, s) in {"conv2": (32, 20, 64, 4, 2), "conv3": (64, 9, 64, 3, 1)}.items():
        x = torch.rand(opt.envs, C, H, H, device=dev).contiguous(memory_format=cl)
        w = (torch.rand(Cout, C, K, K, device=dev) - 0.5).contiguous(memory_format=cl)
        b = torch.rand(Cout, device=dev)
        wm = w.permute(0, 2, 3, 1).reshape(Cout, -1)
        ops.WeightPlanes(fwd=(wm,)).refresh()
        wp = wm._ocppo_planes["fwd"]
        for rows in (True, False):
            ops.CONV_FWD_ROWS = rows
            out[f"{name}_{'rows' if rows else 'loop'}_us"] = round(
                bench(lambda: ops.conv_x6(x, w, b, s, True)), 2)
        ops.CONV_FWD_ROWS = True
        out[f"{name}_rows_planes_us"] = round(
            bench(lambda: ops.conv_x6(x, w, b, s, True, w_planes=wp)), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
