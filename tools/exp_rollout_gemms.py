"""Time the rollout-step trunk layers (config 2: N=128 envs, 4 frames x 12 features) one by one,
each captured 50x in a hipGraph, to see what hipBLASLt reaches on these small-M shapes."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def t(fn, reps=50, rounds=5):
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(rounds):
        g.replay()
    b.record(); torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / (reps * rounds)


def main():
    dev = torch.device("cuda:0")
    shapes = [(512, 12, 256), (512, 256, 512), (512, 512, 1024), (512, 1024, 512), (128, 2048, 512),
              (4096 * 4, 12, 256), (16384, 256, 512), (16384, 512, 1024), (16384, 1024, 512), (4096, 2048, 512)]
    for m, k, n in shapes:
        x = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.05
        b = torch.randn(n, device=dev)
        us = t(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
        print(json.dumps({"m": m, "k": k, "n": n, "us": round(us, 2), "TFs": round(2 * m * k * n / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
