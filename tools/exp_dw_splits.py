"""The update's encoder weight gradients dW [n, k] = g'^T x over 11520 frame rows (the dedup
encoder's layers 3 and 4, ppo_atari_oc.py:605 through architectures/ppo.py:60-84) on gemm_x6:
device time of the split-K product and of its combine (sum_splits_db with the layer's 720
bias-gradient chunk partials) per (tile, splits) (experiment).

    python tools/exp_dw_splits.py > gpurun_out/exp_dw_splits.jsonl
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
from oc_cleanrl_amd import ops  # noqa: E402
from exp_gemm_x6 import dev_time_us  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    R = 11520
    g = torch.Generator(device=dev).manual_seed(0)
    for n, k in ((1024, 512), (512, 1024)):
        gp = torch.randn(R, n, device=dev, generator=g)
        x = torch.relu(torch.randn(R, k, device=dev, generator=g))
        dbp = torch.randn(720, n, device=dev, generator=g)
        out = torch.empty(n, k, device=dev)
        db = torch.empty(n, device=dev)
        for t in range(ops.X6_AUTO, ops.X6_AUTO + 4):
            for S in (4, 8, 16):
                if ops.x6_tile(n, k, S, t) is None or not ops.dw_x6_ok(gp, x, S):
                    continue
                part = torch.empty(S, n, k, device=dev)
                us = dev_time_us(lambda: ops.dw_x6_parts(gp, x, S, part=part, tile=t), 20)
                cu = dev_time_us(lambda: ops.sum_splits_db(part, out, (dbp, 720), db), 20)
                bm, bn = ops.X6_TILES[t]
                print(json.dumps({"n": n, "k": k, "tile": t, "bm": bm, "bn": bn, "splits": S,
                                  "units": S * (n // bm) * (k // bn), "gemm_us": round(us, 2),
                                  "combine_us": round(cu, 2), "total_us": round(us + cu, 2)}),
                      flush=True)


if __name__ == "__main__":
    main()
