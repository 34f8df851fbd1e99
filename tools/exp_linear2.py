"""Rollout encoder's first two layers (F=12 -> 256 -> 512, 128 rows, x a strided frame slice):
two ocppo_linear_act launches vs one ocppo_linear2_act launch, hipGraph-replayed."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import ops  # noqa: E402
from tools.kernel_bench import time_case  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
obs = torch.randint(0, 200, (128, 4, 12), device=dev).float()
x = obs[:, -1]
w1, b1 = torch.randn(256, 12, device=dev) * 0.1, torch.zeros(256, device=dev)
w2, b2 = torch.randn(512, 256, device=dev) * 0.05, torch.zeros(512, device=dev)
h = torch.empty(128, 256, device=dev)
y = torch.empty(128, 512, device=dev)


def two():
    ops.linear_act(x, w1, b1, True, h)
    ops.linear_act(h, w2, b2, True, y)


def one():
    ops.linear2_act(x, w1, b1, w2, b2, out=y)


for name, fn in (("two launches", two), ("linear2_act", one)):
    print(f"{name}: {time_case(fn, reps=50, rounds=5):.2f} us", flush=True)
