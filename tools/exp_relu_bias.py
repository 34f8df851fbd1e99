"""Per-shape timing of ops.relu_bias_grad at the config-2 update shapes (and conv shapes of
config 3), each launch replayed back-to-back in a hipGraph; GB/s over the algorithmic bytes."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import ops  # noqa: E402
from tools.kernel_bench import time_case  # noqa: E402

dev = torch.device("cuda:0")
shapes = [(12288, 1024), (12288, 512), (12288, 256), (4096, 512), (262144, 1024),
          (3276800, 32), (663552, 64), (401408, 64)]
tot_t = tot_b = 0.0
for R, N in shapes:
    g = torch.randn(R, N, device=dev)
    out = torch.relu(torch.randn(R, N, device=dev))
    gp, db = torch.empty_like(g), torch.empty(N, device=dev)
    us = time_case(lambda: ops.relu_bias_grad(g, out, db=db, gp=gp), reps=20, rounds=5)
    nb = R * N * 12 + 4 * N
    print(f"[{R} x {N}] {us:8.2f} us  {nb / us / 1e3:7.0f} GB/s", flush=True)
    del g, out, gp
    torch.cuda.empty_cache()
