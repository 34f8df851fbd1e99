"""Diagnostic: torch.profiler op table of one EAGER PPO iteration at config 2 (which ATen op issues
which kernels, e.g. the fills and reductions around the hipBLASLt GEMMs).

    python tools/exp_iter_profile.py [--set field=value ...]
"""
import argparse
import sys
from pathlib import Path

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd.args import Args, finalize  # noqa: E402
from oc_cleanrl_amd.trainer import PPOTrainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--set", action="append", default=[])
o = ap.parse_args()
args = Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ", num_envs=128,
            num_steps=128, num_features=12, total_timesteps=10_000_000, save_model=False,
            cuda_graphs=False)
for kv in o.set:
    k, v = kv.split("=", 1)
    cur = getattr(args, k)
    setattr(args, k, (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v))
args = finalize(args, 1)
tr = PPOTrainer(args, torch.device("cuda:0"), log=False)
for _ in range(2):
    tr.train_iteration()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=False) as prof:
    tr.train_iteration()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=60))
