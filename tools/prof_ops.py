"""Which aten ops launch the small device kernels of one training iteration (graphs off, so the
same kernels run eagerly): torch.profiler over the second iteration, device kernels grouped by
the aten op that launched them, with input shapes. Usage:
    python tools/prof_ops.py --config 3 [--top 40]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oc_cleanrl_amd.args import Args, finalize  # noqa: E402
from oc_cleanrl_amd.trainer import PPOTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3, choices=(2, 3))
    ap.add_argument("--top", type=int, default=40)
    opt = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if opt.config == 3:
        args = Args(env_id="ALE/Breakout-v5", obs_mode="dqn", architecture="PPO", num_envs=256,
                    num_steps=128, total_timesteps=10_000_000, cuda_graphs=False,
                    save_model=False, torch_deterministic=True)
    else:
        args = Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ", num_envs=128,
                    num_steps=128, num_features=12, total_timesteps=10_000_000,
                    cuda_graphs=False, save_model=False)
    args = finalize(args, 1)
    tr = PPOTrainer(args, dev, 0, 1, kernel_timing=False, log=False)
    tr.train_iteration(collect_metrics=True, lag=False)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        tr.train_iteration(collect_metrics=True, lag=False)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    rows = [e for e in ka if e.key.startswith("aten::") and e.device_time_total > 0]
    rows.sort(key=lambda e: -e.count)
    print(f"{'calls':>6} {'dev us':>10}  op  shapes")
    for e in rows[:opt.top]:
        print(f"{e.count:6d} {e.device_time_total:10.1f}  {e.key}  {str(e.input_shapes)[:150]}")


if __name__ == "__main__":
    main()
