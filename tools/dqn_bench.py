"""Config 5 throughput: dqn_atari_oc.py SpaceInvaders obj-mode, 1M-transition HBM replay buffer,
one process on cuda:0. Times K global steps in the training phase (epsilon-greedy act + env step +
store + replay add every step, sample + fused TD loss + backward + Adam every train_frequency
steps, target sync every target_network_frequency steps), all as replayed hipGraph chunks.

    python tools/dqn_bench.py [--steps K] [--obs-mode obj|dqn] [--num-envs E]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from oc_cleanrl_amd.dqn import DQNArgs, DQNTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=2000)
    ap.add_argument("--obs-mode", default="obj")
    ap.add_argument("--num-envs", type=int, default=1)
    ap.add_argument("--buffer-size", type=int, default=1_000_000)
    o = ap.parse_args()
    env = "ALE/SpaceInvaders-v5"
    args = DQNArgs(env_id=env, obs_mode=o.obs_mode, num_envs=o.num_envs,
                   buffer_size=o.buffer_size, learning_starts=1000, total_timesteps=10_000_000,
                   save_model=False, torch_deterministic=o.obs_mode != "dqn")
    dev = torch.device("cuda:0")
    tr = DQNTrainer(args, dev, log=False)
    tr.steps(args.learning_starts + o.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.steps(o.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = tr.metrics()
    print(json.dumps({
        "metric": "env steps/sec + DQN updates/sec, dqn_atari_oc.py SpaceInvaders-v5 (BASELINE config 5)",
        "value": round(o.steps * o.num_envs / dt, 1), "unit": "env steps/s",
        "updates_per_sec": round(o.steps / args.train_frequency / dt, 1),
        "us_per_global_step": round(dt / o.steps * 1e6, 3),
        "config": {"obs_mode": o.obs_mode, "num_envs": o.num_envs, "replay_rows": tr.rb.size,
                   "replay_obs_dtype": str(tr.obs_dtype).replace("torch.", ""),
                   "replay_bytes": tr.rb.obs.numel() * tr.rb.obs.element_size(),
                   "batch_size": args.batch_size, "train_frequency": args.train_frequency,
                   "gemm_table": tr.gemm_table,
                   "cuda_graphs": tr._graphable()},
        "td_loss": m["losses/td_loss"], "data": "synthetic device env, random-init Q-network"}))


if __name__ == "__main__":
    main()
