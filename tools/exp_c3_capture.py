"""Experiment: hipGraph capture of the NatureCNN (config 3) update -- which variants capture and
replay, which crash. Each variant runs in its own child process (a crash ends only that child).

    python tools/exp_c3_capture.py            # all variants
    python tools/exp_c3_capture.py only ENVS DET CL TIMED   # one variant, in a child process
    python tools/exp_c3_capture.py child ENVS DET CL TIMED  # (used by the parent)
"""
import json
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(envs: int, det: int, cl: int, timed: int = 3):
    import torch

    from oc_cleanrl_amd.args import Args, finalize
    from oc_cleanrl_amd.trainer import PPOTrainer

    a = finalize(Args(env_id="ALE/Breakout-v5", obs_mode="dqn", architecture="PPO",
                      num_envs=envs, num_steps=128, total_timesteps=10_000_000, save_model=False,
                      torch_deterministic=bool(det), conv_channels_last=bool(cl)), 1)
    tr = PPOTrainer(a, torch.device("cuda:0"), log=False)
    tr.graph_update = True  # the capture under test
    print("iteration 1 (eager)", flush=True)
    tr.train_iteration()
    torch.cuda.synchronize()
    print("iteration 2 (capture + replay)", flush=True)
    tr.train_iteration()
    torch.cuda.synchronize()
    print("captured:", tr.graphs_ready, len(tr.g_update), flush=True)
    t0 = time.perf_counter()
    for _ in range(timed):
        tr.train_iteration()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / timed
    print(json.dumps({"envs": envs, "det": det, "cl": cl, "ms_per_iter": round(1e3 * dt, 2),
                      "sps": round(envs * 128 / dt, 1)}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(*map(int, sys.argv[2:6]))
        return
    variants = ((16, 0, 1, 3), (16, 1, 1, 3), (16, 0, 0, 3), (256, 0, 1, 3))
    if len(sys.argv) > 1 and sys.argv[1] == "only":  # e.g. `only 256 1 1 1` (envs det cl timed)
        variants = (tuple(map(int, sys.argv[2:6])),)
    for envs, det, cl, timed in variants:
        r = subprocess.run([sys.executable, __file__, "child", str(envs), str(det), str(cl),
                            str(timed)], capture_output=True, text=True, timeout=560)
        print(f"--- envs={envs} det={det} cl={cl}: rc={r.returncode}")
        print(r.stdout[-1500:])
        print(r.stderr[-2500:])
        if r.returncode < 0 or r.returncode > 128:
            print("(crashed)")


if __name__ == "__main__":
    main()
