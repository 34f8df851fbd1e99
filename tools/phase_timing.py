"""Device time of the two phases of one PPO iteration (config 2 by default): the captured rollout
graph (128 env steps + bootstrap + GAE + minibatch prepare) and the update graphs, each replayed
between HIP events on the trainer's stream.

    python tools/phase_timing.py [--set field=value ...]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from oc_cleanrl_amd.args import Args, finalize  # noqa: E402
from oc_cleanrl_amd.trainer import PPOTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3))
    o = ap.parse_args()
    if o.config == 3:
        args = Args(env_id="ALE/Breakout-v5", obs_mode="dqn", architecture="PPO", num_envs=256,
                    num_steps=128, total_timesteps=10_000_000, save_model=False,
                    torch_deterministic=False)
    else:
        args = Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ", num_envs=128,
                    num_steps=128, num_features=12, total_timesteps=10_000_000, save_model=False)
    for kv in o.set:
        k, v = kv.split("=", 1)
        obj = args
        if k.startswith("agents."):  # a module switch, e.g. agents.HIP_SUM_SPLITS=0
            from oc_cleanrl_amd import agents as obj
            k = k.split(".", 1)[1]
        cur = getattr(obj, k)
        setattr(obj, k, (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v))
    args = finalize(args, 1)
    dev = torch.device("cuda:0")
    tr = PPOTrainer(args, dev, log=False)
    for _ in range(3):
        tr.train_iteration()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    roll, upd = 0.0, 0.0
    for _ in range(o.reps):
        ev[0].record()
        tr.g_rollout.replay()
        ev[1].record()
        tr._run_update()
        ev[2].record()
        torch.cuda.synchronize()
        roll += ev[0].elapsed_time(ev[1])
        upd += ev[1].elapsed_time(ev[2])
    print(json.dumps({"set": o.set, "rollout_ms": round(roll / o.reps, 3),
                      "update_ms": round(upd / o.reps, 3),
                      "per_step_us": round(1e3 * roll / o.reps / args.num_steps, 2)}))


if __name__ == "__main__":
    main()
