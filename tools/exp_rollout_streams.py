"""Experiment: is the config-2 rollout latency-bound enough that two env halves on two HIP
streams overlap? Times the captured rollout graph of one 128-env trainer against the rollout
graphs of two 64-env trainers replayed (a) back to back on one stream, (b) concurrently on two.

    python tools/exp_rollout_streams.py [--reps 20]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd.args import Args, finalize  # noqa: E402
from oc_cleanrl_amd.trainer import PPOTrainer  # noqa: E402


def trainer(n: int, dev):
    a = finalize(Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ", num_envs=n,
                      num_steps=128, num_features=12, total_timesteps=10_000_000,
                      cuda_graphs=True, save_model=False), 1)
    tr = PPOTrainer(a, dev, 0, 1, kernel_timing=False, log=False)
    for _ in range(3):
        tr.train_iteration(collect_metrics=False)
    torch.cuda.synchronize(dev)
    assert tr.graphs_ready and tr.g_rollout is not None
    return tr


def timed(fn, reps, dev):
    fn()
    torch.cuda.synchronize(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize(dev)
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    o = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    big = trainer(128, dev)
    a, b = trainer(64, dev), trainer(64, dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)

    def two_streams():
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            a.g_rollout.replay()
        with torch.cuda.stream(s2):
            b.g_rollout.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    out = {"N128_us": timed(big.g_rollout.replay, o.reps, dev),
           "N64_us": timed(a.g_rollout.replay, o.reps, dev),
           "2xN64_one_stream_us": timed(lambda: (a.g_rollout.replay(), b.g_rollout.replay()),
                                        o.reps, dev),
           "2xN64_two_streams_us": timed(two_streams, o.reps, dev)}
    print(json.dumps({k: round(v, 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
