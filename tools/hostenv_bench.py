"""PCIe-inclusive rate of config 2 (Pong obj, 128 envs, T=128, PPObj): the learner driven by a
HOST vector env through envs.HostVecEnv (actions D2H + newest frame / reward / done H2D per step,
rollout eager, update graphs) vs the same learner on the device synthetic env. The host env is
tests/hostenv_util.NumpyObjVecEnv (numpy, stands in for a CPU emulator); its own step time is
measured separately so the staging cost can be read off."""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd.args import Args, finalize  # noqa: E402
from oc_cleanrl_amd.trainer import PPOTrainer  # noqa: E402
from tests.hostenv_util import NumpyObjVecEnv  # noqa: E402


class Timed:
    def __init__(self, env):
        self.env, self.t = env, 0.0

    def reset(self, seed=None):
        return self.env.reset(seed)

    def step(self, a):
        t0 = time.perf_counter()
        r = self.env.step(a)
        self.t += time.perf_counter() - t0
        return r


def run(host: bool, iters=5, warmup=3):
    dev = torch.device("cuda:0")
    a = finalize(Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ",
                      num_envs=128, num_steps=128, num_features=12, total_timesteps=10_000_000,
                      save_model=False), 1)
    env = Timed(NumpyObjVecEnv(128, 12, seed=1)) if host else None
    tr = PPOTrainer(a, dev, envs=env, log=False)
    for _ in range(warmup):
        tr.train_iteration()
    torch.cuda.synchronize()
    if env:
        env.t = 0.0
    t0 = time.perf_counter()
    for _ in range(iters):
        tr.train_iteration()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = iters * 128 * 128
    out = {"host_env": host, "sps": round(steps / dt, 1), "ms_per_iter": round(1e3 * dt / iters, 3)}
    if env:
        out["host_env_step_ms_per_iter"] = round(1e3 * env.t / iters, 3)
        out["us_per_rollout_step_excl_env"] = round(1e6 * (dt - env.t) / iters / 128, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    run(False)
    run(True)
