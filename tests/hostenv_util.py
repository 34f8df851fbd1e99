"""Host-side vector envs for the HostVecEnv tests and the PCIe-inclusive bench leg.

DeviceEnvAsHost: the device synthetic env seen through gymnasium's vector API (numpy in/out,
FrameStack-style [N, W, *frame] obs, autoreset) -- the host path fed with it must reproduce the
device-env learner bit for bit. NumpyObjVecEnv: a pure-numpy object-vector env (OCAtari obj-mode
statistics of SURVEY §8d), the stand-in for a real CPU emulator when timing the staging path.
"""
from __future__ import annotations

import numpy as np
import torch


class DeviceEnvAsHost:
    def __init__(self, env_id, obs_mode, num_envs, num_features, seed, device, window=4):
        from oc_cleanrl_amd.envs import SyntheticAtariEnv

        self.syn = SyntheticAtariEnv(env_id, obs_mode, num_envs, num_features, seed, device,
                                     window)
        self.window = window
        self.stack = None

    def _frame(self):
        f = self.syn.frame.cpu().numpy()
        return f.reshape(-1, 84, 84) if self.syn.pixels else f

    def reset(self, seed=None):
        f = self._frame_after(self.syn.reset)
        self.stack = np.repeat(f[:, None], self.window, axis=1)
        return self.stack.copy(), {}

    def _frame_after(self, fn):
        fn()
        return self._frame()

    def step(self, actions):
        a = torch.as_tensor(np.asarray(actions, dtype=np.int64), device=self.syn.device)
        self.syn.step(a, 0)
        self.syn.advance(1)
        f = self._frame()
        r = self.syn.reward.cpu().numpy().astype(np.float64)
        d = self.syn.done.cpu().numpy() > 0.5
        self.stack = np.concatenate([self.stack[:, 1:], f[:, None]], axis=1)
        self.stack[d] = f[d][:, None]  # autoreset: FrameStack of the new episode's first frame
        return self.stack.copy(), r, d, np.zeros_like(d), {}


class NumpyObjVecEnv:
    """N object-vector envs on the host: F = 12 integer coordinates per frame, ±1 rewards with
    p = 0.005 each, episode ends with p = 1/3500, FrameStack(W)."""

    def __init__(self, num_envs, num_features=12, window=4, seed=0):
        self.N, self.F, self.W = num_envs, num_features, window
        self.rng = np.random.default_rng(seed)
        self.hi = np.tile(np.array([160, 210, 16, 16], np.float32), num_features // 4 + 1)[:num_features]
        self.stack = np.zeros((num_envs, window, num_features), np.float32)

    def _frames(self):
        return np.floor(self.rng.random((self.N, self.F), dtype=np.float32) * self.hi)

    def reset(self, seed=None):
        self.stack[:] = self._frames()[:, None]
        return self.stack.copy(), {}

    def step(self, actions):
        f = self._frames()
        u = self.rng.random(self.N)
        r = np.where(u < 0.005, 1.0, np.where(u > 0.995, -1.0, 0.0))
        d = self.rng.random(self.N) < 1 / 3500
        self.stack[:, :-1] = self.stack[:, 1:]
        self.stack[:, -1] = f
        self.stack[d] = f[d][:, None]
        return self.stack.copy(), r, d, np.zeros_like(d), {}
