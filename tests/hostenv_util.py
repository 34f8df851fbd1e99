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
    frame_stack_fill_rule = True  # reset stacks are W copies of the first frame (FrameStack)

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

    frame_stack_fill_rule = True

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


class AtariLikeVecEnv:
    """SB3-VecEnv-shaped stand-in for the reference's wrapper chain (ppo_atari_oc.py:278-282):
    RecordEpisodeStatistics -> NoopResetEnv -> EpisodicLifeEnv -> FireResetEnv over a FrameStack.
    A done is a life loss (p_life; the stack is NOT reset and the game goes on) or a game over
    (p_game; the auto-reset stack holds W distinct frames, as the no-op / FIRE steps after reset
    leave it). info["episode"] = {"r", "l"} of the whole game is reported on game over only.
    Every returned stack is recorded in `history` (index 0 = the reset obs)."""

    def __init__(self, num_envs, num_features=12, window=4, seed=0, p_life=0.03, p_game=0.02):
        self.N, self.F, self.W = num_envs, num_features, window
        self.rng = np.random.default_rng(seed)
        self.p_life, self.p_game = p_life, p_game
        self.stack = np.zeros((num_envs, window, num_features), np.float32)
        self.game_ret = np.zeros(num_envs)
        self.game_len = np.zeros(num_envs, np.int64)
        self.history = []
        self.games = []  # (return, length) of every finished game

    def _frames(self, *lead):
        return self.rng.integers(0, 210, lead + (self.F,)).astype(np.float32)

    def reset(self):
        self.stack[:] = self._frames(self.N, self.W)
        self.history = [self.stack.copy()]
        return self.stack.copy()

    def step(self, actions):
        assert len(actions) == self.N
        r = self.rng.choice([-1.0, 0.0, 0.0, 0.0, 1.0], self.N)
        u = self.rng.random(self.N)
        life = u < self.p_life
        game = (u >= self.p_life) & (u < self.p_life + self.p_game)
        self.stack[:, :-1] = self.stack[:, 1:]
        self.stack[:, -1] = self._frames(self.N)
        self.game_ret += r
        self.game_len += 1
        infos = [{} for _ in range(self.N)]
        for n in np.flatnonzero(game):
            infos[n]["episode"] = {"r": float(self.game_ret[n]), "l": int(self.game_len[n])}
            self.games.append((float(self.game_ret[n]), int(self.game_len[n])))
            self.game_ret[n] = 0.0
            self.game_len[n] = 0
            self.stack[n] = self._frames(self.W)  # auto-reset: distinct no-op frames
        self.history.append(self.stack.copy())
        return self.stack.copy(), r, life | game, infos
