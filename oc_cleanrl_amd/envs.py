"""Device-resident vectorised environments.

ALE / OCAtari / HackAtari are not available (no emulator, no network), so the learner is driven
by a synthetic env that lives in HBM and steps with one HIP kernel (ocppo_synth_env_step):
object-vector frames with OCAtari obj-mode statistics or 84x84 u8 pixel frames, Pong-like sparse
rewards and episode ends. It replaces the SubprocVecEnv + per-step host round trip
of cleanrl/ppo_atari_oc.py:411-414, 511-514; its dynamics are NOT Pong's (parity of returns
against real ALE is unpinned).

The env produces the NEWEST frame per env; frame stacking and storage happen in the rollout store
kernel (ops.rollout_store).
"""
from __future__ import annotations

import torch

from . import ops
from .args import ACTION_COUNTS


class SyntheticAtariEnv:
    """num_envs synthetic Atari envs on one device.

    obs_mode "obj": frames [N, F] f32 (F = num_features); "dqn": frames [N, 84*84] u8.
    """

    def __init__(self, env_id: str, obs_mode: str, num_envs: int, num_features: int, seed: int,
                 device, window: int = 4):
        self.env_id = env_id
        self.pixels = obs_mode == "dqn"
        self.num_envs = num_envs
        self.n_actions = ACTION_COUNTS.get(env_id, 6)
        self.window = window
        self.frame_elems = 84 * 84 if self.pixels else num_features
        self.single_obs_shape = (window, 84, 84) if self.pixels else (window, num_features)
        self.frame_dtype = torch.uint8 if self.pixels else torch.float32
        self.seed = int(seed)
        self.device = torch.device(device)
        N = num_envs
        self.frame = torch.zeros((N, self.frame_elems), dtype=self.frame_dtype, device=device)
        self.reward = torch.zeros(N, dtype=torch.float32, device=device)
        self.done = torch.zeros(N, dtype=torch.float32, device=device)
        # RecordEpisodeStatistics counters: run_ret, run_len, fin_ret_sum, fin_len_sum, fin_count
        self.ep_state = torch.zeros((N, 5), dtype=torch.float32, device=device)
        self.step_base = torch.zeros(1, dtype=torch.int64, device=device)

    def reset(self):
        """Initial frames (step id = step_base); advances step_base by one."""
        ops.synth_env_step(self.seed, self.step_base, 0, None, self.frame, self.reward, self.done,
                           None)
        self.step_base.add_(1)
        return self.frame

    def step(self, actions, step_offset: int):
        """Writes frame/reward/done for step id step_base + step_offset (graph-replay safe)."""
        ops.synth_env_step(self.seed, self.step_base, step_offset, actions, self.frame,
                           self.reward, self.done, self.ep_state)

    def advance(self, n: int):
        self.step_base.add_(n)

    def pop_episode_stats(self):
        """(sum of finished-episode returns, sum of lengths, count) since the last call."""
        s = self.ep_state[:, 2:5].sum(0, dtype=torch.float64).tolist()
        self.ep_state[:, 2:5].zero_()
        return s
