"""HostVecEnv host logic on CPU (no kernels): newest-frame staging, done = terminated |
truncated (cleanrl/ppo_atari_oc.py:514), episode return/length counters, obs-shape discovery."""
import numpy as np
import torch

from oc_cleanrl_amd.envs import HostVecEnv


class _Scripted:
    def __init__(self, N, W, F):
        self.N, self.W, self.F, self.t = N, W, F, 0

    def obs(self):
        o = np.zeros((self.N, self.W, self.F), np.float64)
        for w in range(self.W):
            o[:, w] = self.t * 100 + w + np.arange(self.N)[:, None]
        return o

    def reset(self, seed=None):
        return self.obs(), {}

    def step(self, actions):
        self.last_actions = np.array(actions)
        self.t += 1
        r = np.arange(self.N, dtype=np.float64) + 0.5
        term = np.zeros(self.N, bool)
        trunc = np.zeros(self.N, bool)
        if self.t == 2:
            term[0] = True
            trunc[2] = True
        return self.obs(), r, term, trunc, {}


def test_host_env_staging_and_stats():
    N, W, F = 3, 4, 5
    env = HostVecEnv(_Scripted(N, W, F), "ALE/Pong-v5", "obj", N, 1, "cpu", W)
    fr = env.reset()
    assert env.single_obs_shape == (W, F) and fr.shape == (N, F) and fr.dtype == torch.float32
    np.testing.assert_array_equal(fr.numpy(), env.envs.obs()[:, -1])
    env.step(torch.tensor([1, 2, 3]))
    np.testing.assert_array_equal(env.envs.last_actions, [1, 2, 3])
    np.testing.assert_array_equal(env.frame.numpy(), env.envs.obs()[:, -1])
    np.testing.assert_array_equal(env.reward.numpy(), [0.5, 1.5, 2.5])
    np.testing.assert_array_equal(env.done.numpy(), [0, 0, 0])
    env.step(torch.tensor([0, 0, 0]))
    np.testing.assert_array_equal(env.done.numpy(), [1, 0, 1])  # terminated | truncated
    ret, length, n = env.pop_episode_stats()
    assert n == 2 and length == 4 and ret == (0.5 * 2) + (2.5 * 2)
    assert env.pop_episode_stats() == [0.0, 0.0, 0.0]
    env.step(torch.tensor([0, 0, 0]))
    assert env._run_len.tolist() == [1, 3, 1]


def test_host_env_pixels_u8():
    N, W = 2, 4

    class Pix:
        def reset(self, seed=None):
            o = np.zeros((N, W, 84, 84), np.uint8)
            o[:, -1, 3, 5] = 7
            return o, {}

    env = HostVecEnv(Pix(), "ALE/Breakout-v5", "dqn", N, 0, "cpu", W)
    fr = env.reset()
    assert fr.dtype == torch.uint8 and fr.shape == (N, 84 * 84)
    assert int(fr[1, 3 * 84 + 5]) == 7 and int(fr.sum()) == 14


def test_host_env_sb3_api_and_vecnormalize_rejected():
    """The reference's SubprocVecEnv API (:464, :511): reset() -> obs, step -> 4-tuple."""
    import pytest

    N, W, F = 2, 4, 3

    class SB3Like:
        def reset(self):
            return np.ones((N, W, F), np.float32)

        def step(self, actions):
            return (np.full((N, W, F), 2, np.float32), np.array([1.0, -1.0]),
                    np.array([True, False]), [{}, {}])

    env = HostVecEnv(SB3Like(), "ALE/Pong-v5", "obj", N, 0, "cpu", W)
    assert float(env.reset().sum()) == N * F
    env.step(torch.tensor([0, 1]))
    np.testing.assert_array_equal(env.done.numpy(), [1, 0])
    np.testing.assert_array_equal(env.reward.numpy(), [1, -1])
    assert env.pop_episode_stats() == [1.0, 1.0, 1.0]

    class Normed(SB3Like):
        norm_reward = True

    with pytest.raises(ValueError, match="VecNormalize"):
        HostVecEnv(Normed(), "ALE/Pong-v5", "obj", N, 0, "cpu", W)
