"""Host env → device rollout path (envs.HostVecEnv, the env-step boundary of
cleanrl/ppo_atari_oc.py:506-514): fed with the device synthetic env seen through gymnasium's
vector API (tests/hostenv_util.DeviceEnvAsHost), the learner must produce exactly what the
device-env learner produces -- same obs / rewards / dones / actions / advantages bit for bit and
the same weights -- so the staging (actions D2H, newest frame + reward + done H2D) is exact."""
import numpy as np
import pytest
import torch

from tests.hostenv_util import DeviceEnvAsHost, NumpyObjVecEnv

pytestmark = pytest.mark.gpu


def _args(**kw):
    from oc_cleanrl_amd.args import Args, finalize

    base = dict(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ", num_envs=32,
                num_steps=16, num_minibatches=4, update_epochs=2, total_timesteps=32 * 16 * 10,
                encoder_dims=(32, 64), decoder_dims=(64,), save_model=False)
    base.update(kw)
    return finalize(Args(**base), 1)


@pytest.mark.parametrize("pixels", [False, True])
def test_host_env_matches_device_env(dev, pixels):
    from oc_cleanrl_amd.trainer import PPOTrainer

    kw = dict(env_id="ALE/Breakout-v5", obs_mode="dqn", architecture="PPO", num_envs=8,
              num_steps=8, update_epochs=1) if pixels else {}
    # the synthetic frames are integers <= 210: bf16 storage is exact (host envs default to f32)
    a = _args(obs_storage="bf16", **kw)
    names = ("obs", "rewards", "dones", "actions", "logprobs", "values", "advantages", "returns")
    # one learner after the other: both draw their sampling noise from torch's global generator,
    # which each PPOTrainer re-seeds at construction
    ref = PPOTrainer(a, dev)
    snaps = []
    for _ in range(3):
        ref.train_iteration()
        snaps.append({n: getattr(ref, n).clone() for n in names})
    host = DeviceEnvAsHost(a.env_id, a.obs_mode, a.local_num_envs, a.num_features, a.seed, dev,
                           a.buffer_window_size)
    tr = PPOTrainer(a, dev, envs=host)
    assert tr.host_env and tr.obs_shape == ref.obs_shape
    for it in range(3):
        tr.train_iteration()
        torch.cuda.synchronize()
        for name in names:
            x, y = snaps[it][name], getattr(tr, name)
            assert torch.equal(x, y), (it, name, (x.float() - y.float()).abs().max().item())
    assert ref.graphs_ready and tr.graphs_ready and tr.g_rollout is None
    for p, q in zip(ref.agent.parameters(), tr.agent.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-7)


def test_numpy_host_env_trains(dev):
    from oc_cleanrl_amd.trainer import PPOTrainer

    a = _args()
    tr = PPOTrainer(a, dev, envs=NumpyObjVecEnv(a.local_num_envs, a.num_features, seed=3))
    ms = [tr.train_iteration() for _ in range(2)]
    assert all(torch.isfinite(torch.tensor(m["losses/loss"])) for m in ms)
    # the newest frame of every stored obs slot is an integer coordinate frame from the host
    last = tr.obs[:, :, -1].float()
    assert torch.equal(last, last.floor()) and float(last.max()) < 210


@pytest.mark.parametrize("graphs", [True, False])
def test_host_env_reset_stacks_and_episode_infos(dev, graphs):
    """A host env whose reset stacks are NOT the FrameStack fill (no-op steps after reset,
    life-loss dones without a stack reset): every stored obs slot is exactly the stack the env
    returned, and the episodic scalars are whole games from info["episode"] (:516-529), not
    per-life sums."""
    from oc_cleanrl_amd.trainer import PPOTrainer
    from tests.hostenv_util import AtariLikeVecEnv

    a = _args(cuda_graphs=graphs, num_envs=16, num_steps=16)
    env = AtariLikeVecEnv(a.local_num_envs, a.num_features, seed=5)
    tr = PPOTrainer(a, dev, envs=env)
    assert tr.reset_stacks and not tr.frame_cache and not tr.frame_dedup
    assert tr.obs.dtype == torch.float32  # host envs: f32 storage by default
    T = a.num_steps
    games_seen = 0
    for it in range(3):
        m = tr.train_iteration()
        torch.cuda.synchronize()
        got = tr.obs.cpu().numpy()
        for t in range(T + 1):
            exp = env.history[it * T + t]
            assert np.array_equal(got[t], exp), (it, t)
        new = env.games[games_seen:]
        games_seen = len(env.games)
        if new:
            assert m["charts/Episodic_Original_Reward"] == pytest.approx(
                sum(g[0] for g in new) / len(new))
            assert m["charts/Episodic_Length"] == pytest.approx(sum(g[1] for g in new) / len(new))
        else:
            assert "charts/Episodic_Original_Reward" not in m
    assert games_seen > 0
