"""DQN learner of dqn_atari_oc.py (config 5) on the GPU: graph chunks vs the step-by-step
reference order, replay contents, target updates, pixel Q-network, checkpoint payload."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def dqn_args(**kw):
    from oc_cleanrl_amd.dqn import DQNArgs

    base = dict(env_id="ALE/SpaceInvaders-v5", obs_mode="obj", num_envs=4, buffer_size=512,
                learning_starts=64, train_frequency=4, target_network_frequency=32,
                total_timesteps=4000, encoder_dims=(32, 64), decoder_dims=(64,), batch_size=32,
                save_model=False, log_every=40)
    base.update(kw)
    return DQNArgs(**base)


def run(args, n, dev):
    from oc_cleanrl_amd.dqn import DQNTrainer

    tr = DQNTrainer(args, dev, log=False)
    tr.steps(n)
    torch.cuda.synchronize()
    return tr


def test_graph_chunks_match_stepwise(dev):
    """The captured chunk (train_frequency env steps + one train step) replays the reference's
    per-step order (:341-400) exactly: same replay contents, same parameters."""
    a = run(dqn_args(cuda_graphs=False), 160, dev)
    b = run(dqn_args(cuda_graphs=True), 160, dev)
    assert b.graphs and not a.graphs
    assert torch.equal(a.rb.state, b.rb.state)
    assert torch.equal(a.rb.obs, b.rb.obs)
    assert torch.equal(a.rb.actions, b.rb.actions)
    assert torch.equal(a.rb.rewards, b.rb.rewards)
    for p, q in zip(a.q.parameters(), b.q.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    for p, q in zip(a.target.parameters(), b.target.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_training_updates_and_target_sync(dev):
    args = dqn_args(cuda_graphs=True)
    from oc_cleanrl_amd.dqn import DQNTrainer

    tr = DQNTrainer(args, dev, log=False)
    q0 = [p.detach().clone() for p in tr.q.parameters()]
    tr.steps(64)  # up to learning_starts: no train step
    for p, p0 in zip(tr.q.parameters(), q0):
        assert torch.equal(p, p0)
    assert int(tr.rb.state[0]) == 64 and int(tr.rb.state[1]) == 0
    tr.steps(28)  # global step 92: trained, target not yet synced (next sync at 96)
    assert any(not torch.equal(p, p0) for p, p0 in zip(tr.q.parameters(), q0))
    for t, p0 in zip(tr.target.parameters(), q0):
        assert torch.equal(t, p0)
    tr.steps(4)  # 96: tau = 1 -> target == q
    torch.cuda.synchronize()
    for t, p in zip(tr.target.parameters(), tr.q.parameters()):
        assert torch.equal(t, p)
    m = tr.metrics()
    assert np.isfinite(m["losses/td_loss"]) and np.isfinite(m["losses/q_values"])
    # epsilon = linear_schedule(1, .01, .1 * 4000, 96) (dqn_atari_oc.py:230-232, 345)
    assert m["charts/epsilon"] == pytest.approx(max(1 + (0.01 - 1) / 400 * 96, 0.01), rel=1e-6)


def test_replay_wraps_and_holds_env_frames(dev):
    """After more than buffer_size/num_envs steps the ring wraps (full=1); every stored obs row
    is a frame stack whose newest frame equals the next row's second-newest (no done between)."""
    tr = run(dqn_args(buffer_size=256, learning_starts=32, total_timesteps=1000), 96, dev)
    assert tr.rb.size == 64  # SB3: buffer_size // n_envs rows
    pos, full = tr.rb.state.tolist()
    assert full == 1 and pos == 96 % 64
    obs = tr.rb.obs.float().cpu().numpy()  # [size, E, 4, F]
    dn = tr.rb.dones.cpu().numpy()
    for i in range(64):
        j = (i + 1) % 64
        if i == pos:  # row pos is the newest next_obs; row pos+1 is older data
            continue
        for e in range(tr.E):
            if dn[i, e] == 0:
                assert np.array_equal(obs[j, e, :-1], obs[i, e, 1:])


def test_pixel_qnetwork_chunk(dev):
    args = dqn_args(obs_mode="dqn", env_id="ALE/Breakout-v5", num_envs=2, buffer_size=128,
                    learning_starts=16, target_network_frequency=16, torch_deterministic=False,
                    cuda_graphs=False)
    tr = run(args, 32, dev)
    assert tr.rb.obs.dtype == torch.uint8 and tuple(tr.rb.obs.shape[2:]) == (4, 84, 84)
    m = tr.metrics()
    assert np.isfinite(m["losses/td_loss"])
    ck = tr.checkpoint()
    assert list(ck["model_weights"]) == [k for k, _ in tr.q.state_dict().items()]
    assert ck["args"]["env_id"] == "ALE/Breakout-v5"


def test_run_dqn_writes_metrics(dev, tmp_path):
    import json

    from oc_cleanrl_amd.dqn import run_dqn

    args = dqn_args(total_timesteps=160, log_dir=str(tmp_path), save_model=True)
    tr = run_dqn(args, dev)
    assert tr.global_step == 160
    runs = list(tmp_path.iterdir())
    assert len(runs) == 1
    lines = [json.loads(s) for s in (runs[0] / "metrics.jsonl").read_text().splitlines()]
    assert lines[-1]["global_step"] == 160 and "charts/SPS" in lines[-1]
    ck = torch.load(runs[0] / "dqn_atari_oc.cleanrl_model", weights_only=True)
    assert set(ck) == {"model_weights", "args"}


@pytest.mark.parametrize("envs,vecnorm", [(1, True), (4, True), (3, False)])
def test_fused_act_step_is_the_four_launches(dev, monkeypatch, envs, vecnorm):
    """ops.dqn_act_step (Q head + epsilon-greedy + env + store/VecNormalize + replay add in one
    launch) leaves every buffer bitwise as the four launches do, through training chunks."""
    from oc_cleanrl_amd import dqn

    kw = dict(num_envs=envs, encoder_dims=(32, 64), decoder_dims=(256,), cuda_graphs=True,
              vecnorm_reward=vecnorm, start_e=0.5, end_e=0.05)
    monkeypatch.setattr(dqn, "FUSED_ACT_STEP", False)
    a = run(dqn_args(**kw), 160, dev)
    monkeypatch.setattr(dqn, "FUSED_ACT_STEP", True)
    b = run(dqn_args(**kw), 160, dev)
    assert a.fused_act and b.fused_act
    for x, y in ((a.rb.state, b.rb.state), (a.rb.obs, b.rb.obs), (a.rb.actions, b.rb.actions),
                 (a.rb.rewards, b.rb.rewards), (a.rb.dones, b.rb.dones),
                 (a.stacks[0], b.stacks[0]), (a.stacks[1], b.stacks[1]),
                 (a.net_obs, b.net_obs), (a.ret_state, b.ret_state), (a.rms_state, b.rms_state),
                 (a.epsilon, b.epsilon), (a.env.ep_state, b.env.ep_state),
                 (a.env.frame, b.env.frame)):
        assert torch.equal(x, y)
    for p, q in zip(a.q.parameters(), b.q.parameters()):
        assert torch.equal(p, q)
