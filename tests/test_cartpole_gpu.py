"""Config 1: cleanrl/ppo.py (CartPole-v1, 4 envs, clip 0.2) on the GPU learner.

* the device CartPole-v1 env (HIP ocppo_cartpole_step) against the oracle's restatement of
  gymnasium 0.28.1's cartpole.py + TimeLimit + SyncVectorEnv auto-reset (parity with gymnasium
  itself is unpinned: it is not installed; the restatement follows its published source);
* the whole learner step against two updates of ppo.py's own update block (:250-290) on its own
  Agent (:94-126), exec'd by tests/golden/gen_golden.py (tests/golden/update_cartpole.npz);
* the learner end to end (`python -m oc_cleanrl_amd.ppo`): it learns CartPole."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_cartpole_env_matches_oracle(dev):
    from oc_cleanrl_amd.envs import CartPoleVecEnv
    from oracle.ocppo_oracle import CartPoleOracle

    N, steps, seed = 64, 700, 7
    env = CartPoleVecEnv(N, seed, dev)
    ref = CartPoleOracle(N, seed)
    o = env.reset()
    assert np.array_equal(o.cpu().numpy(), ref.reset())
    rng = np.random.default_rng(0)
    worst, ndone = 0.0, 0
    for t in range(steps):
        # mostly-balancing actions so that some episodes reach the 500-step TimeLimit
        theta = ref.obs()[:, 2] + 0.3 * ref.obs()[:, 3]
        act = np.where(rng.random(N) < 0.9, (theta > 0).astype(np.int64), rng.integers(0, 2, N))
        env.step(torch.from_numpy(act).to(dev), t)
        o_ref, r_ref, d_ref = ref.step(act)
        d = env.done.cpu().numpy()
        assert np.array_equal(d, d_ref), t
        assert np.array_equal(env.reward.cpu().numpy(), r_ref)
        worst = max(worst, float(np.abs(env.frame.cpu().numpy() - o_ref).max()))
        # keep the two in lock-step at f64 (the device cos/sin may differ from libm in the last
        # ulp; the comparison above is on the f32 obs the learner sees)
        ref.state = env.state.cpu().numpy().tolist()
        ndone += int(d.sum())
    assert worst <= 1e-6, worst
    assert ndone > 0
    ep = env.ep_state.cpu().numpy()
    np.testing.assert_array_equal(ep[:, 2:], ref.ep[:, 2:])
    assert np.all(env.counters.cpu().numpy()[:, 0] < 500)


def test_cartpole_two_minibatch_updates_match_reference_golden(dev):
    """ppo.py's update (:250-290): CartPoleAgent forward, HIP fused loss (clip 0.2), autograd into
    the flat buffer, HIP clip + Adam -- the reference's parameters after each of two updates."""
    from conftest import golden
    from oc_cleanrl_amd import ops
    from oc_cleanrl_amd.agents import make_agent

    z = golden("update_cartpole.npz")
    ag = make_agent("CARTPOLE_MLP", (4,), 2, dev).to(dev)
    sd = lambda i: {k.split("::", 1)[1]: torch.from_numpy(z[k]) for k in z  # noqa: E731
                    if k.startswith(f"sd{i}::")}
    ag.load_state_dict(sd(0))
    opt = ops.FlatAdam(ag.parameters(), lr=2.5e-4, eps=1e-5, max_grad_norm=0.5)
    T = lambda k: torch.from_numpy(z[k]).to(dev)  # noqa: E731
    b_obs, acts = T("b_obs"), T("b_actions")
    lp, adv, ret, val = T("b_logprobs"), T("b_advantages"), T("b_returns"), T("b_values")
    perm, M = T("perm"), int(z["M"])
    for i, start in enumerate((0, M)):
        idx = perm[start:start + M].contiguous()
        logits, value = ag.logits_and_value(ops.gather_rows(b_obs, idx))
        st, dl, dv = ops.ppo_loss_fwd_bwd(logits.detach(), value.detach().view(-1), acts, lp, adv,
                                          ret, val, mb_inds=idx, clip_coef=0.2, ent_coef=0.01,
                                          vf_coef=0.5, norm_adv=True, clip_vloss=True)
        np.testing.assert_allclose(st[:7].cpu().numpy(), z["stats"][i], rtol=2e-5, atol=1e-7)
        opt.zero_grad()  # nn.Linear grads are accumulated by autograd
        torch.autograd.backward([logits, value], [dl, dv.view(-1, 1)])
        opt.step()
        for k, ref in sd(i + 1).items():
            got = ag.state_dict()[k].cpu()
            torch.testing.assert_close(got, ref, rtol=0, atol=0.01 * 2.5e-4)


def test_ppo_script_learns_cartpole(dev, tmp_path):
    """`python -m oc_cleanrl_amd.ppo` (cleanrl/ppo.py defaults: 4 envs, T=128, clip 0.2, seed 1)
    on the device CartPole-v1: the episodic return climbs from ~20 (random policy) to > 150
    within 100k env steps (ppo.py reaches 490 +- 6 at 500k, docs/rl-algorithms/ppo.md:111)."""
    import json

    from oc_cleanrl_amd.ppo import main

    tr = main(["--total-timesteps", "102400", "--log-dir", str(tmp_path), "--no-save-model"])
    assert tr.env.env_id == "CartPole-v1" and tr.args.clip_coef == 0.2 and tr.N == 4
    assert tr.obs.dtype == torch.float32 and tr.graphs_ready
    rows = [json.loads(x) for x in next(tmp_path.iterdir()).joinpath("metrics.jsonl").open()]
    rets = [r["charts/Episodic_Original_Reward"] for r in rows
            if "charts/Episodic_Original_Reward" in r]
    assert np.mean(rets[:5]) < 60, rets[:5]
    assert np.mean(rets[-10:]) > 150, rets[-10:]
