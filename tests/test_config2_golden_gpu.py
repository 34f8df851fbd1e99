"""BASELINE config 2 at the network's real size through the bench's own update chain.

tests/golden/update_config2.npz is the reference's GAE block (ppo_atari_oc.py:533-547) and two
minibatch updates of 4096 through its update block (:566-610) on PPObj(encoder (256, 512, 1024,
512), decoder (512,)) over a rollout-structured 128 x 128 Pong-obj batch (gen_golden.py
gen_update_config2). Here the fixture is loaded into PPOTrainer's own HBM buffers and run through
exactly the path bench.py times: frame-dedup gather fused with the first encoder layer, the
update GEMMs on the bf16 matrix cores as exact-split f32 (ocppo_gemm_x6, the ReLU backward of the
layer below fused into each dX) and hipBLASLt under the shipped solution table for the rest (and,
with x6_gemm off, for all of them), frame scatter with the last encoder ReLU, deferred bias
grads, heads forward + loss + heads backward in one HIP op at H = 512, FlatAdam (clip + Adam).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LR = 2.5e-4


def config2_weights(agent, seed):
    """The fixture's seeded parameters (gen_golden.config2_weights: numpy PCG64, bit-identical on
    every platform), pinned by the fixture's checksums below."""
    rng = np.random.default_rng(seed)
    sd = {}
    for k, v in agent.state_dict().items():
        if k.endswith("weight"):
            gain = 0.01 if k.startswith("actor") else 1.0 if k.startswith("critic") else 2 ** 0.5
            w = rng.standard_normal(tuple(v.shape)) * (gain / np.sqrt(v.shape[1]))
        else:
            w = rng.standard_normal(tuple(v.shape)) * 0.05
        sd[k] = torch.from_numpy(w.astype(np.float32))
    return sd


@pytest.fixture(scope="module")
def fixture():
    from conftest import golden

    return golden("update_config2.npz")


def config2_trainer(dev, z, **kw):
    from oc_cleanrl_amd.args import Args, finalize
    from oc_cleanrl_amd.trainer import PPOTrainer

    args = finalize(Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ",
                         num_envs=128, num_steps=128, num_features=12, save_model=False, **kw), 1)
    tr = PPOTrainer(args, dev)
    sd0 = config2_weights(tr.agent, int(z["seed"]))
    for k, v in sd0.items():
        v64 = v.double()
        s = z[f"sum0::{k}"]
        assert float(v64.sum()) == pytest.approx(s[0], rel=1e-12, abs=1e-9), k
        assert float((v64 ** 2).sum()) == pytest.approx(s[1], rel=1e-12), k
    with torch.no_grad():
        tr.agent.load_state_dict(sd0)
    T, N = tr.T, tr.N
    D = lambda k, dt=None: torch.from_numpy(z[k]).to(dev, dt)  # noqa: E731
    tr.obs.copy_(D("obs", torch.float32).to(tr.obs.dtype))
    tr.dones.copy_(D("dones"))
    tr.actions.copy_(D("actions").view(T, N))
    tr.logprobs.copy_(D("logprobs").view(T, N))
    tr.values[:T].copy_(D("values").view(T, N))
    tr.values[T].copy_(D("next_value"))
    tr.rewards.copy_(D("rewards"))
    return tr


def full_permutation(z, E, B):
    """Epoch 0 = the fixture's two minibatches, then the remaining samples; every epoch alike."""
    head = z["perm"].astype(np.int64)
    rest = np.setdiff1d(np.arange(B), head)
    return np.tile(np.concatenate([head, rest]), E)


def test_config2_gae_matches_reference(dev, fixture):
    """The HIP GAE on the rollout-structured batch: bit-exact to the reference loop."""
    from oc_cleanrl_amd import ops

    z = fixture
    tr = config2_trainer(dev, z)
    T = tr.T
    ops.gae(tr.rewards, tr.values[:T], tr.dones[:T], tr.values[T], tr.dones[T], 0.99, 0.95,
            tr.advantages, tr.returns)
    torch.cuda.synchronize()
    assert np.array_equal(tr.advantages.cpu().numpy().reshape(-1), z["advantages"])
    assert np.array_equal(tr.returns.cpu().numpy().reshape(-1), z["returns"])


@pytest.mark.parametrize("x6", [True, False])
def test_config2_update_chain_matches_reference(dev, fixture, x6):
    """Two minibatch updates of the bench's chain vs the reference's update block at config 2:
    grad norms to 1e-5, loss scalars to 1e-4, and every parameter (4096 fixed samples of the
    large ones) within 1 % of one Adam step (lr) -- Adam's m / (sqrt(v) + eps) is sensitive to
    the f32 summation order of a gradient element only where |g| ~ eps. (Graph replay of this
    chain is bitwise the eager run: test_trainer_gpu.py::test_graph_replay_matches_eager.)"""
    from oc_cleanrl_amd import ops
    from oc_cleanrl_amd.trainer import KernelTimer

    z = fixture
    tr = config2_trainer(dev, z, x6_gemm=x6)
    assert tr.frame_dedup and tr.fused_heads_loss and tr.direct_grads and tr.H == 512
    assert tr.gemm_table and tr.args.gemm_table
    tr.advantages.view(-1).copy_(torch.from_numpy(z["advantages"]).to(dev))
    tr.returns.view(-1).copy_(torch.from_numpy(z["returns"]).to(dev))
    tr.load_permutation(full_permutation(z, tr.E, tr.B))
    tr._prepare_minibatches()
    M = int(z["M"])
    assert tr.M == M
    params = dict(tr.agent.named_parameters())
    timer = KernelTimer(enabled=True)  # records which launch sites the chain runs
    ops.TIMER = timer
    try:
        for j in range(2):
            _minibatch(tr, z, j, params)
    finally:
        ops.TIMER = None
    x6_sites = sorted(n for n in timer.sites if n.startswith("gemm_x6_"))
    # on: the nine x6 products of config 2 (forward, masked / plain dX, split-K dW); off: none
    assert (len(x6_sites) >= 8) if x6 else not x6_sites, x6_sites


def f64_errors(z, j, params):
    """Per tensor, the PRE-clip gradient error against the fixture's float64 twin of the same
    update block (gen_golden: the same inputs in f64 at the f32 reference's parameters), relative
    to the tensor's largest f64 element: (ours, the f32 reference's own)."""
    out = {}
    for k, p in params.items():
        g = p.grad.detach().double().cpu().reshape(-1)
        if f"pick::{k}" in z:
            g = g[torch.from_numpy(z[f"pick::{k}"])]
        g64 = torch.from_numpy(z[f"grad64pre{j}::{k}"]).reshape(-1)
        g32 = torch.from_numpy(z[f"gradpre{j}::{k}"]).double().reshape(-1)
        mx = float(z[f"gnorm64pre{j}::{k}"][1])
        out[k] = (float((g - g64).abs().max()) / mx, float((g32 - g64).abs().max()) / mx)
    return out


def _minibatch(tr, z, j, params):
    """One minibatch of the chain against the fixture's grads, stats and parameters."""
    tr._forward_backward(j)
    gn = float(torch.linalg.vector_norm(tr.grad_buf.double()))
    e64 = f64_errors(z, j, params)
    print(f"minibatch {j}: grad norm {gn:.10g}, f64 {float(z[f'grad_norm64_{j}']):.10g}, f32 ref "
          f"{z['grad_norms'][j]:.10g}; pre-clip error vs f64 per tensor (ours / reference f32): "
          + ", ".join(f"{k} {a:.2g}/{b:.2g}" for k, (a, b) in e64.items()))
    # the gradients the reference's Adam saw (after clip_grad_norm_: x max_norm / (norm +
    # 1e-6)), per tensor, at the fixture's sample points, relative to the tensor's largest
    coef = min(1.0, 0.5 / (gn + 1e-6))
    gerr = {}
    for k, p in params.items():
        g = p.grad.detach().double().cpu().reshape(-1) * coef
        if f"pick::{k}" in z:
            g = g[torch.from_numpy(z[f"pick::{k}"])]
        ref = torch.from_numpy(z[f"grad{j}::{k}"]).double().reshape(-1)
        gerr[k] = float((g - ref).abs().max()) / float(z[f"gnorm{j}::{k}"][1])
    print(f"minibatch {j}: grad norm {gn:.7g} vs {z['grad_norms'][j]:.7g}; worst relative "
          f"grad error per tensor: " + ", ".join(f"{k} {e:.2g}" for k, e in gerr.items()))
    tr._opt_step()
    torch.cuda.synchronize()
    st = tr.stats[j].cpu().numpy()
    ref = z["stats"][j]
    np.testing.assert_allclose(st, ref, rtol=1e-4, atol=1e-6, err_msg=f"stats mb {j}")
    assert abs(gn - z["grad_norms"][j]) <= 1e-4 * z["grad_norms"][j], (j, gn)
    assert max(gerr.values()) <= 1e-3, gerr
    worst = 0.0
    for k, p in params.items():
        got = p.detach().cpu().reshape(-1)
        if f"pick::{k}" in z:
            got = got[torch.from_numpy(z[f"pick::{k}"])]
        ref = torch.from_numpy(z[f"sd{j + 1}::{k}"]).reshape(-1)
        err = (got - ref).abs()
        worst = max(worst, float(err.max()))
        assert float(err.max()) <= 0.01 * LR, (j, k, float(err.max()))
        assert float((err > 2e-7).float().mean()) < 0.01, (j, k)
    print(f"minibatch {j}: worst |param - ref| = {worst:.3g} ({worst / LR:.3g} lr)")
