"""HIP kernels vs the oracle (and the reference fixtures), through the C-ABI (-m gpu)."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from oracle import ocppo_oracle as O

pytestmark = pytest.mark.gpu


def T(x, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    return t.to(dev) if dtype is None else t.to(device=dev, dtype=dtype)


def bits(t):
    return t.detach().cpu().numpy().view(np.uint32)


@pytest.fixture(scope="module")
def ops():
    from oc_cleanrl_amd import ops

    return ops


# ---------------------------------------------------------------------------------------------
# GAE: bit-exact
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(os.path.basename(p) for p in glob.glob(str(GOLDEN / "gae_*.npz"))))
def test_gae_golden_bitwise(ops, dev, name):
    z = golden(name)
    adv, ret = ops.gae(T(z["rewards"], dev), T(z["values"], dev), T(z["dones"], dev),
                       T(z["next_value"], dev), T(z["next_done"], dev), float(z["gamma"]),
                       float(z["gae_lambda"]))
    torch.cuda.synchronize()
    assert np.array_equal(bits(adv), z["advantages"].view(np.uint32))
    assert np.array_equal(bits(ret), z["returns"].view(np.uint32))


@pytest.mark.parametrize("T_,N", [(1, 1), (128, 1), (7, 5), (128, 128), (200, 130), (64, 1001),
                                  (128, 1024), (33, 1030), (200, 2048), (128, 4096), (300, 8192),
                                  (129, 65535), (128, 65536), (16, 65540), (33, 262144)])
def test_gae_random_bitwise_vs_oracle(ops, dev, T_, N):
    rng = np.random.default_rng(T_ * 7919 + N)
    r = rng.standard_normal((T_, N)).astype(np.float32)
    v = (rng.standard_normal((T_, N)) * 3).astype(np.float32)
    d = (rng.random((T_, N)) < 0.1).astype(np.float32)
    nv = rng.standard_normal(N).astype(np.float32)
    nd = (rng.random(N) < 0.1).astype(np.float32)
    adv, ret = ops.gae(T(r, dev), T(v, dev), T(d, dev), T(nv, dev), T(nd, dev), 0.99, 0.95)
    ea, er = O.gae(r, v, d, nv, nd, 0.99, 0.95)
    assert np.array_equal(bits(adv), ea.view(np.uint32))
    assert np.array_equal(bits(ret), er.view(np.uint32))


def test_gae_rejects_bad_shapes(ops, dev):
    r = torch.zeros(8, 4, device=dev)
    with pytest.raises(ValueError):
        ops.gae(r, r, r, torch.zeros(3, device=dev), torch.zeros(4, device=dev), 0.99, 0.95)
    with pytest.raises(ValueError):
        ops.gae(r.cpu(), r, r, r[0], r[0], 0.99, 0.95)


# ---------------------------------------------------------------------------------------------
# fused PPO loss
# ---------------------------------------------------------------------------------------------
def _loss_args(z, dev):
    return (T(z["logits"], dev), T(z["new_value"], dev), T(z["b_actions"], dev),
            T(z["b_logprobs"], dev), T(z["b_advantages"], dev), T(z["b_returns"], dev),
            T(z["b_values"], dev))


def _cfg(z):
    return dict(clip_coef=float(z["clip_coef"]), ent_coef=float(z["ent_coef"]),
                vf_coef=float(z["vf_coef"]), norm_adv=bool(z["norm_adv"]),
                clip_vloss=bool(z["clip_vloss"]))


@pytest.mark.parametrize("name", sorted(os.path.basename(p) for p in glob.glob(str(GOLDEN / "loss_*.npz"))))
def test_loss_golden(ops, dev, name):
    z = golden(name)
    stats, dl, dv = ops.ppo_loss_fwd_bwd(*_loss_args(z, dev), mb_inds=T(z["mb_inds"], dev),
                                         **_cfg(z))
    np.testing.assert_allclose(stats.cpu().numpy(), z["stats"], rtol=2e-6, atol=3e-7)
    sl = np.abs(z["dlogits"]).max()
    np.testing.assert_allclose(dl.cpu().numpy(), z["dlogits"], rtol=0, atol=1e-6 * sl)
    np.testing.assert_allclose(dv.cpu().numpy(), z["dvalue"], rtol=0,
                               atol=1e-6 * np.abs(z["dvalue"]).max())


@pytest.mark.parametrize("M,A,B", [(1, 6, 1), (255, 4, 1000), (4096, 6, 16384), (8192, 4, 32768),
                                   (5000, 18, 5000), (65536, 6, 131072),
                                   (300000, 6, 300000)])  # > grid cap: blocks walk tiles
@pytest.mark.parametrize("norm_adv,clip_vloss", [(True, True), (False, False)])
def test_loss_random_vs_oracle(ops, dev, M, A, B, norm_adv, clip_vloss):
    if M == 1 and norm_adv:
        pytest.skip("std of one element is NaN in the reference too")
    rng = np.random.default_rng(M + A)
    logits = (rng.standard_normal((M, A)) * 2).astype(np.float32)
    b_actions = rng.integers(0, A, B).astype(np.int64)
    b_logprobs = (rng.standard_normal(B) * 0.2 - 1.7).astype(np.float32)
    b_adv = (rng.standard_normal(B) * 2).astype(np.float32)
    b_ret = rng.standard_normal(B).astype(np.float32)
    b_val = rng.standard_normal(B).astype(np.float32)
    v = (b_val[:M] + rng.standard_normal(M) * 0.2).astype(np.float32)
    mb = rng.permutation(B)[:M].astype(np.int64)
    cfg = dict(clip_coef=0.1, ent_coef=0.01, vf_coef=0.5, norm_adv=norm_adv, clip_vloss=clip_vloss)
    stats, dl, dv = ops.ppo_loss_fwd_bwd(T(logits, dev), T(v, dev), T(b_actions, dev),
                                         T(b_logprobs, dev), T(b_adv, dev), T(b_ret, dev),
                                         T(b_val, dev), mb_inds=T(mb, dev), **cfg)
    es, edl, edv = O.ppo_loss_fwd_bwd(logits, v, b_actions, b_logprobs, b_adv, b_ret, b_val, mb,
                                      **cfg)
    np.testing.assert_allclose(stats.cpu().numpy(), es, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dl.cpu().numpy(), edl, rtol=0, atol=2e-6 * np.abs(edl).max())
    np.testing.assert_allclose(dv.cpu().numpy(), edv, rtol=0, atol=2e-6 * np.abs(edv).max())


@pytest.mark.parametrize("M,A", [(262144, 6), (262144 + 777, 6), (1 << 20, 4), (300001, 3),
                                 (262147, 9), (270000, 18)])
def test_loss_streaming_form_vs_oracle_and_tile_form(ops, dev, M, A):
    """Prepared (contiguous) records at M >= 256 x 1024 take the 16-B-per-lane streaming kernel:
    same per-element arithmetic as the 256-element-tile kernel (dlogits / dvalue bit-identical),
    stats within f32 summation-order noise, both against the oracle."""
    rng = np.random.default_rng(M + A)
    logits = (rng.standard_normal((M, A)) * 2).astype(np.float32)
    acts = rng.integers(0, A, M).astype(np.int64)
    lp = (rng.standard_normal(M) * 0.2 - 1.7).astype(np.float32)
    adv = (rng.standard_normal(M) * 2).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    val = rng.standard_normal(M).astype(np.float32)
    v = (val + rng.standard_normal(M) * 0.2).astype(np.float32)
    cfg = dict(clip_coef=0.1, ent_coef=0.01, vf_coef=0.5, norm_adv=True, clip_vloss=True)
    args = [T(x, dev) for x in (logits, v, acts, lp, adv, ret, val)]
    st = ops.minibatch_adv_stats(args[4], torch.arange(M, device=dev), M)[0]
    s_vec, d_vec, v_vec = ops.ppo_loss_fwd_bwd(*args, adv_stats=st, **cfg)
    # the tile kernel: same records through an identity index
    ident = torch.arange(M, device=dev)
    s_til, d_til, v_til = ops.ppo_loss_fwd_bwd(*args, mb_inds=ident, adv_stats=st, **cfg)
    assert torch.equal(d_vec, d_til) and torch.equal(v_vec, v_til)
    torch.testing.assert_close(s_vec, s_til, rtol=2e-6, atol=1e-7)
    es, edl, edv = O.ppo_loss_fwd_bwd(logits, v, acts, lp, adv, ret, val, np.arange(M), **cfg)
    np.testing.assert_allclose(s_vec.cpu().numpy(), es, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(d_vec.cpu().numpy(), edl, rtol=0, atol=2e-6 * np.abs(edl).max())
    np.testing.assert_allclose(v_vec.cpu().numpy(), edv, rtol=0, atol=2e-6 * np.abs(edv).max())


def test_loss_deterministic_and_graph_replayable(ops, dev):
    z = golden("loss_norm_clip.npz")
    args = _loss_args(z, dev)
    mb = T(z["mb_inds"], dev)
    ws = ops.LossWorkspace(len(z["mb_inds"]), z["logits"].shape[1], dev)
    s1, d1, v1 = ops.ppo_loss_fwd_bwd(*args, mb_inds=mb, workspace=ws, **_cfg(z))
    s1, d1, v1 = s1.clone(), d1.clone(), v1.clone()
    st = torch.empty(9, device=dev)
    dl = torch.empty_like(d1)
    dv = torch.empty_like(v1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.ppo_loss_fwd_bwd(*args, mb_inds=mb, workspace=ws, stats=st, dlogits=dl, dvalue=dv,
                             **_cfg(z))
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.ppo_loss_fwd_bwd(*args, mb_inds=mb, workspace=ws, stats=st, dlogits=dl, dvalue=dv,
                             **_cfg(z))
    for _ in range(3):
        st.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(st, s1) and torch.equal(dl, d1) and torch.equal(dv, v1)


def test_loss_precomputed_adv_stats_match(ops, dev):
    z = golden("loss_norm_clip.npz")
    args = _loss_args(z, dev)
    mb = T(z["mb_inds"], dev)
    st = ops.minibatch_adv_stats(args[4], mb, len(z["mb_inds"]))
    np.testing.assert_allclose(st.cpu().numpy()[0], z["stats"][7:9], rtol=1e-6)
    a = ops.ppo_loss_fwd_bwd(*args, mb_inds=mb, **_cfg(z))
    b = ops.ppo_loss_fwd_bwd(*args, mb_inds=mb, adv_stats=st[0], **_cfg(z))
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_minibatch_adv_stats_many(ops, dev):
    rng = np.random.default_rng(3)
    B, M = 16384, 4096
    adv = (rng.standard_normal(B) * 3 + 0.5).astype(np.float32)
    perm = np.concatenate([rng.permutation(B) for _ in range(4)]).astype(np.int64)
    st = ops.minibatch_adv_stats(T(adv, dev), T(perm, dev), M)
    np.testing.assert_allclose(st.cpu().numpy(), O.adv_stats(adv, perm, M), rtol=2e-6)


def test_loss_autograd_function(ops, dev):
    z = golden("loss_ties.npz")
    lg = T(z["logits"], dev).requires_grad_(True)
    v = T(z["new_value"], dev).view(-1, 1).requires_grad_(True)
    a = _loss_args(z, dev)
    loss, stats = ops.ppo_loss(lg, v, *a[2:], mb_inds=T(z["mb_inds"], dev), **_cfg(z))
    (2.0 * loss).backward()
    np.testing.assert_allclose(lg.grad.cpu().numpy(), 2 * z["dlogits"], rtol=0,
                               atol=2e-6 * np.abs(z["dlogits"]).max())
    np.testing.assert_allclose(v.grad.view(-1).cpu().numpy(), 2 * z["dvalue"], rtol=0,
                               atol=2e-6 * np.abs(z["dvalue"]).max())
    assert float(loss) == pytest.approx(float(z["stats"][0]), rel=2e-6)


# ---------------------------------------------------------------------------------------------
# Categorical action head
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", sorted(os.path.basename(p) for p in glob.glob(str(GOLDEN / "sample_*.npz"))))
def test_sample_golden(ops, dev, name):
    z = golden(name)
    N = len(z["action"])
    val = torch.arange(N, dtype=torch.float32, device=dev)
    vout = torch.empty(N, device=dev)
    ent = torch.empty(N, device=dev)
    a, lp, _ = ops.categorical_sample(T(z["logits"], dev), T(z["noise"], dev), entropy_out=ent,
                                      value_in=val, value_out=vout)
    assert np.array_equal(a.cpu().numpy(), z["action"])
    np.testing.assert_allclose(lp.cpu().numpy(), z["logprob"], rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(ent.cpu().numpy(), z["entropy"], rtol=1e-6, atol=2e-6)
    assert torch.equal(vout, val)


@pytest.mark.parametrize("A", [2, 4, 6, 18])
def test_sample_matches_torch_categorical_on_device(ops, dev, A):
    """Same generator state → torch's own Categorical.sample() and our kernel pick the same
    actions (torch draws Exp(1) noise of shape [N, A] and takes argmax(probs / noise))."""
    N = 8192
    g = torch.Generator(device=dev)
    logits = torch.randn(N, A, device=dev, generator=g.manual_seed(5)) * 3
    g.manual_seed(11)
    dist = torch.distributions.Categorical(logits=logits)
    ref = torch.multinomial(dist.probs, 1, True, generator=g).view(-1)
    g.manual_seed(11)
    noise = torch.empty(N, A, device=dev).exponential_(generator=g)
    a, lp, _ = ops.categorical_sample(logits, noise)
    assert torch.equal(a, ref)
    torch.testing.assert_close(lp, dist.log_prob(a), rtol=1e-6, atol=2e-6)


def _gen_state(gen, dev):
    """A generator's (seed, philox offset) as the device [2] state the sampling kernels read."""
    seed = gen.initial_seed()
    return torch.tensor([seed if seed < 1 << 63 else seed - (1 << 64), gen.get_offset()],
                        dtype=torch.int64, device=dev)


def _default_gen(dev):
    torch.cuda.init()  # default_generators is empty until the runtime is initialised
    return torch.cuda.default_generators[dev.index or 0]


@pytest.mark.parametrize("numel", [1, 6, 768, 1000, 3072 * 7, 256 * 2048 + 5,
                                   4 * 256 * 2048 + 17, 9 * 256 * 2048 + 1])
@pytest.mark.parametrize("seed", [0, 1, 2 ** 63 + 12345])
def test_philox_exponential_is_torch_exponential(ops, dev, numel, seed):
    """ocppo_philox_exponential = torch.empty(numel).exponential_() on the device generator,
    bit for bit: torch's grid geometry (one uniform4 per thread up to 4 grid strides, components
    1-3 and later draws beyond), its Philox counter layout, uniform conversion and log transform
    (ocppo_philox.h); and the generator advances by the increment the geometry reports."""
    g = _default_gen(dev)
    g.manual_seed(seed)
    g.set_offset(8 * 4)
    state = _gen_state(g, dev)
    stride, inc = ops.torch_exponential_geometry(numel, dev)
    ref = torch.empty(numel, device=dev).exponential_()
    assert g.get_offset() == 8 * 4 + inc
    out = ops.philox_exponential(torch.empty(numel, device=dev), state, 0, stride)
    assert torch.equal(out, ref), int((out != ref).sum())
    # the next draw of the same shape: offset + inc
    ref2 = torch.empty(numel, device=dev).exponential_()
    out2 = ops.philox_exponential(torch.empty(numel, device=dev), state, inc, stride)
    assert torch.equal(out2, ref2)


@pytest.mark.parametrize("numel,steps", [(768, 128), (6, 3), (256 * 2048 + 5, 2)])
def test_philox_exponential_steps_are_successive_draws(ops, dev, numel, steps):
    """ocppo_philox_exponential_steps: `steps` successive torch exponential_ draws of one shape in
    one launch, bit for bit (a rollout's Categorical.sample noise)."""
    g = _default_gen(dev)
    g.manual_seed(77)
    g.set_offset(4 * 3)
    state = _gen_state(g, dev)
    stride, inc = ops.torch_exponential_geometry(numel, dev)
    ref = torch.stack([torch.empty(numel, device=dev).exponential_() for _ in range(steps)])
    out = ops.philox_exponential_steps(torch.empty(steps, numel, device=dev), state, 0, inc,
                                       stride)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("N,H,A", [(128, 512, 6), (7, 64, 18), (300001, 512, 6), (33, 100, 6)])
def test_policy_head_draws_the_torch_stream_itself(ops, dev, N, H, A):
    """The sampling kernels with philox state: the Exp(1) values they draw (and write) are
    torch's exponential_ at that generator state, and every output equals the same kernel fed
    torch's noise tensor -- fast head (E = 1 and E > 1), generic head, categorical sampler."""
    g = torch.Generator(device=dev).manual_seed(N + H + A)
    hidden = torch.relu(torch.randn(N, H, device=dev, generator=g))
    wa = torch.randn(A, H, device=dev, generator=g) * 0.05
    ba = torch.randn(A, device=dev, generator=g) * 0.1
    wc = torch.randn(1, H, device=dev, generator=g)
    bc = torch.randn(1, device=dev, generator=g)
    dg = _default_gen(dev)
    dg.manual_seed(77)
    state = _gen_state(dg, dev)
    stride, inc = ops.torch_exponential_geometry(N * A, dev)
    for step in range(2):
        ref_noise = torch.empty(N, A, device=dev).exponential_()
        ref = ops.policy_head_sample(hidden, wa, ba, wc, bc, ref_noise,
                                     entropy_out=torch.empty(N, device=dev))
        drawn = torch.empty(N, A, device=dev)
        got = ops.policy_head_sample(hidden, wa, ba, wc, bc, drawn,
                                     entropy_out=torch.empty(N, device=dev),
                                     philox=(state, step * inc, stride))
        assert torch.equal(drawn, ref_noise), step
        for x, y in zip(got, ref):
            assert torch.equal(x, y), step
        logits = torch.randn(N, A, device=dev, generator=g)
        a_ref, lp_ref, _ = ops.categorical_sample(logits, ref_noise)
        a, lp, _ = ops.categorical_sample(logits, None, philox=(state, step * inc, stride))
        assert torch.equal(a, a_ref) and torch.equal(lp, lp_ref)


def test_policy_head_env_step_draws_the_torch_stream_itself(ops, dev):
    from oc_cleanrl_amd.envs import SyntheticAtariEnv

    N, H, A, D = 128, 512, 6, 12
    g = torch.Generator(device=dev).manual_seed(3)
    hidden = torch.relu(torch.randn(N, H, device=dev, generator=g))
    wa = torch.randn(A, H, device=dev, generator=g) * 0.05
    ba = torch.randn(A, device=dev, generator=g) * 0.1
    wc = torch.randn(1, H, device=dev, generator=g)
    bc = torch.randn(1, device=dev, generator=g)
    envs = [SyntheticAtariEnv("ALE/Pong-v5", "obj", N, D, 5, dev) for _ in range(2)]
    for e in envs:
        e.reset()
    dg = _default_gen(dev)
    dg.manual_seed(5)
    state = _gen_state(dg, dev)
    stride, inc = ops.torch_exponential_geometry(N * A, dev)
    for t in range(3):
        noise = torch.empty(N, A, device=dev).exponential_()
        outs = [(torch.empty(N, dtype=torch.int64, device=dev), torch.empty(N, device=dev),
                 torch.empty(N, device=dev)) for _ in range(2)]
        ops.policy_head_env_step(hidden, wa, ba, wc, bc, noise, *outs[0], envs[0], t)
        ops.policy_head_env_step(hidden, wa, ba, wc, bc, None, *outs[1], envs[1], t,
                                 philox=(state, t * inc, stride))
        for x, y in zip(*outs):
            assert torch.equal(x, y), t
        for k in ("frame", "reward", "done", "ep_state"):
            assert torch.equal(getattr(envs[0], k), getattr(envs[1], k)), (t, k)


@pytest.mark.parametrize("A", [4, 18])
def test_logprob_entropy_fwd_bwd_vs_torch(ops, dev, A):
    N = 3000
    logits = (torch.randn(N, A, device=dev) * 2).requires_grad_(True)
    act = torch.randint(0, A, (N,), device=dev)
    lp, ent = ops.categorical_logprob_entropy(logits, act)
    g1, g2 = torch.randn(N, device=dev), torch.randn(N, device=dev)
    ((lp * g1).sum() + (ent * g2).sum()).backward()
    ours = logits.grad.clone()
    logits.grad = None
    d = torch.distributions.Categorical(logits=logits)
    rl, re = d.log_prob(act), d.entropy()
    ((rl * g1).sum() + (re * g2).sum()).backward()
    torch.testing.assert_close(lp, rl.detach(), rtol=1e-6, atol=2e-6)
    torch.testing.assert_close(ent, re.detach(), rtol=1e-6, atol=2e-6)
    torch.testing.assert_close(ours, logits.grad, rtol=1e-5, atol=2e-6)


# ---------------------------------------------------------------------------------------------
# rollout store / reset / gather: bit-exact
# ---------------------------------------------------------------------------------------------
STORE_DT = {"f32": torch.float32, "bf16": torch.bfloat16, "u8": torch.uint8}


@pytest.mark.parametrize("obs_dt", ["f32", "bf16", "u8"])
@pytest.mark.parametrize("pixel,N,D", [(False, 128, 12), (False, 7, 6), (False, 5, 3),
                                       (True, 16, 7056), (True, 3, 5)])
def test_rollout_store_bitwise(ops, dev, obs_dt, pixel, N, D):
    rng = np.random.default_rng(N * D)
    W = 4
    hi = 256 if pixel else 210
    prev = rng.integers(0, hi, (N, W, D)).astype(np.float32)
    frame = rng.integers(0, hi, (N, D))
    frame = frame.astype(np.uint8) if pixel else frame.astype(np.float32)
    done = (rng.random(N) < 0.3).astype(np.float32)
    reward = rng.standard_normal(N).astype(np.float32)
    dt = STORE_DT[obs_dt]
    prev_t = T(prev, dev).to(dt)
    out = torch.empty_like(prev_t)
    net = torch.empty(N, W, D, device=dev)
    rout = torch.empty(N, device=dev)
    dout = torch.empty(N, device=dev)
    ops.rollout_store(T(frame, dev), T(reward, dev), T(done, dev), prev_t, out, net, rout, dout)
    exp = O.rollout_store(frame.astype(np.float32), done, prev, obs_dt)
    assert np.array_equal(out.float().cpu().numpy(), exp)
    assert np.array_equal(net.cpu().numpy(), exp)
    assert torch.equal(rout.cpu(), torch.from_numpy(reward))
    assert torch.equal(dout.cpu(), torch.from_numpy(done))


@pytest.mark.parametrize("layout", ["plain", "cl", "vecnorm"])
@pytest.mark.parametrize("pixel,N,W,D", [(False, 64, 4, 12), (False, 9, 3, 6), (True, 8, 4, 7056),
                                         (True, 5, 3, 36)])
def test_rollout_store_reset_stack_bitwise(ops, dev, layout, pixel, N, W, D):
    """Done rows take the env's own reset observation (reset_prev ++ frame) instead of the
    FrameStack fill -- a host env whose reset stack holds distinct frames (NoopReset/FireReset
    steps, EpisodicLifeEnv's life-loss dones, ppo_atari_oc.py:278-282)."""
    rng = np.random.default_rng(N * D + W)
    hi = 256 if pixel else 210
    npdt = np.uint8 if pixel else np.float32
    prev = rng.integers(0, hi, (N, W, D)).astype(np.float32)
    frame = rng.integers(0, hi, (N, D)).astype(npdt)
    rp = rng.integers(0, hi, (N, W - 1, D)).astype(npdt)
    done = (rng.random(N) < 0.4).astype(np.float32)
    done[0] = 1.0
    reward = rng.standard_normal(N).astype(np.float32)
    dt = torch.uint8 if pixel else torch.bfloat16
    prev_t = T(prev, dev).to(dt)
    out = torch.empty_like(prev_t)
    exp = O.rollout_store(frame.astype(np.float32), done, prev, "u8" if pixel else "bf16",
                          reset_prev=rp)
    args = (T(frame, dev), T(reward, dev), T(done, dev), prev_t, out)
    if layout == "cl":
        if not pixel:
            pytest.skip("channels-last network input is a pixel-stack layout")
        side = int(round(D ** 0.5))
        net = torch.empty((N, W, side, side), device=dev, memory_format=torch.channels_last)
        ops.rollout_store(*args, net, reset_prev=T(rp, dev))
        got_net = net.contiguous().cpu().numpy().reshape(N, W, D)
    elif layout == "vecnorm":
        net = torch.empty(N, W, D, device=dev)
        ret = torch.zeros(N, dtype=torch.float64, device=dev)
        rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=dev)
        rout = torch.empty(N, device=dev)
        ops.rollout_store_vecnorm(*args, net, torch.empty(N, device=dev), ret, rms, rout,
                                  reset_prev=T(rp, dev))
        got_net = net.cpu().numpy()
    else:
        net = torch.empty(N, W, D, device=dev)
        ops.rollout_store(*args, net, reset_prev=T(rp, dev))
        got_net = net.cpu().numpy()
    assert np.array_equal(out.float().cpu().numpy(), exp)
    assert np.array_equal(got_net, exp)


def test_bf16_conversion_rounds_to_nearest_even(ops, dev):
    x = torch.tensor([[1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, 300.5, -0.0]], device=dev)
    prev = torch.zeros(1, 1, 4, dtype=torch.bfloat16, device=dev)
    out = torch.empty_like(prev)
    ops.rollout_store(x, torch.zeros(1, device=dev), torch.ones(1, device=dev), prev, out)
    assert torch.equal(out.view(-1), x.view(-1).to(torch.bfloat16))


@pytest.mark.parametrize("src_dt", ["f32", "bf16", "u8"])
@pytest.mark.parametrize("B,shape,M", [(16384, (4, 12), 4096), (300, (4, 84, 84), 64),
                                       (50, (3, 5), 77)])
def test_gather_rows_bitwise(ops, dev, src_dt, B, shape, M):
    rng = np.random.default_rng(B + M)
    src = rng.integers(0, 256, (B,) + shape).astype(np.float32)
    idx = rng.integers(0, B, M).astype(np.int64)
    out = ops.gather_rows(T(src, dev).to(STORE_DT[src_dt]), T(idx, dev))
    assert np.array_equal(out.cpu().numpy(), src[idx])


@pytest.mark.parametrize("N,W,E,ld", [(128, 4, 512, 512), (128, 4, 512, 1536), (7, 3, 5, 9),
                                       (1, 4, 12, 12), (300, 2, 64, 64)])
def test_frame_cache_shift_bitwise(ops, dev, N, W, E, ld):
    """The rollout's encoding cache follows the frame stack's shift / reset-fill rule exactly."""
    rng = np.random.default_rng(N * W + E)
    enc = rng.standard_normal((N, W, E)).astype(np.float32)
    big = rng.standard_normal((N, ld)).astype(np.float32)
    done = (rng.random(N) < 0.3).astype(np.float32)
    enc_t = T(enc, dev)
    fresh = T(big, dev)[:, :E]
    ops.frame_cache_shift(enc_t, fresh, T(done, dev))
    exp = O.frame_cache_shift(enc, big[:, :E], done)
    assert np.array_equal(enc_t.cpu().numpy(), exp)
    # done=None: a pure shift
    enc_t = T(enc, dev)
    ops.frame_cache_shift(enc_t, fresh)
    assert np.array_equal(enc_t.cpu().numpy(), O.frame_cache_shift(enc, big[:, :E], done * 0))


def test_frame_cache_shift_rejects_bad_shapes(ops, dev):
    enc = torch.zeros(4, 4, 8, device=dev)
    with pytest.raises(ValueError):
        ops.frame_cache_shift(enc, torch.zeros(4, 7, device=dev))
    with pytest.raises(ValueError):
        ops.frame_cache_shift(enc, torch.zeros(4, 8, device="cpu"))


@pytest.mark.parametrize("M,K,N,ldx", [(128, 12, 256, 48), (512, 256, 512, 256), (128, 2048, 512, 2048),
                                      (37, 7, 19, 7), (1, 512, 1024, 512), (130, 1024, 513, 1028),
                                      (256, 3136, 512, 3136), (16, 16, 16, 16)])
@pytest.mark.parametrize("relu", [True, False])
def test_linear_act_vs_torch(ops, dev, M, K, N, ldx, relu):
    """Rollout Linear(+ReLU) on the f32 matrix cores: within f32 summation-order error of
    F.linear (error bound relative to sum |x*w|, the f32 dot-product error scale)."""
    g = torch.Generator(device=dev).manual_seed(M * K + N)
    big = torch.randn(M, ldx, device=dev, generator=g) * 3
    x = big[:, :K]
    w = torch.randn(N, K, device=dev, generator=g) * 0.05
    b = torch.randn(N, device=dev, generator=g)
    y = ops.linear_act(x, w, b, relu)
    ref = x.double() @ w.double().t() + b.double()
    if relu:
        ref = torch.relu(ref)
    scale = (x.double().abs() @ w.double().abs().t() + b.double().abs()).max().item()
    assert (y.double() - ref).abs().max().item() <= 4e-7 * scale
    # no bias, strided output rows
    full = torch.full((M, N + 3), 7.0, device=dev)
    out = full[:, :N]
    ops.linear_act(x, w, None, False, out)
    ref0 = x.double() @ w.double().t()
    assert (out.double() - ref0).abs().max().item() <= 4e-7 * scale
    assert torch.all(full[:, N:] == 7.0)


def test_linear_act_deterministic(ops, dev):
    x = torch.randn(128, 2048, device=dev)
    w = torch.randn(512, 2048, device=dev)
    b = torch.randn(512, device=dev)
    y1 = ops.linear_act(x, w, b, True)
    y2 = ops.linear_act(x, w, b, True)
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("S,shape", [(8, (1024, 512)), (4, (512, 256)), (16, (256, 12)),
                                     (8, (6, 512)), (1, (4, 4)), (2, (3, 4))])
def test_sum_splits_is_the_split_order_fold(ops, dev, S, shape):
    """Split-K combine: bit-identical to ((p0 + p1) + p2) + ... added in f64 and rounded once to
    f32, written into a view."""
    g = torch.Generator(device=dev).manual_seed(S * 1000 + shape[0])
    part = torch.randn((S,) + shape, device=dev, generator=g)
    ref = part[0].double()
    for s in range(1, S):
        ref = ref + part[s].double()
    ref = ref.float()
    flat = torch.full((shape[0] * shape[1] + 8,), 5.0, device=dev)
    out = flat[4:4 + shape[0] * shape[1]].view(shape)
    ops.sum_splits(part, out)
    assert torch.equal(out, ref)
    assert torch.all(flat[:4] == 5.0) and torch.all(flat[-4:] == 5.0)


def test_obs_reset(ops, dev):
    frame = torch.randint(0, 256, (9, 7056), dtype=torch.uint8, device=dev)
    out = torch.empty(9, 4, 7056, dtype=torch.bfloat16, device=dev)
    net = torch.empty(9, 4, 7056, device=dev)
    ops.obs_reset(frame, out, net)
    assert torch.equal(net, frame.float()[:, None].expand(9, 4, 7056))
    assert torch.equal(out.float(), net)


# ---------------------------------------------------------------------------------------------
# VecNormalize reward normalisation (f64) and the synthetic env
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("N", [1, 128, 1500])
def test_vecnorm_vs_oracle(ops, dev, N):
    rng = np.random.default_rng(N)
    ret_t = torch.zeros(N, dtype=torch.float64, device=dev)
    rms_t = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=dev)
    ret, rms = np.zeros(N), (0.0, 1.0, 1e-4)
    for step in range(20):
        r = np.where(rng.random(N) < 0.1, rng.choice([-1.0, 1.0], N), 0.0).astype(np.float32)
        d = (rng.random(N) < 0.05).astype(np.float32)
        out_t = torch.empty(N, device=dev)
        ops.vecnorm_reward(T(r, dev), T(d, dev), ret_t, rms_t, out_t)
        out, ret, rms = O.vecnorm_reward(r, d, ret, rms)
        np.testing.assert_allclose(out_t.cpu().numpy(), out, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(ret_t.cpu().numpy(), ret, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(rms_t.cpu().numpy(), np.array(rms), rtol=1e-12)


@pytest.mark.parametrize("pixel,N,D", [(False, 128, 12), (False, 33, 6), (True, 8, 7056)])
def test_synth_env_bitwise_vs_oracle(ops, dev, pixel, N, D):
    base = torch.tensor([1000], dtype=torch.int64, device=dev)
    acts = torch.arange(N, device=dev) % 6
    frame = torch.empty(N, D, dtype=torch.uint8 if pixel else torch.float32, device=dev)
    rew = torch.empty(N, device=dev)
    done = torch.empty(N, device=dev)
    ops.synth_env_step(42, base, 5, acts, frame, rew, done)
    ef, er, ed = O.synth_env_step(42, 1005, acts.cpu().numpy(), N, D, pixel)
    assert np.array_equal(frame.cpu().numpy(), ef)
    assert np.array_equal(rew.cpu().numpy(), er)
    assert np.array_equal(done.cpu().numpy(), ed)


# ---------------------------------------------------------------------------------------------
# fused rollout policy head; fused store + VecNormalize
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("N,H,A", [(128, 512, 6), (256, 512, 4), (7, 64, 18), (33, 100, 6),
                                   (4096, 512, 6), (65, 256, 7), (9, 1024, 1), (130, 768, 3),
                                   (5, 2048, 6), (17, 512, 8),
                                   (300001, 512, 6), (20000, 1024, 3)])  # E > 1 env per wave
def test_policy_head_sample(ops, dev, N, H, A):
    g = torch.Generator(device=dev).manual_seed(N + H + A)
    hidden = torch.relu(torch.randn(N, H, device=dev, generator=g))
    wa = torch.randn(A, H, device=dev, generator=g) * 0.05
    ba = torch.randn(A, device=dev, generator=g) * 0.1
    wc = torch.randn(1, H, device=dev, generator=g)
    bc = torch.randn(1, device=dev, generator=g)
    noise = torch.empty(N, A, device=dev).exponential_(generator=g)
    logits = torch.empty(N, A, device=dev)
    ent = torch.empty(N, device=dev)
    act, lp, val = ops.policy_head_sample(hidden, wa, ba, wc, bc, noise, entropy_out=ent,
                                          logits_out=logits)
    ref_logits = torch.nn.functional.linear(hidden, wa, ba)
    ref_value = torch.nn.functional.linear(hidden, wc, bc).view(-1)
    torch.testing.assert_close(logits, ref_logits, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(val, ref_value, rtol=1e-5, atol=1e-4)
    # the sampler applied to the head's own logits: bit-exact actions / log-probs / entropy
    a2, lp2, e2 = ops.categorical_sample(logits, noise, entropy_out=torch.empty(N, device=dev))
    assert torch.equal(act, a2) and torch.equal(lp, lp2) and torch.equal(ent, e2)


@pytest.mark.parametrize("N,H,A,D", [(128, 512, 6, 12), (1, 256, 3, 4), (3072, 512, 7, 12),
                                     (2048, 1024, 6, 100), (77, 768, 1, 65)])
def test_policy_head_env_step_is_bitwise_the_two_launches(ops, dev, N, H, A, D):
    """ocppo_policy_head_env_step = ocppo_policy_head_sample then ocppo_synth_env_step on its
    actions: bit for bit (actions, log-probs, values, next frame, reward, done, episode counters),
    over several steps so the counters carry."""
    from oc_cleanrl_amd.envs import SyntheticAtariEnv

    g = torch.Generator(device=dev).manual_seed(N + H + A + D)
    hidden = torch.relu(torch.randn(N, H, device=dev, generator=g))
    wa = torch.randn(A, H, device=dev, generator=g) * 0.05
    ba = torch.randn(A, device=dev, generator=g) * 0.1
    wc = torch.randn(1, H, device=dev, generator=g)
    bc = torch.randn(1, device=dev, generator=g)
    envs = [SyntheticAtariEnv("ALE/Pong-v5", "obj", N, D, 5, dev) for _ in range(2)]
    for e in envs:
        e.reset()
    envs[0].ep_state.uniform_(0, 3, generator=g)
    envs[1].ep_state.copy_(envs[0].ep_state)
    assert ops.policy_head_env_ok(hidden, wa, wc, envs[0])
    for t in range(4):
        noise = torch.empty(N, A, device=dev).exponential_(generator=g)
        a0, l0, v0 = ops.policy_head_sample(hidden, wa, ba, wc, bc, noise)
        envs[0].step(a0, t)
        a1, l1, v1 = (torch.empty_like(a0), torch.empty_like(l0), torch.empty_like(v0))
        ops.policy_head_env_step(hidden, wa, ba, wc, bc, noise, a1, l1, v1, envs[1], t)
        torch.cuda.synchronize()
        assert torch.equal(a0, a1) and torch.equal(l0, l1) and torch.equal(v0, v1)
        for k in ("frame", "reward", "done", "ep_state"):
            assert torch.equal(getattr(envs[0], k), getattr(envs[1], k)), (t, k)
        hidden = torch.relu(hidden + 0.01 * torch.randn(N, H, device=dev, generator=g))
    # past one env per wave (N > 3072): the host gate says no and the C entry refuses
    n = 3073
    e = SyntheticAtariEnv("ALE/Pong-v5", "obj", n, D, 5, dev)
    big, w5, c5 = (torch.zeros(n, 512, device=dev), torch.zeros(A, 512, device=dev),
                   torch.zeros(1, 512, device=dev))
    assert not ops.policy_head_env_ok(big, w5, c5, e)
    with pytest.raises(RuntimeError, match="bad sizes"):
        ops.policy_head_env_step(big, w5, ba, c5, bc, torch.ones(n, A, device=dev),
                                 torch.empty(n, dtype=torch.int64, device=dev),
                                 torch.empty(n, device=dev), torch.empty(n, device=dev), e, 0)


@pytest.mark.parametrize("pixel,N,D", [(False, 128, 12), (True, 16, 7056), (False, 1000, 6)])
def test_store_vecnorm_equals_separate_kernels(ops, dev, pixel, N, D):
    rng = np.random.default_rng(N)
    W = 4
    frame = rng.integers(0, 200, (N, D))
    frame = T(frame.astype(np.uint8) if pixel else frame.astype(np.float32), dev)
    prev = T(rng.integers(0, 200, (N, W, D)).astype(np.float32), dev).to(torch.bfloat16)
    done = T((rng.random(N) < 0.2).astype(np.float32), dev)
    rew = T(np.where(rng.random(N) < 0.3, 1.0, 0.0).astype(np.float32), dev)
    ret0 = T(rng.standard_normal(N), dev)
    rms0 = torch.tensor([0.1, 2.0, 50.0], dtype=torch.float64, device=dev)
    outs = []
    for fused in (False, True):
        ret, rms = ret0.clone(), rms0.clone()
        o = torch.empty_like(prev)
        net = torch.empty(N, W, D, device=dev)
        dout, rout = torch.empty(N, device=dev), torch.empty(N, device=dev)
        if fused:
            ops.rollout_store_vecnorm(frame, rew, done, prev, o, net, dout, ret, rms, rout)
        else:
            ops.rollout_store(frame, rew, done, prev, o, net, None, dout)
            ops.vecnorm_reward(rew, done, ret, rms, rout)
        outs.append((o, net, dout, rout, ret, rms))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


# ---------------------------------------------------------------------------------------------
# fused clip_grad_norm_ + Adam over flat buffers
# ---------------------------------------------------------------------------------------------
def _mlp(dev, seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 64), torch.nn.ReLU(), torch.nn.Linear(64, 33),
                               torch.nn.ReLU(), torch.nn.Linear(33, 7)).to(dev)


@pytest.mark.parametrize("max_norm,scale", [(0.5, 1.0), (0.0, 1.0), (100.0, 0.25)])
def test_flat_adam_matches_torch_adam_and_clip(ops, dev, max_norm, scale):
    a, b = _mlp(dev), _mlp(dev)
    opt_ref = torch.optim.Adam(a.parameters(), lr=2.5e-4, eps=1e-5)
    opt = ops.FlatAdam(b.parameters(), lr=2.5e-4, eps=1e-5, max_grad_norm=max_norm)
    g = torch.Generator(device=dev).manual_seed(1)
    for it in range(5):
        x = torch.randn(256, 12, device=dev, generator=g) * 3
        for p in a.parameters():
            p.grad = None
        (a(x) ** 2).mean().backward()
        for p in a.parameters():
            p.grad.mul_(scale)
        gn = torch.nn.utils.clip_grad_norm_(a.parameters(), max_norm) if max_norm > 0 else None
        opt_ref.step()
        opt.zero_grad()
        (b(x) ** 2).mean().backward()
        opt.step(grad_scale=scale)
        if gn is not None:
            torch.testing.assert_close(opt.scalars[1], gn, rtol=1e-5, atol=0)
    for p, q in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(q, p, rtol=2e-5, atol=2e-7)
    assert float(opt.scalars[0]) == 5.0


def test_flat_adam_vs_oracle_bit_level(ops, dev):
    rng = np.random.default_rng(0)
    P = 1000003  # the flat buffer pads it to a multiple of ops.FLAT_ALIGN; padding stays zero
    p0 = rng.standard_normal(P).astype(np.float32)
    w = torch.nn.Parameter(T(p0, dev))
    opt = ops.FlatAdam([w], lr=2.5e-4, eps=1e-5, max_grad_norm=0.5)
    assert opt.numel % ops.FLAT_ALIGN == 0 and opt.numel >= P
    p, m, v, step = p0, np.zeros(P, np.float32), np.zeros(P, np.float32), 0
    for it in range(3):
        gr = (rng.standard_normal(P) * 0.01).astype(np.float32)
        opt.grads[:P].copy_(T(gr, dev))
        opt.step()
        assert float(opt.params[P:].abs().sum()) == 0 and float(opt.exp_avg_sq[P:].abs().sum()) == 0
        p, m, v, step, total = O.clip_adam_step(p, gr, m, v, step, 2.5e-4, max_norm=0.5)
        np.testing.assert_allclose(float(opt.scalars[1]), total, rtol=1e-5)
        # the clip coefficient (f32 on device, f64 norm in the oracle) may differ by an ulp,
        # so compare at the scale of the moments / the update, not element-relative
        np.testing.assert_allclose(opt.exp_avg[:P].cpu().numpy(), m, rtol=0,
                                   atol=2e-6 * np.abs(m).max())
        np.testing.assert_allclose(w.detach().cpu().numpy(), p, rtol=1e-6, atol=1e-9)


def test_flat_adam_graph_replay(ops, dev):
    net = _mlp(dev)
    opt = ops.FlatAdam(net.parameters(), lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    x = torch.randn(64, 12, device=dev)

    def step():
        opt.zero_grad()
        (net(x) ** 2).mean().backward()
        opt.step()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    before = opt.params.clone()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert float(opt.scalars[0]) == 4.0 and not torch.equal(before, opt.params)


def test_minibatch_prepare_then_loss_equals_indexed_loss(ops, dev):
    rng = np.random.default_rng(9)
    B, M, A = 16384, 4096, 6
    b_act = T(rng.integers(0, A, B).astype(np.int64), dev)
    b_lp, b_adv, b_ret, b_val = (T(rng.standard_normal(B).astype(np.float32), dev) for _ in range(4))
    perm = T(np.concatenate([rng.permutation(B) for _ in range(2)]).astype(np.int64), dev)
    mb = ops.minibatch_prepare(perm, M, b_act, b_lp, b_adv, b_ret, b_val)
    ref_st = ops.minibatch_adv_stats(b_adv, perm, M)
    assert torch.equal(mb["adv_stats"], ref_st)
    for k, src in (("actions", b_act), ("logprobs", b_lp), ("advantages", b_adv),
                   ("returns", b_ret), ("values", b_val)):
        assert torch.equal(mb[k], src[perm])
    logits = T(rng.standard_normal((M, A)).astype(np.float32), dev)
    v = T(rng.standard_normal(M).astype(np.float32), dev)
    cfg = dict(clip_coef=0.1, ent_coef=0.01, vf_coef=0.5, norm_adv=True, clip_vloss=True)
    j = 1
    sl = slice(j * M, (j + 1) * M)
    a = ops.ppo_loss_fwd_bwd(logits, v, b_act, b_lp, b_adv, b_ret, b_val, mb_inds=perm[sl],
                             adv_stats=ref_st[j], **cfg)
    b = ops.ppo_loss_fwd_bwd(logits, v, mb["actions"][sl], mb["logprobs"][sl],
                             mb["advantages"][sl], mb["returns"][sl], mb["values"][sl],
                             adv_stats=mb["adv_stats"][j], **cfg)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("M,nmb,B", [(1, 3, 5), (333, 7, 1000), (20000, 3, 30011)])
def test_minibatch_prepare_shapes(ops, dev, M, nmb, B):
    """The gather runs over all nmb * M elements on one grid (ragged tails) and the statistics
    are ocppo_minibatch_adv_stats' over the same values (bitwise), for any M."""
    rng = np.random.default_rng(M + nmb)
    b_act = T(rng.integers(0, 6, B).astype(np.int64), dev)
    b_lp, b_adv, b_ret, b_val = (T(rng.standard_normal(B).astype(np.float32), dev) for _ in range(4))
    perm = T(rng.integers(0, B, nmb * M).astype(np.int64), dev)
    mb = ops.minibatch_prepare(perm, M, b_act, b_lp, b_adv, b_ret, b_val)
    for k, src in (("actions", b_act), ("logprobs", b_lp), ("advantages", b_adv),
                   ("returns", b_ret), ("values", b_val)):
        assert torch.equal(mb[k], src[perm]), k
    if M > 1:
        assert torch.equal(mb["adv_stats"], ops.minibatch_adv_stats(b_adv, perm, M))


# ---------------------------------------------------------------------------------------------
# DQN: fused TD loss, epsilon-greedy, HBM replay buffer
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["td_b32_a6.npz", "td_b256_a18.npz"])
def test_td_loss_golden(ops, dev, name):
    z = golden(name)
    stats, dq = ops.td_loss_fwd_bwd(T(z["q"], dev), T(z["q_next"], dev), T(z["actions"], dev),
                                    T(z["rewards"], dev), T(z["dones"], dev), float(z["gamma"]))
    np.testing.assert_allclose(stats.cpu().numpy(), [z["loss"], z["q_values"]], rtol=1e-6)
    assert np.array_equal(dq.cpu().numpy().view(np.uint32), z["dq"].view(np.uint32))


def test_epsilon_greedy(ops, dev):
    q = torch.randn(64, 6, device=dev)
    step = torch.tensor([10_000_000], dtype=torch.int64, device=dev)  # epsilon = end_e
    eps = torch.empty(1, device=dev)
    a = ops.epsilon_greedy(q, 1, step, 1.0, 0.0, 1000.0, epsilon_out=eps)
    assert float(eps) == 0.0 and torch.equal(a, q.argmax(1))
    step.fill_(0)  # epsilon = 1: every action random, uniform over A
    seen = torch.zeros(6, device=dev)
    for t in range(200):
        step.fill_(t)
        a = ops.epsilon_greedy(q, 1, step, 1.0, 1.0, 1e9)
        seen += torch.bincount(a, minlength=6).float()
    assert seen.min() > 0.1 * seen.mean()


@pytest.mark.parametrize("E,H,A", [(1, 512, 6), (37, 256, 8), (5, 1024, 3)])
def test_q_head_epsilon_greedy(ops, dev, E, H, A):
    """Q head + epsilon-greedy in one launch: q to f32 rounding of F.linear, and the action is
    exactly ocppo_epsilon_greedy's on the kernel's own q, greedy (epsilon = 0), random (1) and
    mixed."""
    g = torch.Generator(device=dev).manual_seed(E + H + A)
    h = torch.relu(torch.randn(E, H, device=dev, generator=g))
    wq = torch.randn(A, H, device=dev, generator=g) * H ** -0.5
    bq = torch.randn(A, device=dev, generator=g) * 0.1
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    for start_e, end_e, dur in ((0.0, 0.0, 10.0), (1.0, 1.0, 10.0), (1.0, 0.05, 50.0)):
        for t in (0, 7, 30, 100):
            step.fill_(t)
            q = torch.empty(E, A, device=dev)
            eps = torch.empty(1, device=dev)
            a = ops.q_head_epsilon_greedy(h, wq, bq, 3, step, start_e, end_e, dur,
                                          epsilon_out=eps, step_offset=1, q_out=q)
            torch.testing.assert_close(q, torch.nn.functional.linear(h, wq, bq), rtol=1e-5,
                                       atol=1e-5)
            eps2 = torch.empty(1, device=dev)
            a2 = ops.epsilon_greedy(q, 3, step, start_e, end_e, dur, epsilon_out=eps2,
                                    step_offset=1)
            assert torch.equal(a, a2) and torch.equal(eps, eps2)


@pytest.mark.parametrize("dt", [torch.uint8, torch.bfloat16])
def test_replay_buffer_semantics(ops, dev, dt):
    from oracle import ocppo_oracle as O

    size, E, shape = 10, 2, (4, 3)
    rb = ops.ReplayBuffer(size, E, shape, dev, obs_dtype=dt, seed=3)
    frames = [torch.full((E,) + shape, float(i), device=dev) + torch.arange(E, device=dev).view(E, 1, 1) * 100
              for i in range(14)]
    for i in range(13):  # wraps around once
        rb.add(frames[i], frames[i + 1], torch.full((E,), i, device=dev, dtype=torch.int64),
               torch.full((E,), float(i), device=dev), torch.zeros(E, device=dev))
        st = rb.state.cpu().tolist()
        assert st == [(i + 1) % size, int(i + 1 >= size)]
        out = rb.sample(64, with_indices=True)
        idx = out["indices"].cpu().numpy()
        allowed = O.replay_sample_law(st[0], st[1], size, 64)
        assert set(idx[:, 0].tolist()) <= allowed
        # obs of slot s is transition s's obs, the next obs is slot s+1's content
        for b in range(64):
            s, e = idx[b]
            tr = int(out["actions"][b])  # action == transition number
            assert float(out["rewards"][b]) == tr
            assert torch.equal(out["observations"][b], frames[tr][e].float())
            assert torch.equal(out["next_observations"][b], frames[tr + 1][e].float())


def test_clip_adam_abi_scalar_tail(ops, dev):
    """ocppo_clip_adam_step called through the C ABI with P % 4 != 0 (the scalar tail)."""
    from oc_cleanrl_amd import _lib

    rng = np.random.default_rng(3)
    P = 1003
    p0 = rng.standard_normal(P).astype(np.float32)
    gr = (rng.standard_normal(P) * 0.1).astype(np.float32)
    p, g = T(p0, dev), T(gr, dev)
    m, v = torch.zeros(P, device=dev), torch.zeros(P, device=dev)
    lr = torch.tensor([1e-3], device=dev)
    sc = torch.zeros(8, device=dev)
    ws = torch.zeros(int(_lib.LIB.ocppo_clip_adam_workspace_bytes(P)), dtype=torch.uint8, device=dev)
    _lib.call("ocppo_clip_adam_step", torch.cuda.current_stream(dev).cuda_stream, p.data_ptr(),
              g.data_ptr(), m.data_ptr(), v.data_ptr(), P, lr.data_ptr(), 0.9, 0.999, 1e-5, 0.5,
              0.5, sc.data_ptr(), ws.data_ptr(), ws.numel(), 0, None, None, None, None, None)
    ep, em, ev, step, total = O.clip_adam_step(p0, gr, np.zeros(P, np.float32),
                                               np.zeros(P, np.float32), 0, 1e-3, max_norm=0.5,
                                               grad_scale=0.5)
    np.testing.assert_allclose(float(sc[1]), total, rtol=1e-5)
    np.testing.assert_allclose(p.cpu().numpy(), ep, rtol=1e-6, atol=1e-9)


# ---------------------------------------------------------------------------------------------
# channels-last (NHWC) network input for the NatureCNN: same values, NHWC memory order
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("W,H,X", [(4, 84, 84), (4, 3, 5), (3, 4, 4), (1, 2, 6)])
@pytest.mark.parametrize("vecnorm", [False, True])
def test_store_channels_last_net_equals_plain(ops, dev, W, H, X, vecnorm):
    rng = np.random.default_rng(H * X + W)
    N, D = 9, H * X
    frame = T(rng.integers(0, 256, (N, D)).astype(np.uint8), dev)
    prev = T(rng.integers(0, 256, (N, W, D)).astype(np.uint8), dev)
    done = T((rng.random(N) < 0.3).astype(np.float32), dev)
    rew = T(rng.standard_normal(N).astype(np.float32), dev)
    res = []
    for cl in (False, True):
        o = torch.empty_like(prev)
        net = torch.empty((N, W, H, X), device=dev,
                          memory_format=torch.channels_last if cl else torch.contiguous_format)
        net.fill_(-1.0)
        dout, rout = torch.empty(N, device=dev), torch.empty(N, device=dev)
        if vecnorm:
            ret = torch.zeros(N, dtype=torch.float64, device=dev)
            rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=dev)
            ops.rollout_store_vecnorm(frame, rew, done, prev, o, net, dout, ret, rms, rout)
        else:
            ops.rollout_store(frame, rew, done, prev, o, net, rout, dout)
        res.append((o, net, dout, rout))
    assert res[1][1].is_contiguous(memory_format=torch.channels_last) or W == 1
    for x, y in zip(*res):
        assert torch.equal(x, y)
    exp = O.rollout_store(frame.cpu().numpy().astype(np.float32), done.cpu().numpy(),
                          prev.cpu().numpy().astype(np.float32), "u8")
    assert np.array_equal(res[1][1].cpu().numpy().reshape(N, W, D), exp)


def test_obs_reset_channels_last(ops, dev):
    frame = torch.randint(0, 256, (5, 84 * 84), dtype=torch.uint8, device=dev)
    out = torch.empty(5, 4, 84 * 84, dtype=torch.uint8, device=dev)
    net = torch.empty(5, 4, 84, 84, device=dev, memory_format=torch.channels_last)
    ops.obs_reset(frame, out, net)
    assert torch.equal(net, frame.float().view(5, 1, 84, 84).expand(5, 4, 84, 84))


@pytest.mark.parametrize("src_dt", ["u8", "bf16", "f32"])
@pytest.mark.parametrize("B,shape,M", [(300, (4, 84, 84), 64), (50, (3, 5, 7), 77), (20, (4, 2, 2), 5)])
def test_gather_rows_channels_last(ops, dev, src_dt, B, shape, M):
    rng = np.random.default_rng(B * M)
    src = rng.integers(0, 256, (B,) + shape).astype(np.float32)
    idx = rng.integers(0, B, M).astype(np.int64)
    out = torch.empty((M,) + shape, device=dev, memory_format=torch.channels_last).fill_(-1.0)
    ops.gather_rows(T(src, dev).to(STORE_DT[src_dt]), T(idx, dev), out)
    assert out.is_contiguous(memory_format=torch.channels_last)
    assert np.array_equal(out.cpu().numpy(), src[idx])


# ---------------------------------------------------------------------------------------------
# fused ReLU backward + bias gradient (autograd of Linear -> ReLU inside loss.backward())
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("R,N", [(12288, 1024), (4096, 512), (12288, 256), (7, 4), (33, 260),
                                 (100000, 12), (1, 16384)])
@pytest.mark.parametrize("relu", [True, False])
def test_relu_bias_grad_vs_torch(ops, dev, R, N, relu):
    g = torch.randn(R, N, device=dev)
    out = torch.relu(torch.randn(R, N, device=dev)) if relu else None
    if relu:
        out[::3, ::5] = 0.0  # exact zeros: threshold_backward's `<= 0` boundary
    gp, db = ops.relu_bias_grad(g, out)
    want = torch.ops.aten.threshold_backward(g, out, 0) if relu else g
    assert torch.equal(gp, want)
    ref = want.double().sum(0)
    scale = want.double().abs().sum(0).clamp_min(1e-30)
    assert ((db.double() - ref).abs() / scale).max().item() < 1e-6
    gp2, db2 = ops.relu_bias_grad(g, out)  # deterministic; tickets re-armed
    assert torch.equal(db, db2) and torch.equal(gp, gp2)


@pytest.mark.parametrize("R,N,K,S", [(12288, 512, 256, 4), (12288, 1024, 512, 8),
                                     (12288, 512, 1024, 8), (1000, 20, 8, 2)])
@pytest.mark.parametrize("relu", [True, False])
def test_relu_bias_grad_deferred_db(ops, dev, R, N, K, S, relu):
    """relu_bias_grad_partial + sum_splits_db (the bias gradient finished in the launch that
    combines the split-K weight gradient): gp bit-identical to threshold_backward, the weight
    gradient bit-identical to sum_splits, db to 1e-6 of sum |gp| per column."""
    g = torch.randn(R, N, device=dev)
    out = torch.relu(torch.randn(R, N, device=dev)) if relu else None
    if relu:
        out[::3, ::5] = 0.0
    x = torch.randn(R, K, device=dev)
    gp, dbp = ops.relu_bias_grad_partial(g, out)
    want = torch.ops.aten.threshold_backward(g, out, 0) if relu else g
    assert torch.equal(gp, want)
    part = torch.bmm(gp.view(S, R // S, N).transpose(1, 2), x.view(S, R // S, K))
    dw, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
    ops.sum_splits_db(part, dw, dbp, db)
    assert torch.equal(dw, ops.sum_splits(part))
    ref = want.double().sum(0)
    scale = want.double().abs().sum(0).clamp_min(1e-30)
    assert ((db.double() - ref).abs() / scale).max().item() < 1e-6
    db2 = torch.empty_like(db)
    ops.relu_bias_grad_partial(g, out)
    ops.sum_splits_db(part, dw, dbp, db2)
    assert torch.equal(db, db2)  # deterministic


def test_relu_bias_grad_graph_replay(ops, dev):
    g = torch.randn(3000, 512, device=dev)
    out = torch.relu(torch.randn(3000, 512, device=dev))
    gp = torch.empty_like(g)
    db = torch.empty(512, device=dev)
    ops.relu_bias_grad(g, out, db=db, gp=gp)
    ref = db.clone()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        ops.relu_bias_grad(g, out, db=db, gp=gp)
    db.zero_()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(db, ref)


def test_relu_bias_grad_rejects_bad_shapes(ops, dev):
    from oc_cleanrl_amd._lib import OcppoError

    with pytest.raises(OcppoError, match="bad sizes"):
        ops.relu_bias_grad(torch.randn(8, 6, device=dev))


@pytest.mark.parametrize("cl", [False, True])
def test_store_and_gather_scale255_equal_torch_division(ops, dev, cl):
    """OCPPO_NET_SCALE_255: the network copy holds exactly what NormalizeImg (x / 255.0 on the
    GPU, architectures/common.py:19-22) computes from the plain copy."""
    rng = np.random.default_rng(5)
    N, W, H, X = 6, 4, 84, 84
    D = H * X
    frame = T(rng.integers(0, 256, (N, D)).astype(np.uint8), dev)
    prev = T(rng.integers(0, 256, (N, W, D)).astype(np.uint8), dev)
    done = T((rng.random(N) < 0.3).astype(np.float32), dev)
    rew = torch.zeros(N, device=dev)
    fmt = torch.channels_last if cl else torch.contiguous_format
    nets = []
    for sc in (False, True):
        net = torch.empty((N, W, H, X), device=dev, memory_format=fmt)
        ops.rollout_store(frame, rew, done, prev, torch.empty_like(prev), net, scale255=sc)
        nets.append(net)
    assert torch.equal(nets[0] / 255.0, nets[1])
    r0 = torch.empty((N, W, H, X), device=dev, memory_format=fmt)
    r1 = torch.empty((N, W, H, X), device=dev, memory_format=fmt)
    ops.obs_reset(frame, torch.empty_like(prev), r0)
    ops.obs_reset(frame, torch.empty_like(prev), r1, scale255=True)
    assert torch.equal(r0 / 255.0, r1)
    if cl:
        src = prev.view(N, W, H, X)
        idx = torch.tensor([5, 0, 3, 3], device=dev)
        g0 = torch.empty((4, W, H, X), device=dev, memory_format=fmt)
        g1 = torch.empty((4, W, H, X), device=dev, memory_format=fmt)
        ops.gather_rows(src, idx, g0)
        ops.gather_rows(src, idx, g1, scale255=True)
        assert torch.equal(g0 / 255.0, g1)


@pytest.mark.parametrize("R,N", [(3276800, 32), (401408, 64), (100, 16), (7, 8), (5000, 128)])
def test_relu_bias_grad_narrow_rows_packed(ops, dev, R, N):
    """N/4 < 64 lanes per row: several rows per wave instruction (NHWC conv outputs)."""
    g = torch.randn(R, N, device=dev)
    out = torch.relu(torch.randn(R, N, device=dev))
    gp, db = ops.relu_bias_grad(g, out)
    want = torch.ops.aten.threshold_backward(g, out, 0)
    assert torch.equal(gp, want)
    ref = want.double().sum(0)
    scale = want.double().abs().sum(0).clamp_min(1e-30)
    assert ((db.double() - ref).abs() / scale).max().item() < 1e-6


@pytest.mark.parametrize("relu", [True, False])
def test_bias_act_equals_torch(ops, dev, relu):
    y = torch.randn(50000, 64, device=dev)
    b = torch.randn(64, device=dev)
    want = torch.relu(y + b) if relu else y + b
    ops.bias_act(y, b, relu)
    assert torch.equal(y, want)


@pytest.mark.parametrize("M,K1,N1,N2,ldx", [(128, 12, 256, 512, 48), (128, 6, 256, 512, 6),
                                           (7, 12, 64, 33, 12), (256, 64, 512, 1024, 64),
                                           (1, 5, 16, 7, 5)])
def test_linear2_act_vs_torch(ops, dev, M, K1, N1, N2, ldx):
    """Two Linear+ReLU layers in one launch == the two layers in f64, to f32 rounding."""
    torch.manual_seed(M + K1)
    xb = torch.randint(0, 200, (M, ldx), device=dev).float()
    x = xb[:, :K1]
    w1, b1 = torch.randn(N1, K1, device=dev) * 0.1, torch.randn(N1, device=dev) * 0.1
    w2, b2 = torch.randn(N2, N1, device=dev) * 0.05, torch.randn(N2, device=dev) * 0.1
    y = ops.linear2_act(x, w1, b1, w2, b2)
    h = torch.relu(x.double() @ w1.double().t() + b1.double())
    ref = torch.relu(h @ w2.double().t() + b2.double())
    scale = (torch.relu(x.double().abs() @ w1.double().abs().t() + b1.double().abs())
             @ w2.double().abs().t()).max().item() + 1.0
    assert (y.double() - ref).abs().max().item() <= 1e-5 * scale
    y2 = ops.linear2_act(x, w1, b1, w2, b2)
    assert torch.equal(y, y2)  # deterministic


@pytest.mark.parametrize("R,N,K", [(12288, 256, 12), (12288, 256, 6), (4096, 32, 12), (7, 4, 1),
                                   (33, 260, 16), (100000, 64, 3), (1, 16384, 5)])
@pytest.mark.parametrize("relu", [True, False])
def test_relu_bias_wgrad_vs_torch(ops, dev, R, N, K, relu):
    """First-layer backward in one pass vs autograd's threshold_backward + g'^T x + sum (f64)."""
    g = torch.randn(R, N, device=dev)
    out = torch.relu(torch.randn(R, N, device=dev)) if relu else None
    if relu:
        out[::3, ::5] = 0.0
    xs = torch.randn(R, K + 3, device=dev)
    x = xs[:, 1:K + 1]  # row stride K + 3: the kernel takes ldx
    dw, db = ops.relu_bias_wgrad(g, out, x)
    gp = (torch.ops.aten.threshold_backward(g, out, 0) if relu else g).double()
    ref_w, ref_b = gp.t() @ x.double(), gp.sum(0)
    sw = gp.abs().t() @ x.double().abs()
    assert ((dw.double() - ref_w).abs() / sw.clamp_min(1e-30)).max().item() < 1e-6
    sb = gp.abs().sum(0).clamp_min(1e-30)
    assert ((db.double() - ref_b).abs() / sb).max().item() < 1e-6
    dw2, db2 = ops.relu_bias_wgrad(g, out, x)  # deterministic; tickets re-armed
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    # deferred finish: folded into a sum_splits_db launch, or run alone: bitwise the same, and
    # the combine's own outputs unchanged
    S, n2, N2 = 4, 512 * 256, 512
    part = torch.randn(S, n2, device=dev)
    dbp = torch.randn(90, N2, device=dev)
    o_ref, b_ref = torch.empty(n2, device=dev), torch.empty(N2, device=dev)
    ops.sum_splits_db(part, o_ref, (dbp, 90), b_ref)
    for fold in (True, False):
        fin = ops.DeferredFinish(dev)
        dw3, db3 = torch.full_like(dw, float("nan")), torch.full_like(db, float("nan"))
        ops.relu_bias_wgrad(g, out, x, dw=dw3, db=db3, defer=fin)
        assert fin.pending
        if fold:
            o, b_ = torch.empty(n2, device=dev), torch.empty(N2, device=dev)
            ops.sum_splits_db(part, o, (dbp, 90), b_, finish=fin)
            assert torch.equal(o, o_ref) and torch.equal(b_, b_ref)
        else:
            fin.run()
        assert not fin.pending
        assert torch.equal(dw3, dw) and torch.equal(db3, db)


def test_relu_bias_wgrad_graph_replay_and_zero_rows(ops, dev):
    g = torch.randn(3000, 256, device=dev)
    out = torch.relu(torch.randn(3000, 256, device=dev))
    x = torch.randn(3000, 12, device=dev)
    dw, db = torch.empty(256, 12, device=dev), torch.empty(256, device=dev)
    ops.relu_bias_wgrad(g, out, x, dw, db)
    torch.cuda.synchronize()
    want_w, want_b = dw.clone(), db.clone()
    dw.zero_(); db.zero_()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        ops.relu_bias_wgrad(g, out, x, dw, db)
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(dw, want_w) and torch.equal(db, want_b)
    e = torch.empty(0, 8, device=dev)
    w0, b0 = ops.relu_bias_wgrad(e, e, torch.empty(0, 3, device=dev))
    torch.cuda.synchronize()
    assert not w0.any() and not b0.any()
    with pytest.raises(RuntimeError, match="bad sizes"):
        ops.relu_bias_wgrad(g, None, torch.randn(3000, 17, device=dev))  # K > 16


@pytest.mark.parametrize("M,H,A", [(4096, 512, 6), (8192, 512, 4), (33, 12, 7), (1, 4, 1),
                                   (5000, 64, 3)])
@pytest.mark.parametrize("relu", [True, False])
def test_heads_bwd_vs_autograd(ops, dev, M, H, A, relu):
    """Heads + producing-ReLU backward in one pass vs autograd of relu -> two Linears (f64)."""
    z = torch.randn(M, H, device=dev, dtype=torch.float64)
    z[::4, ::3] = 0.0
    hd = (torch.relu(z) if relu else z).requires_grad_(True)
    wa = torch.randn(A, H, device=dev, dtype=torch.float64, requires_grad=True)
    ba = torch.randn(A, device=dev, dtype=torch.float64, requires_grad=True)
    wc = torch.randn(1, H, device=dev, dtype=torch.float64, requires_grad=True)
    bc = torch.randn(1, device=dev, dtype=torch.float64, requires_grad=True)
    dl = torch.randn(M, A, device=dev, dtype=torch.float64)
    dv = torch.randn(M, device=dev, dtype=torch.float64)
    logits, value = hd @ wa.t() + ba, hd @ wc.t() + bc
    torch.autograd.backward([logits, value], [dl, dv.view(-1, 1)])
    gh = hd.grad * (z > 0) if relu else hd.grad
    f = torch.float32
    gp, db_h, dwa, dwc, dba, dbc = ops.heads_bwd(
        hd.detach().to(f).contiguous(), dl.to(f), dv.to(f), wa.detach().to(f), wc.detach().to(f).reshape(-1),
        relu=relu, db_h=torch.empty(H, device=dev))
    def close(got, want, scale, tol=1e-5):
        assert ((got.double() - want).abs() / scale.clamp_min(1e-30)).max().item() < tol
    h32 = hd.detach().abs()
    close(gp, gh, dl.abs() @ wa.detach().abs() + dv.abs().view(-1, 1) * wc.detach().abs())
    close(db_h, gh.sum(0), gh.abs().sum(0))
    close(dwa, wa.grad, dl.abs().t() @ h32)
    close(dwc, wc.grad, dv.abs().view(1, -1) @ h32)
    close(dba, ba.grad, dl.abs().sum(0))
    close(dbc, bc.grad, dv.abs().sum().view(1))
    again = ops.heads_bwd(hd.detach().to(f).contiguous(), dl.to(f), dv.to(f), wa.detach().to(f),
                          wc.detach().to(f).reshape(-1), relu=relu, db_h=torch.empty(H, device=dev))
    for x, y in zip((gp, db_h, dwa, dwc, dba, dbc), again):
        assert torch.equal(x, y)  # deterministic; tickets re-armed


def test_heads_function_matches_module_autograd(dev):
    """agents._Heads (with the decoder's premasked box) == plain decoder ReLU + two Linears."""
    from oc_cleanrl_amd import agents, ops as O

    torch.manual_seed(0)
    M, K, H, A = 700, 64, 128, 6
    dec, act, cri = (torch.nn.Linear(K, H).to(dev), torch.nn.Linear(H, A).to(dev),
                     torch.nn.Linear(H, 1).to(dev))
    x = torch.randn(M, K, device=dev)
    dl, dv = torch.randn(M, A, device=dev), torch.randn(M, 1, device=dev)
    h = torch.relu(dec(x))
    torch.autograd.backward([act(h), cri(h)], [dl, dv])
    want = [p.grad.clone() for p in (dec.weight, dec.bias, act.weight, act.bias, cri.weight,
                                     cri.bias)]
    params = [dec.weight, dec.bias, act.weight, act.bias, cri.weight, cri.bias]
    for p in params:  # FlatAdam-style in-place grads
        p.grad = torch.zeros_like(p)
        p._ocppo_direct_grad = True
    h2 = agents.linear_act(x, dec, True)
    assert getattr(h2, "_ocppo_box", None) is not None
    logits, value = agents._Heads.apply(h2, act.weight, act.bias, cri.weight, cri.bias,
                                        h2._ocppo_box)
    torch.autograd.backward([logits, value], [dl, dv])
    for p, w in zip(params, want):
        torch.testing.assert_close(p.grad, w, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("M,H,A", [(32, 512, 6), (300, 64, 7), (5, 8, 2)])
def test_heads_bwd_single_head(ops, dev, M, H, A):
    """No critic row (wc = dvalue = None): the DQN Q head + producing ReLU, vs autograd (f64)."""
    z = torch.randn(M, H, device=dev, dtype=torch.float64)
    hd = torch.relu(z).requires_grad_(True)
    wq = torch.randn(A, H, device=dev, dtype=torch.float64, requires_grad=True)
    bq = torch.randn(A, device=dev, dtype=torch.float64, requires_grad=True)
    g = torch.randn(M, A, device=dev, dtype=torch.float64)
    (hd @ wq.t() + bq).backward(g)
    gh = hd.grad * (z > 0)
    f = torch.float32
    gp, db_h, dw, dwc, db, dbc = ops.heads_bwd(hd.detach().to(f).contiguous(), g.to(f), None,
                                               wq.detach().to(f), None, relu=True,
                                               db_h=torch.empty(H, device=dev))
    assert dwc is None and dbc is None
    h32 = hd.detach().abs()
    for got, want, scale in ((gp, gh, g.abs() @ wq.detach().abs()), (db_h, gh.sum(0), gh.abs().sum(0)),
                             (dw, wq.grad, g.abs().t() @ h32), (db, bq.grad, g.abs().sum(0))):
        assert ((got.double() - want).abs() / scale.clamp_min(1e-30)).max().item() < 1e-5


def test_q_head_matches_module_autograd(dev):
    """agents.q_head (fused single-head backward, premasked decoder) == ReLU Linear + Linear."""
    from oc_cleanrl_amd import agents

    torch.manual_seed(1)
    M, K, H, A = 32, 48, 512, 6
    dec, qh = torch.nn.Linear(K, H).to(dev), torch.nn.Linear(H, A).to(dev)
    x, g = torch.randn(M, K, device=dev), torch.randn(M, A, device=dev)
    qh(torch.relu(dec(x))).backward(g)
    params = [dec.weight, dec.bias, qh.weight, qh.bias]
    want = [p.grad.clone() for p in params]
    for p in params:
        p.grad = torch.zeros_like(p)
        p._ocppo_direct_grad = True
    h = agents.linear_act(x, dec, True)
    q = agents.q_head(h, qh)
    assert q.grad_fn is not None and "QHead" in type(q.grad_fn).__name__
    q.backward(g)
    for p, w in zip(params, want):
        torch.testing.assert_close(p.grad, w, rtol=1e-4, atol=1e-5)


# ---------------------------------------------------------------------------------------------
# rollout fusions (PPObj frame-cache path): bit-identical to the launches they replace
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("obs_dt,vecnorm", [("bf16", True), ("f32", False), ("bf16", False)])
@pytest.mark.parametrize("N,F,N1,N2", [(128, 12, 256, 512), (37, 6, 64, 96)])
def test_store_linear2_equals_store_then_linear2(ops, dev, obs_dt, vecnorm, N, F, N1, N2):
    rng = np.random.default_rng(N + F)
    W = 4
    dt = STORE_DT[obs_dt]
    frame = T(rng.integers(0, 210, (N, F)).astype(np.float32) + (0.3 if obs_dt == "f32" else 0), dev)
    reward = T(rng.choice([-1.0, 0.0, 1.0], N).astype(np.float32), dev)
    done = T((rng.random(N) < 0.2).astype(np.float32), dev)
    prev = T(rng.integers(0, 210, (N, W, F)).astype(np.float32), dev).to(dt)
    w1 = torch.randn(N1, F, device=dev) * 0.1
    b1 = torch.randn(N1, device=dev) * 0.1
    w2 = torch.randn(N2, N1, device=dev) * 0.05
    b2 = torch.randn(N2, device=dev) * 0.1
    outs = []
    for fused in (False, True):
        out = torch.empty_like(prev)
        net = torch.empty(N, W, F, device=dev)
        rew = torch.full((N,), 7.0, device=dev)
        dn = torch.empty(N, device=dev)
        ret = torch.linspace(-1, 1, N, dtype=torch.float64, device=dev)
        rms = torch.tensor([0.1, 2.0, 50.0], dtype=torch.float64, device=dev)
        y = torch.empty(N, N2 + 8, device=dev)[:, :N2]  # row stride > N2
        vn = (ret, rms) if vecnorm else None
        if fused:
            ops.store_linear2(frame, reward, done, prev, out, net, dn, rew, w1, b1, w2, b2, y,
                              vecnorm_state=vn)
        else:
            if vecnorm:
                ops.rollout_store_vecnorm(frame, reward, done, prev, out, net, dn, ret, rms, rew)
            else:
                ops.rollout_store(frame, reward, done, prev, out, net, rew, dn)
            y.copy_(ops.linear2_act(net[:, -1], w1, b1, w2, b2))
        outs.append([out.float(), net, rew, dn, ret, rms, y])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,K,E,W", [(128, 1024, 512, 4), (50, 96, 40, 3), (128, 512, 256, 1)])
def test_linear_cache_shift_equals_linear_then_shift(ops, dev, M, K, E, W):
    x = torch.randn(M, K, device=dev)
    w = torch.randn(E, K, device=dev) * K ** -0.5
    b = torch.randn(E, device=dev)
    enc0 = torch.randn(M, W, E, device=dev)
    done = (torch.rand(M, device=dev) < 0.3).float()
    a = enc0.clone()
    fresh = ops.linear_act(x, w, b, relu=True)
    ops.frame_cache_shift(a, fresh, done)
    c = ops.linear_cache_shift(x, w, b, enc0.clone(), done)
    assert torch.equal(a, c)
    d = ops.linear_cache_shift(x, w, b, enc0.clone(), None)  # no resets: a pure shift
    assert torch.equal(d[:, :-1], enc0[:, 1:]) and torch.equal(d[:, -1], fresh)


@pytest.mark.parametrize("M,K,E,W", [(128, 1024, 512, 4), (50, 96, 64, 3), (128, 512, 32, 1)])
def test_linear_cache_ring_is_the_shift_rotated(ops, dev, M, K, E, W):
    """Ring form of the cache: after every step t, the ring rolled by t mod W equals the shifted
    cache bit for bit (resets included)."""
    w = torch.randn(E, K, device=dev) * K ** -0.5
    b = torch.randn(E, device=dev)
    enc0 = torch.randn(M, W, E, device=dev)
    shift, ring = enc0.clone(), enc0.clone()
    for t in range(1, 2 * W + 3):
        x = torch.relu(torch.randn(M, K, device=dev))
        done = (torch.rand(M, device=dev) < 0.2).float()
        ops.linear_cache_shift(x, w, b, shift, done)
        ops.linear_cache_ring(x, w, b, ring, (t - 1) % W, done)
        assert torch.equal(torch.roll(ring, -(t % W), dims=1), shift), t


@pytest.mark.parametrize("M,W,E,N", [(128, 4, 512, 512), (50, 3, 64, 40), (128, 4, 64, 64),
                                     (7, 2, 32, 16)])
def test_linear_act_ring_equals_linear_on_logical_order(ops, dev, M, W, E, N):
    x = torch.randn(M, W, E, device=dev)
    w = torch.randn(N, W * E, device=dev) * (W * E) ** -0.5
    b = torch.randn(N, device=dev)
    want = ops.linear_act(x.view(M, W * E), w, b, relu=True)
    for rot in range(W):
        phys = torch.roll(x, rot, dims=1).contiguous()  # logical s at physical (s + rot) mod W
        got = ops.linear_act(phys.view(M, W * E), w, b, relu=True, ring=(E, rot))
        assert torch.equal(got, want), rot
    with pytest.raises(RuntimeError, match="seg"):
        ops.linear_act(x.view(M, W * E), w, b, relu=True, ring=(E + 1, 0))
    with pytest.raises(RuntimeError, match="seg"):  # not a power of two
        ops.linear_act(torch.zeros(4, 192, device=dev), torch.zeros(8, 192, device=dev), None,
                       ring=(96, 1))
    with pytest.raises(RuntimeError, match="seg"):  # not a power of two
        ops.linear_act(torch.zeros(4, 96 * 2, device=dev), torch.zeros(8, 192, device=dev), None,
                       ring=(96, 1))


@pytest.mark.parametrize("B,Cin,H,W,Cout,k,s,relu", [
    (256, 4, 84, 84, 32, 8, 4, True),    # NatureCNN conv1 at the rollout batch
    (37, 32, 20, 20, 64, 4, 2, True),    # conv2, ragged batch
    (5, 64, 9, 9, 64, 3, 1, False),      # conv3, no ReLU
    (3, 4, 11, 13, 20, 4, 3, True),      # non-square input, Cout not a multiple of 16
    (0, 4, 84, 84, 32, 8, 4, True)])     # empty batch
def test_conv2d_act_vs_torch(ops, dev, B, Cin, H, W, Cout, k, s, relu):
    """NHWC implicit-GEMM conv + bias (+ ReLU) vs torch's conv2d in f64 (tolerance: f32 rounding
    of a K = k*k*Cin sum)."""
    import torch.nn.functional as F
    g = torch.Generator(device=dev).manual_seed(B + Cin + k)
    cl = torch.channels_last
    x = torch.rand(B, Cin, H, W, device=dev, generator=g).contiguous(memory_format=cl)
    w = (torch.randn(Cout, Cin, k, k, device=dev, generator=g) * (Cin * k * k) ** -0.5
         ).contiguous(memory_format=cl)
    b = torch.randn(Cout, device=dev, generator=g) * 0.1
    y = ops.conv2d_act(x, w, b, s, relu)
    assert y.shape == (B, Cout, (H - k) // s + 1, (W - k) // s + 1)
    assert y.is_contiguous(memory_format=cl)
    if B == 0:
        return
    ref = F.conv2d(x.double(), w.double(), b.double(), stride=s)
    ref = F.relu(ref) if relu else ref
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
    assert torch.equal(y, ops.conv2d_act(x, w, b, s, relu))  # deterministic
    with pytest.raises(ValueError, match="channels_last"):
        ops.conv2d_act(x.contiguous(), w, b, s, relu)


def test_rollout_conv_trunk_matches_miopen(ops, dev):
    """The NatureCNN trunk under no_grad with the HIP input convolution vs the MIOpen path."""
    from oc_cleanrl_amd import agents
    from oc_cleanrl_amd.agents import make_agent

    ag = make_agent("PPO", (4, 84, 84), 4, dev).to(dev).to(memory_format=torch.channels_last)
    x = (torch.randint(0, 256, (64, 4, 84, 84), device=dev).float() / 255).contiguous(
        memory_format=torch.channels_last)
    torch.backends.cudnn.benchmark = False
    with torch.no_grad():
        agents.HIP_ROLLOUT_CONV = False
        try:
            want = ag.trunk(x, prescaled=True)
        finally:
            agents.HIP_ROLLOUT_CONV = True
        got = ag.trunk(x, prescaled=True)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,C,H,W,relu", [(256, 64, 7, 7, True), (3, 20, 5, 9, False),
                                           (1, 1, 1, 1, True), (0, 64, 7, 7, True),
                                           (5, 96, 8, 16, True)])  # P * (C + 1) = 12416 > max
def test_bias_act_nchw(ops, dev, B, C, H, W, relu):
    """ocppo_bias_act_nchw: act(y + b) of a channels_last tensor written NCHW-contiguous, bit for
    bit torch's (y + b).relu() (one f32 add, then max)."""
    g = torch.Generator(device=dev).manual_seed(C + H)
    y = torch.randn(B, C, H, W, device=dev, generator=g).contiguous(
        memory_format=torch.channels_last)
    b = torch.randn(C, device=dev, generator=g)
    if H * W * (C + 1) > 12288:
        with pytest.raises(RuntimeError, match="bad sizes"):
            ops.bias_act_nchw(y, b, relu)
        return
    out = ops.bias_act_nchw(y, b, relu)
    assert out.is_contiguous() and out.shape == y.shape
    want = y + b.view(1, C, 1, 1)
    want = want.relu() if relu else want
    assert torch.equal(out, want.contiguous())


def test_rollout_trunk_nchw_flatten_matches_module(ops, dev):
    """The NatureCNN trunk under no_grad (the last conv's bias/ReLU pass writing NCHW for the
    Flatten) == the module's own forward; the path is taken."""
    from oc_cleanrl_amd import agents
    from oc_cleanrl_amd.agents import make_agent

    ag = make_agent("PPO", (4, 84, 84), 4, dev).to(dev).to(memory_format=torch.channels_last)
    x = (torch.randint(0, 256, (32, 4, 84, 84), device=dev).float() / 255).contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        feat = ag.network[1:5](x)
        assert agents._conv_nchw_out_ok(feat, ag.network[5], list(ag.network)[6:8])
        got = ag.trunk(x, prescaled=True)
        agents.CONV_NCHW_OUT = False
        try:
            want = ag.trunk(x, prescaled=True)
        finally:
            agents.CONV_NCHW_OUT = True
        ref = ag.network[1:](x)
    assert torch.equal(got, want)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------------------------------------
# policy heads forward + fused PPO loss + heads backward in one pass (ocppo_heads_loss_fwd_bwd)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("M,H,A", [(4096, 512, 6), (1000, 256, 4), (77, 64, 7), (300, 128, 3),
                                   (20000, 512, 6), (70001, 128, 6)])
@pytest.mark.parametrize("norm_adv,clip_vloss", [(True, True), (False, False)])
def test_heads_loss_equals_heads_then_loss_then_heads_bwd(ops, dev, M, H, A, norm_adv, clip_vloss):
    g = torch.Generator(device=dev).manual_seed(M + H)
    h = torch.relu(torch.randn(M, H, device=dev, generator=g))
    h[::7, ::3] = 0.0
    wa = torch.randn(A, H, device=dev, generator=g) * 0.05
    ba = torch.randn(A, device=dev, generator=g) * 0.1
    wc = torch.randn(1, H, device=dev, generator=g) * 0.05
    bc = torch.randn(1, device=dev, generator=g)
    logits = torch.addmm(ba, h, wa.t())
    value = torch.addmm(bc, h, wc.t()).view(-1)
    acts = torch.randint(0, A, (M,), device=dev, generator=g)
    with torch.no_grad():
        lp_now = torch.log_softmax(logits, -1).gather(1, acts.view(-1, 1)).view(-1)
    old_lp = lp_now + 0.2 * torch.randn(M, device=dev, generator=g)
    old_lp[: M // 5] = lp_now[: M // 5]  # ratio 1: max() ties
    adv = 2.0 * torch.randn(M, device=dev, generator=g)
    ret = value + torch.randn(M, device=dev, generator=g)
    val = value + 0.3 * torch.randn(M, device=dev, generator=g)
    st = ops.minibatch_adv_stats(adv, torch.arange(M, device=dev), M)[0]
    cfg = dict(clip_coef=0.1, ent_coef=0.01, vf_coef=0.5, norm_adv=norm_adv, clip_vloss=clip_vloss)
    s_ref, dl_ref, dv_ref = ops.ppo_loss_fwd_bwd(logits, value, acts, old_lp, adv, ret, val,
                                                 adv_stats=st if norm_adv else None, **cfg)
    gp_ref, dbh_ref, dwa_ref, dwc_ref, dba_ref, dbc_ref = ops.heads_bwd(
        h, dl_ref, dv_ref, wa, wc.reshape(-1), relu=True, db_h=torch.empty(H, device=dev))
    dl, dv = torch.empty(M, A, device=dev), torch.empty(M, device=dev)
    gp, dbh, dwa, dwc, dba, dbc, stats = ops.heads_loss_fwd_bwd(
        h, wa, ba, wc, bc, acts, old_lp, adv, ret, val, adv_stats=st if norm_adv else None,
        db_h=torch.empty(H, device=dev), dlogits=dl, dvalue=dv, **cfg)
    # the head dot products run in another order than the GEMM: f32 rounding differences only
    torch.testing.assert_close(stats, s_ref, rtol=2e-5, atol=1e-7)
    scale = lambda t: float(t.abs().max()) + 1e-30  # noqa: E731
    for got, ref in ((dl, dl_ref), (dv, dv_ref), (gp, gp_ref), (dbh, dbh_ref), (dwa, dwa_ref),
                     (dwc.view(-1), dwc_ref.view(-1)), (dba, dba_ref), (dbc, dbc_ref)):
        assert float((got - ref).abs().max()) <= 2e-5 * scale(ref), (got, ref)
    again = ops.heads_loss_fwd_bwd(h, wa, ba, wc, bc, acts, old_lp, adv, ret, val,
                                   adv_stats=st if norm_adv else None,
                                   db_h=torch.empty(H, device=dev), **cfg)
    for x, y in zip((gp, dbh, dwa, dwc, dba, dbc, stats), again):
        assert torch.equal(x, y)  # deterministic
    # deferred finish: the rows launch alone, then the finish folded into a split-K combine
    # (ocppo_sum_splits_finish) or run alone (ocppo_deferred_finish_run): bitwise the same
    part = torch.randn(8, 512, 2048, device=dev, generator=g)
    for fold in (True, False):
        fin = ops.DeferredFinish(dev)
        outs = [torch.full_like(t, float("nan")) for t in (gp, dbh, dwa, dwc, dba, dbc, stats)]
        ops.heads_loss_fwd_bwd(h, wa, ba, wc, bc, acts, old_lp, adv, ret, val,
                               adv_stats=st if norm_adv else None, gp=outs[0], db_h=outs[1],
                               dwa=outs[2], dwc=outs[3], dba=outs[4], dbc=outs[5], stats=outs[6],
                               defer=fin, **cfg)
        assert fin.pending and torch.equal(outs[0], gp)
        if fold:
            comb = ops.sum_splits(part, finish=fin)
            assert torch.equal(comb, ops.sum_splits(part))  # the combine itself unchanged
        else:
            fin.run()
        assert not fin.pending
        for x, y in zip((gp, dbh, dwa, dwc, dba, dbc, stats), outs):
            assert torch.equal(x, y)


@pytest.mark.parametrize("H", [192, 320, 384, 448, 576])
def test_heads_loss_rejects_uninstantiated_widths(ops, dev, H):
    """Only H / 64 in {1, 2, 4, 8} has a rows kernel: other widths are refused by every gate
    (the C entry point, ops.heads_loss_ok and the trainer's fused_heads_loss) instead of running
    the 8-column instance past the end of each row."""
    from oc_cleanrl_amd._lib import OcppoError

    M, A = 64, 6
    h = torch.relu(torch.randn(M, H, device=dev))
    assert not ops.heads_loss_ok(h, A)
    wa, ba = torch.zeros(A, H, device=dev), torch.zeros(A, device=dev)
    wc, bc = torch.zeros(1, H, device=dev), torch.zeros(1, device=dev)
    acts = torch.zeros(M, dtype=torch.int64, device=dev)
    z = torch.zeros(M, device=dev)
    with pytest.raises(OcppoError, match="bad sizes"):
        ops.heads_loss_fwd_bwd(h, wa, ba, wc, bc, acts, z, z, z, z, adv_stats=None,
                               clip_coef=0.1, ent_coef=0.01, vf_coef=0.5, norm_adv=False,
                               clip_vloss=True)
    from test_trainer_gpu import small_args
    from oc_cleanrl_amd.trainer import PPOTrainer

    tr = PPOTrainer(small_args(decoder_dims=(H,)), dev)
    assert not tr.fused_heads_loss


@pytest.mark.parametrize("T_,N", [(7, 5), (128, 128), (200, 130), (33, 1030), (128, 4096),
                                  (16, 65540)])
def test_gae_records_are_the_arrays(ops, dev, T_, N):
    """ocppo_gae_records: advantages / returns bitwise those of ocppo_gae (every tile width and
    the streaming form), and each sample's 16-B record holds exactly its log-prob, advantage,
    value and action (advantage + value is its return, bitwise)."""
    g = torch.Generator(device=dev).manual_seed(T_ * 31 + N)
    r = torch.randn(T_, N, device=dev, generator=g)
    v = torch.randn(T_, N, device=dev, generator=g)
    d = (torch.rand(T_, N, device=dev, generator=g) < 0.1).float()
    nv, nd = torch.randn(N, device=dev, generator=g), torch.zeros(N, device=dev)
    lp = torch.randn(T_, N, device=dev, generator=g)
    act = torch.randint(0, 1 << 31, (T_, N), device=dev, generator=g)
    a0, r0 = ops.gae(r, v, d, nv, nd, 0.99, 0.95)
    rec = ops.sample_records(T_ * N, dev)
    a1, r1 = ops.gae(r, v, d, nv, nd, 0.99, 0.95, logprobs=lp, actions=act, records=rec)
    torch.cuda.synchronize()
    assert torch.equal(a0, a1) and torch.equal(r0, r1)
    f = rec.view(torch.float32).view(T_ * N, 4)
    assert torch.equal(f[:, 0], lp.view(-1)) and torch.equal(f[:, 1], a1.view(-1))
    assert torch.equal(f[:, 2], v.view(-1)) and torch.equal(rec[:, 3].long(), act.view(-1))
    assert torch.equal(f[:, 1] + f[:, 2], r1.view(-1))


@pytest.mark.parametrize("M,nmb,B", [(4096, 16, 16384), (100, 7, 700), (16384, 4, 65536),
                                     (16384, 64, 1 << 20), (1000, 1049, 1 << 20)])
def test_minibatch_prepare_from_records_is_bitwise_the_soa_form(ops, dev, M, nmb, B):
    """The 16-B record form (at >= 2^20 samples its statistics taken by a second launch from the
    gathered advantages) is bitwise the SoA form, statistics included."""
    g = torch.Generator(device=dev).manual_seed(M + nmb)
    T_ = 4 if B % 4 == 0 else 1
    acts = torch.randint(0, 6, (B,), device=dev, generator=g)
    lp, bv = torch.randn(B, device=dev, generator=g), torch.randn(B, device=dev, generator=g)
    adv, ret = torch.empty(B, device=dev), torch.empty(B, device=dev)
    z = torch.zeros(B // T_, device=dev)
    rec = ops.sample_records(B, dev)
    ops.gae(torch.randn(T_, B // T_, device=dev, generator=g), bv.view(T_, -1),
            torch.zeros(T_, B // T_, device=dev), z, z, 0.99, 0.95, adv.view(T_, -1),
            ret.view(T_, -1), logprobs=lp.view(T_, -1), actions=acts.view(T_, -1), records=rec)
    reps = (nmb * M + B - 1) // B
    perm = torch.cat([torch.randperm(B, device=dev, generator=g) for _ in range(reps)])[:nmb * M]
    a = ops.minibatch_prepare(perm, M, acts, lp, adv, ret, bv)
    b = ops.minibatch_prepare(perm, M, acts, lp, adv, ret, bv, records=rec)
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k
