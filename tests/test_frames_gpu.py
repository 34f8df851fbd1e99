"""Frame-deduplicated PPObj minibatch kernels (ocppo_frames_gather / _expand / _scatter) on the
GPU through the C-ABI, against the oracle's restatement (bit-exact), plus the trainer's dedup
update against the plain per-slot update (ppo_atari_oc.py:566-605 through PPObj)."""
import numpy as np
import pytest
import torch

from oc_cleanrl_amd import ops
from oc_cleanrl_amd.frames import FramePlanner
from oracle import ocppo_oracle as O
from test_frames_cpu import _rollout

pytestmark = pytest.mark.gpu


def _setup(T, N, W, F, M, E, nmb, p_done, seed, dev, dtype=torch.bfloat16):
    rng = np.random.default_rng(seed)
    obs, dones = _rollout(T, N, W, F, p_done, rng, (rng.random(N) < 0.3).astype(np.float32))
    pl = FramePlanner(T, N, W, M, E, nmb)
    perm = np.concatenate([rng.permutation(T * N) for _ in range(E)]).astype(np.int64)
    used, inv = pl.plan(perm)
    cap = pl.cap_for(pl.counts)
    buf = np.zeros(pl.size(cap), np.int32)
    pl.fill(buf, cap, used, inv)
    d_buf = torch.from_numpy(buf).to(dev)
    return dict(obs=obs, dones=dones, perm=perm, plan=pl.views(buf, cap), pl=pl, cap=cap,
                d_obs=torch.from_numpy(obs).to(dev).to(dtype), d_dones=torch.from_numpy(dones).to(dev),
                d_perm=torch.from_numpy(perm).to(dev), d_plan=pl.views(d_buf, cap))


@pytest.mark.parametrize("T,N,W,F,M,E,nmb,p_done", [
    (16, 8, 4, 12, 32, 2, 4, 0.2),     # resets in every window
    (9, 5, 3, 6, 15, 1, 3, 0.5),       # ragged sizes, odd W / F
    (24, 7, 4, 12, 42, 1, 4, 0.0),     # no resets
    (12, 4, 1, 12, 12, 2, 4, 0.3),     # W = 1
    (10, 3, 16, 5, 10, 1, 3, 0.1),     # W = 16 (the kernels' maximum)
])
def test_frames_kernels_match_oracle(dev, T, N, W, F, M, E, nmb, p_done):
    s = _setup(T, N, W, F, M, E, nmb, p_done, 11, dev)
    uniq, pos_of, inv = s["plan"]
    du, dp, di = s["d_plan"]
    Ed = 20
    rng = np.random.default_rng(5)
    for j in range(E * nmb):
        e, k = divmod(j, nmb)
        x = ops.frames_gather(s["d_obs"], du[j])
        assert np.array_equal(x.cpu().numpy(), O.frames_gather(s["obs"], uniq[j]))
        enc = rng.standard_normal((s["cap"], Ed)).astype(np.float32)
        mb = s["perm"][j * M:(j + 1) * M]
        h = ops.frames_expand(torch.from_numpy(enc).to(dev), dp[j], s["d_perm"][j * M:(j + 1) * M],
                              s["d_dones"], T, N, W)
        assert np.array_equal(h.cpu().numpy(), O.frames_expand(enc, pos_of[j], mb, s["dones"], N, W))
        dh = rng.standard_normal((M, W, Ed)).astype(np.float32)
        denc = ops.frames_scatter(torch.from_numpy(dh).to(dev), du[j], di[e], k, s["d_dones"], T, N, W)
        want = O.frames_scatter(dh, uniq[j], inv[e], k, s["dones"], T, N, W)
        assert np.array_equal(denc.cpu().numpy(), want)  # same summation order: bit-exact


@pytest.mark.parametrize("T,N,W,M,E,nmb,p_done,Ed", [
    (16, 8, 4, 32, 2, 4, 0.2, 20),      # resets in every window
    (9, 5, 3, 15, 1, 3, 0.5, 8),        # ragged sizes, odd W
    (24, 7, 4, 42, 1, 4, 0.0, 64),      # no resets
    (10, 3, 16, 10, 1, 3, 0.1, 12),     # W = 16 (the kernels' maximum)
    (12, 6, 4, 24, 1, 4, 0.1, 516),     # E not a multiple of 512: a partial column pass
    (12, 6, 4, 24, 1, 4, 0.1, 544),     # ... and a multiple of 32 (the bitmask form)
])
def test_frames_scatter_relu_is_scatter_then_relu_backward(dev, T, N, W, M, E, nmb, p_done, Ed):
    """ocppo_frames_scatter_relu: gp = out <= 0 ? 0 : frames_scatter(...) bit for bit (same
    per-frame summation order as the oracle), the bias-gradient chunk partials summing to the
    column sums of gp, and out = None the plain scatter."""
    s = _setup(T, N, W, 12, M, E, nmb, p_done, 13, dev)
    uniq, pos_of, inv = s["plan"]
    du, dp, di = s["d_plan"]
    rng = np.random.default_rng(6)
    for j in range(E * nmb):
        e, k = divmod(j, nmb)
        dh = rng.standard_normal((M, W, Ed)).astype(np.float32)
        out = np.maximum(rng.standard_normal((s["cap"], Ed)), 0).astype(np.float32)
        want = O.frames_scatter(dh, uniq[j], inv[e], k, s["dones"], T, N, W)
        want = np.where(out <= 0, 0, want).astype(np.float32)
        gp, (part, chunks) = ops.frames_scatter_relu(torch.from_numpy(dh).to(dev), du[j], di[e], k,
                                                     s["d_dones"], T, N, W,
                                                     out=torch.from_numpy(out).to(dev))
        assert np.array_equal(gp.cpu().numpy(), want)
        assert chunks == -(-s["cap"] // 16)
        torch.testing.assert_close(part.sum(0).double(), gp.double().sum(0), rtol=1e-5, atol=1e-5)
        part = part.clone()  # the partials buffer is per shape: the next call rewrites it
        if Ed % 32 == 0:  # the same mask as the row-major ReLU bitmask of out: the same gp
            on = (out > 0).astype(np.uint64).reshape(s["cap"], -1, 32)
            words = (on << np.arange(32, dtype=np.uint64)).sum(-1).astype(np.uint32)
            gpb, (partb, _) = ops.frames_scatter_relu(
                torch.from_numpy(dh).to(dev), du[j], di[e], k, s["d_dones"], T, N, W,
                mbits=torch.from_numpy(words.view(np.int32)).to(dev))
            assert np.array_equal(gpb.cpu().numpy(), want)
            assert torch.equal(partb, part)
        plain, none = ops.frames_scatter_relu(torch.from_numpy(dh).to(dev), du[j], di[e], k,
                                              s["d_dones"], T, N, W, with_db=False)
        assert none is None
        assert np.array_equal(plain.cpu().numpy(), O.frames_scatter(dh, uniq[j], inv[e], k,
                                                                     s["dones"], T, N, W))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.uint8])
@pytest.mark.parametrize("T,N,W,F,N1,p_done,bias,relu", [
    (16, 8, 4, 12, 256, 0.2, True, True),    # PPObj's first encoder layer shape
    (9, 5, 3, 6, 20, 0.5, False, True),      # ragged sizes, no bias
    (10, 3, 16, 16, 1024, 0.1, True, False),  # F = 16, N1 = 1024 (the maxima), identity
    (12, 4, 4, 3, 100, 0.2, True, True),     # N1 not a multiple of the 64-column block
])
def test_frames_gather_linear_is_gather_then_linear(dev, dtype, T, N, W, F, N1, p_done, bias,
                                                    relu):
    """ocppo_frames_gather_linear: x is frames_gather bit for bit (the oracle), and h = act(x W^T
    + b) to f32 rounding of an f64 product (padding rows -1 give x = 0, h = act(b))."""
    s = _setup(T, N, W, F, 2 * N, 1, max(T // 2, 1), p_done, 21, dev, dtype)
    uniq, _, _ = s["plan"]
    du, _, _ = s["d_plan"]
    g = torch.Generator(device=dev).manual_seed(1)
    w = torch.randn((N1, F), device=dev, generator=g) * F ** -0.5
    b = torch.randn(N1, device=dev, generator=g) if bias else None
    for j in range(du.shape[0]):
        x, h = ops.frames_gather_linear(s["d_obs"], du[j], w, b, relu=relu)
        want_x = O.frames_gather(s["obs"], uniq[j])
        if dtype != torch.float32:  # the device obs are stored rounded
            want_x = ops.frames_gather(s["d_obs"], du[j]).cpu().numpy()
        assert np.array_equal(x.cpu().numpy(), want_x)
        ref = x.double() @ w.double().t() + (b.double() if bias else 0)
        ref = ref.clamp_min(0) if relu else ref
        # f32 fma chain over F terms + bias: |err| <= (F + 1) u sum |x_f w_f| + |b| (u = 2^-24)
        scale = x.double().abs() @ w.double().abs().t() + (b.double().abs() if bias else 0)
        assert bool(((h.double() - ref).abs() <= (F + 2) * 2.0 ** -24 * scale + 1e-30).all())


@pytest.mark.parametrize("N1", [256, 512])  # the wide form (row table in the same launch), narrow
def test_frames_gather_linear_makes_the_row_table_too(dev, N1):
    """ocppo_frames_gather_linear with idx_out: x and h bitwise the plain call's, and the row table
    bitwise ocppo_frames_expand_index's (extra workgroups of the same launch, or a second launch
    after the narrow form); an empty frame set still writes the table."""
    T, N, W, F, M, E, nmb = 32, 64, 4, 12, 512, 2, 4
    s = _setup(T, N, W, F, M, E, nmb, 1 / 20, 9, dev, torch.bfloat16)
    du, dp, di = s["d_plan"]
    g = torch.Generator(device=dev).manual_seed(3)
    w = torch.randn((N1, F), device=dev, generator=g) * F ** -0.5
    b = torch.randn(N1, device=dev, generator=g)
    for j in (0, 5):
        perm = s["d_perm"][j * M:(j + 1) * M]
        x0, h0 = ops.frames_gather_linear(s["d_obs"], du[j], w, b, relu=True)
        x1, h1, idx = ops.frames_gather_linear(s["d_obs"], du[j], w, b, relu=True,
                                               index=(dp[j], perm, s["d_dones"]))
        assert torch.equal(x0, x1) and torch.equal(h0, h1)
        assert torch.equal(idx, ops.frames_expand_index(dp[j], perm, s["d_dones"], T, N, W))
    empty = du[0][:0]
    _, _, idx = ops.frames_gather_linear(s["d_obs"], empty, w, b, relu=True,
                                         index=(dp[0], s["d_perm"][:M], s["d_dones"]))
    assert torch.equal(idx, ops.frames_expand_index(dp[0], s["d_perm"][:M], s["d_dones"], T, N, W))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.uint8])
def test_frames_at_config_size_reproduce_the_minibatch(dev, dtype):
    """Config 2 sizes (T=128, N=128, W=4, F=12, 4 x 4 minibatches of 4096): the deduplicated
    frames, expanded, ARE b_obs[mb_inds] bit for bit; scatter is expand's adjoint."""
    T, N, W, F, M, E, nmb = 128, 128, 4, 12, 4096, 4, 4
    s = _setup(T, N, W, F, M, E, nmb, 1 / 50, 3, dev, dtype)
    du, dp, di = s["d_plan"]
    b_obs = s["d_obs"][:T].reshape(T * N, W, F).float()
    g = torch.Generator(device=dev).manual_seed(0)
    for j in range(E * nmb):
        e, k = divmod(j, nmb)
        idx = s["d_perm"][j * M:(j + 1) * M]
        x = ops.frames_gather(s["d_obs"], du[j])
        h = ops.frames_expand(x, dp[j], idx, s["d_dones"], T, N, W)
        assert torch.equal(h, b_obs[idx])
        enc = torch.randn((s["cap"], 16), device=dev, generator=g, dtype=torch.float64).float()
        dh = torch.randn((M, W, 16), device=dev, generator=g, dtype=torch.float64).float()
        he = ops.frames_expand(enc, dp[j], idx, s["d_dones"], T, N, W)
        denc = ops.frames_scatter(dh, du[j], di[e], k, s["d_dones"], T, N, W)
        lhs = torch.dot(he.double().ravel(), dh.double().ravel())
        rhs = torch.dot(enc.double().ravel(), denc.double().ravel())
        torch.testing.assert_close(lhs, rhs, rtol=1e-5, atol=1e-3)
        assert torch.all(denc[int(s["pl"].counts[j]):] == 0)


def test_trainer_dedup_update_matches_per_slot_update(dev):
    """One minibatch's loss and gradients with the dedup encoder == the per-slot encoder (the
    reference's b_obs[mb_inds] forward) up to f32 summation order."""
    from oc_cleanrl_amd.args import Args, finalize
    from oc_cleanrl_amd.trainer import PPOTrainer

    args = finalize(Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ",
                         num_envs=64, num_steps=32, num_minibatches=4, update_epochs=2,
                         total_timesteps=64 * 32 * 10, encoder_dims=(64, 128), decoder_dims=(128,),
                         save_model=False, cuda_graphs=False), 1)
    tr = PPOTrainer(args, dev)
    assert tr.frame_dedup
    tr.train_iteration()
    tr._load_staged()
    with torch.no_grad():
        tr._rollout()
    for j in (0, 5):
        tr.frame_dedup = True
        tr._forward_backward(j)
        g1, st1 = tr.grad_buf.clone(), tr.stats[j].clone()
        tr.frame_dedup = False
        tr._forward_backward(j)
        g2, st2 = tr.grad_buf.clone(), tr.stats[j].clone()
        torch.testing.assert_close(st1, st2, rtol=1e-5, atol=1e-6)
        scale = g2.abs().max()
        torch.testing.assert_close(g1, g2, rtol=0, atol=2e-5 * float(scale))
        assert not torch.equal(g1, torch.zeros_like(g1))


def test_gathered_decoder_gemms_equal_the_materialised_ones(dev):
    """ocppo_frames_expand_index + ocppo_gemm_x6_gather at config 2 sizes: idx rows ARE
    frames_expand's sources; the gathered forward (mode 1, one split per stack slot) and weight
    gradient (mode 2) are bitwise the same gemm_x6 products on the materialised [M, W * E] input."""
    T, N, W, F, M, E, nmb = 128, 128, 4, 12, 4096, 4, 4
    Ed, H = 512, 512
    s = _setup(T, N, W, F, M, E, nmb, 1 / 50, 7, dev)
    du, dp, di = s["d_plan"]
    g = torch.Generator(device=dev).manual_seed(2)
    enc = torch.relu(torch.randn((s["cap"], Ed), device=dev, generator=g))
    w = torch.randn((H, W * Ed), device=dev, generator=g) * (W * Ed) ** -0.5
    b = torch.randn(H, device=dev, generator=g) * 0.1
    gp = torch.randn((M, H), device=dev, generator=g)
    for j in (0, 9):
        perm = s["d_perm"][j * M:(j + 1) * M]
        idx = ops.frames_expand_index(dp[j], perm, s["d_dones"], T, N, W)
        x = ops.frames_expand(enc, dp[j], perm, s["d_dones"], T, N, W).view(M, W * Ed)
        assert torch.equal(enc[idx.long()].view(M, W * Ed), x)
        for planes in (False, True):
            pl = None
            if planes:
                ops.WeightPlanes(fwd=[w]).refresh()
                pl = w._ocppo_planes["fwd"]
            got = ops.linear_x6_split(enc, w, b, True, W, planes=pl, gather=(idx, Ed))
            want = ops.linear_x6_split(x, w, b, True, W, planes=pl)
            assert torch.equal(got, want)
        for S in (8, 4):
            pg = ops.dw_x6_parts_gather(gp, enc, idx, S)
            pw = ops.dw_x6_parts(gp, x, S, tile=ops.X6_AUTO)
            assert torch.equal(pg, pw)
