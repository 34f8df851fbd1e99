"""ocppo_gemm_x6: the update's f32 GEMMs as six bf16 piece products (include/ocppo.h).

Accuracy is checked against an f64 product, scaled by (|A| |B|)[m, n] — the bound an f32 dot
product's rounding obeys — next to hipBLASLt's own f32 GEMM on the same operands: the x6 product
must stay at f32 accuracy (the reference's Linear layers, ppo_atari_oc.py:566-606, are f32 with
TF32 off)."""
import pytest
import numpy as np
import torch

from oc_cleanrl_amd import ops

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


def _rand(*shape, gen, scale=1.0):
    return (torch.rand(*shape, device=DEV, generator=gen) * 2 - 1) * scale


def _rel(c, ref, scale):
    d = (c.double() - ref).abs() / scale.clamp_min(1e-300)
    return float(d.max()), float(d.mean())


def _check(c, ref, scale, torch_c):
    mx, mean = _rel(c, ref, scale)
    tmx, tmean = _rel(torch_c, ref, scale)
    # f32 level: a few units of 2^-24 relative to sum |a b|, and no worse on average than the
    # f32 library GEMM (tolerance for its different summation order)
    assert mx <= 4e-7, (mx, tmx)
    assert mean <= 2.0 * tmean + 1e-9, (mean, tmean)


@pytest.mark.parametrize("tile", ops.X6_BUILT)
@pytest.mark.parametrize("M,N,K", [(256, 256, 96), (128, 384, 320), (384, 128, 1024)])
def test_forward_bias_relu(tile, M, N, K):
    if ops.x6_tile(M, N, 1, tile) is None:
        pytest.skip("tile does not divide")
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    x = _rand(M, K, gen=g)
    w = _rand(N, K, gen=g, scale=K ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    pre64 = x.double() @ w.double().t() + b.double()
    scale = x.double().abs() @ w.double().abs().t() + b.double().abs()
    out = torch.empty(M, N, device=DEV)
    ops.gemm_x6(x, K, 1, w, K, 1, out, N, M, N, K, bias=b, relu=True, tile=tile)
    torch_c = torch._addmm_activation(b, x, w.t())
    _check(out, pre64.clamp_min(0), scale, torch_c)
    # ReLU exactly where the f64 pre-activation is clearly negative
    assert bool(((pre64 < -1e-5 * scale) <= (out == 0)).all())


@pytest.mark.parametrize("tile", [0, 3, 16, 24, 28, 30, 31])
def test_dx_and_linear_helpers(tile):
    g = torch.Generator(device=DEV).manual_seed(11)
    M, N, K = 512, 256, 384  # dX [M, K] = g [M, N] W [N, K]
    gg = _rand(M, N, gen=g)
    w = _rand(N, K, gen=g, scale=N ** -0.5)
    ref = gg.double() @ w.double()
    scale = gg.double().abs() @ w.double().abs()
    out = torch.empty(M, K, device=DEV)
    ops.gemm_x6(gg, N, 1, w, 1, K, out, K, M, K, N, tile=tile)
    _check(out, ref, scale, gg @ w)
    assert ops.dx_x6_ok(gg, w)
    _check(ops.dx_x6(gg, w), ref, scale, gg @ w)
    x = _rand(M, K, gen=g)
    assert ops.linear_x6_ok(x, w)
    y = ops.linear_x6(x, w)
    _check(y, x.double() @ w.double().t(), x.double().abs() @ w.double().abs().t(), x @ w.t())


@pytest.mark.parametrize("tile", [None, 0, 24, 28])
@pytest.mark.parametrize("splits", [1, 4, 8, 5])
def test_weight_grad_splits(splits, tile):
    g = torch.Generator(device=DEV).manual_seed(splits)
    R, N, K = 2048, 256, 128  # dW [N, K] = g [R, N]^T x [R, K]; 64 steps of 32 rows
    gg = _rand(R, N, gen=g)
    x = _rand(R, K, gen=g)
    assert ops.dw_x6_ok(gg, x, splits)
    if tile is None:
        part = ops.dw_x6_parts(gg, x, splits)
    else:
        part = torch.empty(splits, N, K, device=DEV)
        ops.gemm_x6(gg, 1, N, x, 1, K, part, K, N, K, R, splits=splits, split_c=N * K, tile=tile)
    nk = R // 32
    for s in range(splits):
        r0, r1 = 32 * (s * nk // splits), 32 * ((s + 1) * nk // splits)
        ref = gg[r0:r1].double().t() @ x[r0:r1].double()
        scale = gg[r0:r1].double().abs().t() @ x[r0:r1].double().abs()
        _check(part[s], ref, scale, gg[r0:r1].t() @ x[r0:r1])


def test_deterministic_and_exact_on_bf16_operands():
    # operands that are already bf16 values: the split is (x, 0, 0) and every product is exact,
    # so the result is an exact sum of exact products when the sums fit in f32 (small integers)
    g = torch.Generator(device=DEV).manual_seed(5)
    M, N, K = 256, 128, 512
    x = torch.randint(-8, 9, (M, K), device=DEV, generator=g).float()
    w = torch.randint(-8, 9, (N, K), device=DEV, generator=g).float()
    out1 = ops.linear_x6(x, w)
    out2 = ops.linear_x6(x, w)
    assert torch.equal(out1, out2)
    assert torch.equal(out1, (x.double() @ w.double().t()).float())


def test_rejects_bad_shapes():
    x = torch.zeros(128, 48, device=DEV)
    w = torch.zeros(128, 48, device=DEV)
    assert not ops.linear_x6_ok(x, w)  # K % 32 != 0
    out = torch.empty(128, 128, device=DEV)
    with pytest.raises(ops._lib.OcppoError):
        ops.gemm_x6(x, 48, 1, w, 48, 1, out, 128, 128, 128, 48, tile=0)
    x2 = torch.zeros(96, 64, device=DEV)
    assert ops.x6_tile(96, 128) is None
    assert not ops.linear_x6_ok(x2, torch.zeros(128, 64, device=DEV))


@pytest.mark.parametrize("tile", [0, 3, 16, 24, 28, 30])
def test_dx_mask_epilogue(tile):
    # the dX product of the layer above a Linear+ReLU with that ReLU's backward fused in:
    # gp = threshold_backward(g W, out, 0) and the per-row-tile column sums of gp (bias grad)
    g = torch.Generator(device=DEV).manual_seed(21)
    M, N, K = 512, 256, 384
    gg = _rand(M, N, gen=g)
    w = _rand(N, K, gen=g, scale=N ** -0.5)
    out = torch.relu(_rand(M, K, gen=g))  # the layer-below's ReLU output (mask)
    bm = ops.X6_TILES[tile][0]
    gp = torch.empty(M, K, device=DEV)
    dbp = torch.empty(M // bm, K, device=DEV)
    ops.gemm_x6(gg, N, 1, w, 1, K, gp, K, M, K, N, mask=out, dbp=dbp, tile=tile)
    ref = torch.where(out > 0, gg.double() @ w.double(), torch.zeros((), dtype=torch.float64, device=DEV))
    scale = gg.double().abs() @ w.double().abs()
    _check(gp, ref, scale, torch.ops.aten.threshold_backward(gg @ w, out, 0))
    assert bool((gp[out <= 0] == 0).all())
    # each partial is the sum of gp over its row tile (fixed order: close to an f64 sum)
    ps = gp.double().view(M // bm, bm, K).sum(1)
    assert torch.allclose(dbp.double(), ps, rtol=1e-5, atol=1e-5)
    gp2, dbp2 = ops.dx_x6_relu(gg, w, out)
    assert torch.equal(gp2, gp if ops.x6_tile(M, K) == tile else gp2)


@pytest.mark.parametrize("tile", [24, 25, 0])
def test_relu_bitmask_roundtrip(tile):
    # forward with ReLU writes the fragment-order bitmask; the dX mask epilogue over the same
    # [M, N] with the same tile reads it: identical to the f32-mask epilogue
    g = torch.Generator(device=DEV).manual_seed(33)
    M, K0, N, N2 = 512, 256, 256, 128  # layer L: x [M, K0] -> h [M, N]; layer L+1: N -> N2
    x = _rand(M, K0, gen=g)
    w = _rand(N, K0, gen=g, scale=K0 ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    h = torch.empty(M, N, device=DEV)
    bits = torch.empty(ops.x6_mbits_words(M, N, tile), dtype=torch.int64, device=DEV)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h, N, M, N, K0, bias=b, relu=True, tile=tile, mbits_out=bits)
    h_ref = torch.empty_like(h)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h_ref, N, M, N, K0, bias=b, relu=True, tile=tile)
    assert torch.equal(h, h_ref)
    gg = _rand(M, N2, gen=g)
    w2 = _rand(N2, N, gen=g, scale=N2 ** -0.5)
    bm = ops.X6_TILES[tile][0]
    gp_f, dbp_f = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    gp_b, dbp_b = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_f, N, M, N, N2, mask=h, dbp=dbp_f, tile=tile)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_b, N, M, N, N2, dbp=dbp_b, tile=tile, mbits_in=bits)
    assert torch.equal(gp_f, gp_b) and torch.equal(dbp_f, dbp_b)
    assert bool((gp_b[h <= 0] == 0).all())
    # the helpers: linear_x6(mbits=True) -> dx_x6_relu(mbits=...)
    y, mb = ops.linear_x6(x, w, b, relu=True, mbits=True)
    assert torch.equal(y, h_ref if mb[1] == tile else y)
    gp2, _ = ops.dx_x6_relu(gg, w2, y, mbits=mb)
    gp3, _ = ops.dx_x6_relu(gg, w2, y)
    assert torch.equal(gp2, gp3)


def _rows_bits_ref(h):
    """The row-major ReLU bitmask of h [M, N] (bit n % 32 of int32 word [m, n // 32] =
    !(h <= 0)), built on the host."""
    on = (~(h <= 0)).cpu().numpy().astype(np.uint64).reshape(h.shape[0], -1, 32)
    words = (on << np.arange(32, dtype=np.uint64)).sum(-1).astype(np.uint32)
    return torch.from_numpy(words.view(np.int32))


@pytest.mark.parametrize("tile,M,N", [(24, 512, 256), (25, 512, 256), (26, 512, 256),
                                      (27, 512, 256), (28, 512, 256), (29, 512, 256),
                                      (56, 1024, 256), (57, 512, 256), (58, 512, 512),
                                      (59, 512, 256), (60, 512, 256), (56, 11520, 512)])
def test_relu_bitmask_rows_layout(tile, M, N):
    """relu | OCPPO_X6_MBITS_ROWS: the forward writes the row-major bitmask of its ReLU output
    (every tile shape: 4 / 8 waves, 16 FM x 16 FN wave fragments of FN = 2 or 4), the output
    unchanged; a NaN output (relu keeps it) is 'on', as threshold_backward treats it."""
    if ops.x6_tile(M, N, tile=tile) is None:
        pytest.skip("tile not built")
    g = torch.Generator(device=DEV).manual_seed(91)
    K0 = 256
    x = _rand(M, K0, gen=g)
    w = _rand(N, K0, gen=g, scale=K0 ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    x[3, 5] = float("nan")  # row 3 all NaN
    h = torch.empty(M, N, device=DEV)
    bits = torch.full((M, N // 32), -1, dtype=torch.int32, device=DEV)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h, N, M, N, K0, bias=b, relu=True, tile=tile,
                mbits_out=bits, mbits_rows=True)
    h_ref = torch.empty_like(h)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h_ref, N, M, N, K0, bias=b, relu=True, tile=tile)
    assert torch.equal(h.nan_to_num(7.0), h_ref.nan_to_num(7.0))
    assert bool(h[3].isnan().all())
    assert torch.equal(bits.cpu(), _rows_bits_ref(h))
    y, (rb, kind) = ops.linear_x6(x, w, b, relu=True, mbits="rows")
    assert kind == "rows" and torch.equal(rb.cpu(), _rows_bits_ref(y))


@pytest.mark.parametrize("mbig", [0, 512, 1024, None])
def test_mixed_tiles(mbig):
    # variant 56: rows [0, mbig) in 128 x 128 tiles, the rest in 64 x 128 (None: the library's
    # own split); forward with bias + ReLU + bitmask, then the masked dX reading that bitmask
    t = ops.X6_MIXED
    g = torch.Generator(device=DEV).manual_seed(57)
    M, K0, N, N2 = 1024, 256, 256, 128  # x [M, K0] -> h [M, N] -> [M, N2]
    x = _rand(M, K0, gen=g)
    w = _rand(N, K0, gen=g, scale=K0 ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    h = torch.empty(M, N, device=DEV)
    bits = torch.empty(ops.x6_mbits_words(M, N, t), dtype=torch.int64, device=DEV)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h, N, M, N, K0, bias=b, relu=True, tile=t, mbits_out=bits, mbig=mbig)
    pre64 = x.double() @ w.double().t() + b.double()
    scale = x.double().abs() @ w.double().abs().t() + b.double().abs()
    _check(h, pre64.clamp_min(0), scale, torch._addmm_activation(b, x, w.t()))
    gg = _rand(M, N2, gen=g)
    w2 = _rand(N2, N, gen=g, scale=N2 ** -0.5)
    gp_f, dbp_f = torch.empty(M, N, device=DEV), torch.full((M // 64, N), 7.0, device=DEV)
    gp_b, dbp_b = torch.empty(M, N, device=DEV), torch.full((M // 64, N), 7.0, device=DEV)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_f, N, M, N, N2, mask=h, dbp=dbp_f, tile=t, mbig=mbig)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_b, N, M, N, N2, dbp=dbp_b, tile=t, mbits_in=bits, mbig=mbig)
    assert torch.equal(gp_f, gp_b) and torch.equal(dbp_f, dbp_b)
    ref = torch.where(h > 0, gg.double() @ w2.double(), torch.zeros((), dtype=torch.float64, device=DEV))
    _check(gp_f, ref, gg.double().abs() @ w2.double().abs(), torch.ops.aten.threshold_backward(gg @ w2, h, 0))
    # every dbp row written (128-row tiles: their sum, then a zero row); pairs of rows sum to the
    # 128-row column sums of gp
    assert not bool((dbp_f == 7.0).any())
    pairs = dbp_f.double().view(M // 128, 2, N).sum(1)
    assert torch.allclose(pairs, gp_f.double().view(M // 128, 128, N).sum(1), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("R,C,trans", [(512, 256, 0), (1024, 512, 1), (100, 136, 0), (136, 96, 1),
                                       (2048, 512, 1)])
def test_split_planes_is_the_exact_split(R, C, trans):
    """ocppo_split_planes writes, bitwise, the three round-to-nearest bf16 pieces of every element
    (of W or W^T), the pieces gemm_x6 forms in its K loop; x0 + x1 + x2 == x exactly."""
    g = torch.Generator(device=DEV).manual_seed(R + C + trans)
    w = torch.randn(R, C, device=DEV, generator=g) * torch.exp(
        torch.randn(R, C, device=DEV, generator=g) * 3)
    w[0, :4] = torch.tensor([0.0, -0.0, 1e-30, 3.0e38])
    src = w.t().contiguous() if trans else w
    wp = ops.WeightPlanes(fwd=[] if trans else [w], dx=[w] if trans else [])
    wp.refresh()
    torch.cuda.synchronize()
    got = w._ocppo_planes["dx" if trans else "fwd"]
    ref = ops.split_planes_ref(src)
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    tot = got[0].double() + got[1].double() + got[2].double()
    assert torch.equal(tot, src.double())


def test_adam_step_writes_the_weight_planes():
    """FlatAdam.write_planes: the optimizer step also writes each registered weight's new values
    as its three exact bf16 pieces (of W, or of W^T), bitwise what ocppo_split_planes writes."""
    g = torch.Generator(device=DEV).manual_seed(5)
    lin1 = torch.nn.Linear(512, 256).to(DEV)
    lin2 = torch.nn.Linear(136, 1024).to(DEV)
    opt = ops.FlatAdam(list(lin1.parameters()) + list(lin2.parameters()), lr=1e-3, eps=1e-5,
                       max_grad_norm=0.5)
    w1, w2 = lin1.weight, lin2.weight
    p1 = torch.zeros(3, 256, 512, dtype=torch.bfloat16, device=DEV)
    p2 = torch.zeros(3, 136, 1024, dtype=torch.bfloat16, device=DEV)  # of W2^T
    opt.write_planes([(w1, 0, p1), (w2, 1, p2)])
    for _ in range(2):
        opt.grads.copy_(torch.randn(opt.numel, device=DEV, generator=g))
        opt.step()
    torch.cuda.synchronize()
    assert torch.equal(p1.view(torch.int16), ops.split_planes_ref(w1.detach()).view(torch.int16))
    assert torch.equal(p2.view(torch.int16),
                       ops.split_planes_ref(w2.detach().t().contiguous()).view(torch.int16))


@pytest.mark.parametrize("tile", [24, 25, 26, 27, 56])
def test_gemm_x6_presplit_b_is_bitwise_the_f32_b(tile):
    """The forward (bias + ReLU + bitmask) and the masked dX with B read as pre-split planes
    (WeightPlanes) give bitwise the outputs, bitmasks and bias-gradient partials of the f32 B."""
    g = torch.Generator(device=DEV).manual_seed(tile)
    M, K0, N, N2 = 1024, 256, 256, 128
    x = _rand(M, K0, gen=g)
    w = _rand(N, K0, gen=g, scale=K0 ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    w2 = _rand(N2, N, gen=g, scale=N2 ** -0.5)
    wp = ops.WeightPlanes(fwd=[w], dx=[w2])
    wp.refresh()
    if ops.x6_tile(M, N, 1, tile) is None or ops.x6_tile(M, N, 1, tile) != tile:
        pytest.skip("tile does not divide")
    t = tile
    # zeros: the mixed tile's 128-row tiles fill half of the 64-row-tile word slots
    bits_a = torch.zeros(ops.x6_mbits_words(M, N, t), dtype=torch.int64, device=DEV)
    bits_b = torch.zeros_like(bits_a)
    h_a, h_b = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h_a, N, M, N, K0, bias=b, relu=True, tile=t, mbits_out=bits_a)
    ops.gemm_x6(x, K0, 1, None, K0, 1, h_b, N, M, N, K0, bias=b, relu=True, tile=t,
                mbits_out=bits_b, b_planes=w._ocppo_planes["fwd"])
    assert torch.equal(h_a, h_b) and torch.equal(bits_a, bits_b)
    gg = _rand(M, N2, gen=g)
    bm = ops.X6_TILES[t][0]
    gp_a, dbp_a = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    gp_b, dbp_b = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_a, N, M, N, N2, dbp=dbp_a, tile=t, mbits_in=bits_a)
    ops.gemm_x6(gg, N2, 1, None, 1, N, gp_b, N, M, N, N2, dbp=dbp_b, tile=t, mbits_in=bits_a,
                b_planes=w2._ocppo_planes["dx"])
    assert torch.equal(gp_a, gp_b) and torch.equal(dbp_a, dbp_b)
    # unmasked dX and plain forward through the helpers
    assert torch.equal(ops.dx_x6(gg, w2), ops.dx_x6(gg, w2, planes=w2._ocppo_planes["dx"]))
    assert torch.equal(ops.linear_x6(x, w, b), ops.linear_x6(x, w, b, planes=w._ocppo_planes["fwd"]))


@pytest.mark.parametrize("M,N,K", [(4096, 512, 2048), (2048, 1024, 2048), (4096, 256, 4096)])
@pytest.mark.parametrize("planes", [False, True])
def test_forward_split_k_with_bias_relu_combine(M, N, K, planes):
    """The K-split forward (ops.linear_x6_split: gemm_x6 partials + ocppo_sum_splits_act) at
    f32 accuracy; the combine bitwise = the partials added in split order in f64, rounded once,
    + bias, then ReLU; pre-split weight planes bitwise the in-kernel split."""
    S = ops.x6_fwd_splits(M, N, K)
    assert S is not None and S * (M // 128) * (N // 128) >= 512
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = _rand(M, K, gen=g)
    w = _rand(N, K, gen=g, scale=K ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    pre64 = x.double() @ w.double().t() + b.double()
    scale = x.double().abs() @ w.double().abs().t() + b.double().abs()
    pl = None
    if planes:
        ops.WeightPlanes(fwd=[w]).refresh()
        pl = w._ocppo_planes["fwd"]
    out = ops.linear_x6_split(x, w, b, True, S, planes=pl)
    _check(out, pre64.clamp_min(0), scale, torch._addmm_activation(b, x, w.t()))
    # the combine itself, against its definition on the same partials
    part = torch.empty(S, M, N, device=DEV)
    ops.gemm_x6(x, K, 1, w, K, 1, part, N, M, N, K, splits=S, split_c=M * N, tile=ops.X6_AUTO)
    acc = part[0].double()
    for s in range(1, S):
        acc = acc + part[s].double()
    want = torch.relu(acc.float() + b)
    assert torch.equal(out, want)
    assert torch.equal(ops.linear_x6_split(x, w, b, True, S, planes=pl), out)  # repeatable
    nob = ops.linear_x6_split(x, w, None, False, S)
    assert torch.equal(nob, acc.float())


@pytest.mark.parametrize("tile", [24, 56])
@pytest.mark.parametrize("kind", ["fwd", "dw"])
def test_one_accumulator_variants_at_long_k(tile, kind):
    """The shipped one-accumulator variants (24, and the mixed 56) at K = 4096 in one split — the
    longest reduction config 2 runs (the decoder's weight gradient over 4096 sample rows) — at f32
    accuracy against f64 and beside hipBLASLt's f32 GEMM."""
    g = torch.Generator(device=DEV).manual_seed(4096 + tile)
    M, N, K = 256, 384, 4096
    if kind == "fwd":
        x = _rand(M, K, gen=g)
        w = _rand(N, K, gen=g, scale=K ** -0.5)
        ref = x.double() @ w.double().t()
        scale = x.double().abs() @ w.double().abs().t()
        out = torch.empty(M, N, device=DEV)
        ops.gemm_x6(x, K, 1, w, K, 1, out, N, M, N, K, tile=tile)
        _check(out, ref, scale, x @ w.t())
    else:
        if tile == 56:
            pytest.skip("the mixed tiles are not split-K / m-contiguous weight-gradient variants")
        gg = _rand(K, M, gen=g)  # dW [M, N] = g^T x over K rows, both operands row-contiguous
        x = _rand(K, N, gen=g)
        ref = gg.double().t() @ x.double()
        scale = gg.double().abs().t() @ x.double().abs()
        out = torch.empty(M, N, device=DEV)
        ops.gemm_x6(gg, 1, M, x, 1, N, out, N, M, N, K, tile=tile)
        _check(out, ref, scale, gg.t() @ x)


@pytest.mark.parametrize("tile", [27, 24])
@pytest.mark.parametrize("M,N,K,K1", [(4096, 256, 256, 12), (2048, 512, 256, 6), (128, 64, 64, 16),
                                      (8192, 256, 512, 3), (1024, 96, 128, 9)])
def test_dx_with_lower_layer_backward_epilogue(tile, M, N, K, K1):
    """ocppo_gemm_x6_wgrad: dX = g W is never stored; the epilogue forms gp = (mask > 0 ? dX : 0)
    and the lower layer's per-row-tile (gp^T x, gp.sum) records, finished by a deferred finish
    (alone or folded into a sum_splits_db combine). Checked against f64 threshold_backward(g W) ->
    gp^T x / gp.sum(0), scaled by (|g| |W|) masked, times |x| — f32 accuracy of both products."""
    if tile == 24 and (K % 128 or M % 128):
        pytest.skip("the 128 x 128 tile needs M and K multiples of 128")
    gen = torch.Generator(device=DEV).manual_seed(M + N + K + K1 + tile)
    g = _rand(M, N, gen=gen)
    w = _rand(N, K, gen=gen, scale=0.1)
    mask = torch.relu(_rand(M, K, gen=gen))
    mask[::7, ::3] = 0.0
    xs = _rand(M, K1 + 2, gen=gen)
    x = xs[:, 1:K1 + 1]  # row stride K1 + 2
    assert ops.dx_x6_wgrad_ok(g, w, mask, x)
    live = (mask > 0).double()
    gp = (g.double() @ w.double()) * live
    ref_w, ref_b = gp.t() @ x.double(), gp.sum(0)
    sgp = (g.double().abs() @ w.double().abs()) * live
    sw, sb = sgp.t() @ x.double().abs(), sgp.sum(0)
    outs = []
    for fold in (False, True):
        dw = torch.full((K, K1), float("nan"), device=DEV)
        db = torch.full((K,), float("nan"), device=DEV)
        fin = ops.DeferredFinish(DEV)
        ops.dx_x6_wgrad(g, w, mask, x, dw, db, fin, tile=tile)
        assert fin.pending
        if fold:
            part = _rand(4, 256 * 64, gen=gen)
            dbp = _rand(30, 128, gen=gen)
            o_ref, b_ref = torch.empty(256 * 64, device=DEV), torch.empty(128, device=DEV)
            ops.sum_splits_db(part, o_ref, (dbp, 30), b_ref)
            o, b_ = torch.empty_like(o_ref), torch.empty_like(b_ref)
            ops.sum_splits_db(part, o, (dbp, 30), b_, finish=fin)
            assert torch.equal(o, o_ref) and torch.equal(b_, b_ref)
        else:
            fin.run()
        assert not fin.pending
        torch.cuda.synchronize()
        assert ((dw.double() - ref_w).abs() / sw.clamp_min(1e-30)).max().item() < 1e-6
        assert ((db.double() - ref_b).abs() / sb.clamp_min(1e-30)).max().item() < 1e-6
        outs.append((dw, db))
    # alone or folded, bitwise the same (one fixed order)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_dx_with_lower_layer_backward_rejects_bad_sizes():
    g = torch.randn(4096, 256, device=DEV)
    w = torch.randn(256, 256, device=DEV)
    mask = torch.relu(torch.randn(4096, 256, device=DEV))
    fin = ops.DeferredFinish(DEV)
    dw, db = torch.empty(256, 17, device=DEV), torch.empty(256, device=DEV)
    with pytest.raises(RuntimeError, match="bad sizes"):
        ops.dx_x6_wgrad(g, w, mask, torch.randn(4096, 17, device=DEV), dw, db, fin)
    assert not fin.pending
    with pytest.raises(RuntimeError, match="bad sizes"):
        ops.dx_x6_wgrad(g[:4032], w, mask[:4032], torch.randn(4032, 12, device=DEV),
                        torch.empty(256, 12, device=DEV), db, fin, tile=24)  # M % 128


@pytest.mark.parametrize("tile", [57, 58, 59, 60])
def test_pipelined_tiles_every_epilogue(tile):
    """The pipelined family (two LDS stages, one barrier per K step): forward with bias + ReLU +
    bitmask, masked dX from the f32 mask and from the bitmask, plain dX and split-K dW -- each at
    f32 accuracy against f64, the two masked forms bitwise equal."""
    g = torch.Generator(device=DEV).manual_seed(tile)
    M, K0, N, N2 = 1024, 288, 512, 256
    x = _rand(M, K0, gen=g)
    w = _rand(N, K0, gen=g, scale=K0 ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    h = torch.empty(M, N, device=DEV)
    bits = torch.zeros(ops.x6_mbits_words(M, N, tile), dtype=torch.int64, device=DEV)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h, N, M, N, K0, bias=b, relu=True, tile=tile, mbits_out=bits)
    pre = x.double() @ w.double().t() + b.double()
    _check(h, pre.clamp_min(0), x.double().abs() @ w.double().abs().t() + b.double().abs(),
           torch.relu(x @ w.t() + b))
    gg = _rand(M, N2, gen=g)
    w2 = _rand(N2, N, gen=g, scale=N2 ** -0.5)
    bm = ops.X6_TILES[tile][0]
    gp_f, dbp_f = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    gp_b, dbp_b = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_f, N, M, N, N2, mask=h, dbp=dbp_f, tile=tile)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp_b, N, M, N, N2, dbp=dbp_b, tile=tile, mbits_in=bits)
    assert torch.equal(gp_f, gp_b) and torch.equal(dbp_f, dbp_b)
    ref = (gg.double() @ w2.double()) * (h > 0)
    _check(gp_f, ref, gg.double().abs() @ w2.double().abs(), (gg @ w2) * (h > 0))
    torch.testing.assert_close(dbp_f.double().sum(0), ref.sum(0), rtol=1e-5, atol=1e-4)
    out = torch.empty(M, N, device=DEV)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, out, N, M, N, N2, tile=tile)
    _check(out, gg.double() @ w2.double(), gg.double().abs() @ w2.double().abs(), gg @ w2)
    R, S = 2048, 4  # dW [N, K0] = gd [R, N]^T xd [R, K0]
    gd, xd = _rand(R, N, gen=g), _rand(R, K0, gen=g)
    if ops.x6_tile(N, K0, S, tile) is None:
        return
    part = torch.empty(S, N, K0, device=DEV)
    ops.gemm_x6(gd, 1, N, xd, 1, K0, part, K0, N, K0, R, splits=S, split_c=N * K0, tile=tile)
    nk = R // 32
    for s in range(S):
        r0, r1 = 32 * (s * nk // S), 32 * ((s + 1) * nk // S)
        _check(part[s], gd[r0:r1].double().t() @ xd[r0:r1].double(),
               gd[r0:r1].double().abs().t() @ xd[r0:r1].double().abs(), gd[r0:r1].t() @ xd[r0:r1])


@pytest.mark.parametrize("tile", [57, 58])
def test_pipelined_presplit_b_is_bitwise_the_f32_b(tile):
    g = torch.Generator(device=DEV).manual_seed(100 + tile)
    M, K0, N = 1024, 256, 512
    x = _rand(M, K0, gen=g)
    w = _rand(N, K0, gen=g, scale=K0 ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    wp = ops.WeightPlanes(fwd=[w])
    wp.refresh()
    h_a, h_b = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    ops.gemm_x6(x, K0, 1, w, K0, 1, h_a, N, M, N, K0, bias=b, relu=True, tile=tile)
    ops.gemm_x6(x, K0, 1, None, K0, 1, h_b, N, M, N, K0, bias=b, relu=True, tile=tile,
                b_planes=w._ocppo_planes["fwd"])
    assert torch.equal(h_a, h_b)


@pytest.mark.parametrize("tile", [57, 58])
@pytest.mark.parametrize("M,N,K", [(2048, 1024, 512), (1280, 768, 1024), (768, 1536, 96)])
def test_stream_k_products(tile, M, N, K):
    """The persistent stream-K launch (tiles split over the CUs of one XCD in K, finished by the
    workgroup holding each tile's first K steps): f32 accuracy against f64 with the bias / ReLU /
    bitmask epilogue and the masked dX, bitwise repeatable, and the workspace flags back at zero.
    Shapes: 4 parts per tile, uneven XCD shares, and more workgroups than K steps (empty ranges)."""
    if ops.x6_tile(M, N, 1, tile) is None:
        pytest.skip("tile does not divide")
    g = torch.Generator(device=DEV).manual_seed(M + N + K + tile)
    x = _rand(M, K, gen=g)
    w = _rand(N, K, gen=g, scale=K ** -0.5)
    b = _rand(N, gen=g, scale=0.1)
    h = torch.empty(M, N, device=DEV)
    bits = torch.zeros(ops.x6_mbits_words(M, N, tile), dtype=torch.int64, device=DEV)
    ops.gemm_x6(x, K, 1, w, K, 1, h, N, M, N, K, bias=b, relu=True, tile=tile, mbits_out=bits,
                stream_k=True)
    pre = x.double() @ w.double().t() + b.double()
    _check(h, pre.clamp_min(0), x.double().abs() @ w.double().abs().t() + b.double().abs(),
           torch.relu(x @ w.t() + b))
    h2 = torch.empty_like(h)
    for _ in range(3):
        ops.gemm_x6(x, K, 1, w, K, 1, h2, N, M, N, K, bias=b, relu=True, tile=tile, stream_k=True)
        assert torch.equal(h, h2)
    N2 = 256
    gg = _rand(M, N2, gen=g)
    w2 = _rand(N2, N, gen=g, scale=N2 ** -0.5)
    bm = ops.X6_TILES[tile][0]
    gp, dbp = torch.empty(M, N, device=DEV), torch.empty(M // bm, N, device=DEV)
    ops.gemm_x6(gg, N2, 1, w2, 1, N, gp, N, M, N, N2, dbp=dbp, tile=tile, mbits_in=bits,
                stream_k=True)
    ref = (gg.double() @ w2.double()) * (h > 0)
    _check(gp, ref, gg.double().abs() @ w2.double().abs(), (gg @ w2) * (h > 0))
    torch.cuda.synchronize()
    # the workspace ends with one int32 flag per workgroup (one per CU): all back at zero
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count // 8 * 8
    assert int(ops.x6_sk_workspace(tile, DEV).view(torch.int32)[-cus:].abs().sum()) == 0
