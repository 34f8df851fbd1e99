"""ocppo_conv_x6: the NatureCNN convolutions (cleanrl/architectures/ppo.py:20-31) as implicit GEMMs
on the x6 products — forward (+ bias + ReLU), weight gradient and data gradient (include/ocppo.h).

Accuracy against a float64 convolution on the host, scaled by the same convolution of |x| and |w|
(the bound an f32 dot product's rounding obeys), next to MIOpen's own f32 convolution on the same
operands; determinism as bitwise-equal repeats (the reference runs with
torch.use_deterministic_algorithms(True), ppo_atari_oc.py:200-211)."""
import pytest
import torch
import torch.nn.functional as F

from oc_cleanrl_amd import ops

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
CL = torch.channels_last

# (B, C, H, Cout, K, stride): the NatureCNN layers at batches whose row counts the tiles divide
LAYERS = {
    "conv1": (16, 4, 84, 32, 8, 4),
    "conv2": (128, 32, 20, 64, 4, 2),
    "conv3": (128, 64, 9, 64, 3, 1),
}


def _operands(name, seed=0):
    B, C, H, Cout, K, s = LAYERS[name]
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.rand(B, C, H, H, device=DEV, generator=g).contiguous(memory_format=CL)
    w = ((torch.rand(Cout, C, K, K, device=DEV, generator=g) * 2 - 1) / (C * K * K) ** 0.5
         ).contiguous(memory_format=CL)
    b = (torch.rand(Cout, device=DEV, generator=g) * 2 - 1) * 0.1
    return x, w, b, s


def _rel(y, ref, scale):
    d = (y.double().cpu() - ref).abs() / scale.clamp_min(1e-300)
    return float(d.max()), float(d.mean())


def _check(y, ref, scale, lib):
    mx, mean = _rel(y, ref, scale)
    lmx, lmean = _rel(lib, ref, scale)
    # f32 level: at most a few units of 2^-24 of sum |x w|, on average below one f32 rounding
    # (2^-24 ~ 6e-8) or within 2x of MIOpen's f32 convolution, whichever is looser (MIOpen's
    # own error depends on the solution it picks: 9e-10 .. 6e-9 in these tests)
    assert mx <= 1e-6, (mx, lmx)
    assert mean <= max(2.0 * lmean, 2e-8), (mean, lmean)


@pytest.mark.parametrize("name", list(LAYERS))
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("form", ["rows", "splits", "loop"])
def test_forward_bias_relu(name, relu, form, monkeypatch):
    """rows: tile 7, a 32-row tile per workgroup with its K steps split over 8 waves (the
    rollout's form, ops.CONV_FWD_ROWS); splits: K-split partials + ocppo_sum_splits_act; loop: one
    product with bias + ReLU in its epilogue (the update's form)."""
    monkeypatch.setattr(ops, "CONV_FWD_ROWS", form == "rows")
    monkeypatch.setattr(ops, "CONV_FWD_SPLITS", form == "splits")
    x, w, b, s = _operands(name)
    assert ops.conv_x6_ok(x, w, s)
    y = ops.conv_x6(x, w, b, s, relu)
    assert y.is_contiguous(memory_format=CL)
    x64, w64, b64 = x.double().cpu(), w.double().cpu(), b.double().cpu()
    ref = F.conv2d(x64, w64, b64, stride=s)
    scale = F.conv2d(x64.abs(), w64.abs(), b64.abs(), stride=s)
    lib = F.conv2d(x, w, b, stride=s)
    if relu:
        ref, lib = ref.clamp_min(0), lib.clamp_min(0)
    _check(y, ref, scale, lib)
    assert torch.equal(y, ops.conv_x6(x, w, b, s, relu))  # deterministic


@pytest.mark.parametrize("name", list(LAYERS))
def test_weight_gradient(name):
    x, w, _, s = _operands(name, 1)
    Cout, C, K, _ = w.shape
    OH = (x.shape[2] - K) // s + 1
    g = torch.Generator(device=DEV).manual_seed(2)
    gp = (torch.rand(x.shape[0], Cout, OH, OH, device=DEV, generator=g) * 2 - 1
          ).contiguous(memory_format=CL)
    rows = gp.permute(0, 2, 3, 1).reshape(-1, Cout)
    assert ops.conv_x6_ok(x, w, s, wgrad=True)
    dw = ops.conv_x6_wgrad(rows, x, (K, K), s)  # [Cout, K K C]
    dw = dw.view(Cout, K, K, C).permute(0, 3, 1, 2)
    x64, gp64 = x.double().cpu(), gp.double().cpu()
    ref = torch.nn.grad.conv2d_weight(x64, w.shape, gp64, stride=s)
    scale = torch.nn.grad.conv2d_weight(x64.abs(), w.shape, gp64.abs(), stride=s)
    lib = torch.nn.grad.conv2d_weight(x, w.shape, gp, stride=s)
    _check(dw, ref, scale, lib)
    dw2 = ops.conv_x6_wgrad(rows, x, (K, K), s).view(Cout, K, K, C).permute(0, 3, 1, 2)
    assert torch.equal(dw, dw2)  # deterministic: split partials summed in order


@pytest.mark.parametrize("name", ["conv2", "conv3"])
@pytest.mark.parametrize("pad_copy", [False, True])
def test_data_gradient(name, pad_copy, monkeypatch):
    """pad_copy: over an F.pad copy of the output gradient; else the loader's bounds (default)."""
    monkeypatch.setattr(ops, "CONV_DGRAD_PAD_COPY", pad_copy)
    x, w, _, s = _operands(name, 3)
    Cout, C, K, _ = w.shape
    H = x.shape[2]
    OH = (H - K) // s + 1
    g = torch.Generator(device=DEV).manual_seed(4)
    gp = (torch.rand(x.shape[0], Cout, OH, OH, device=DEV, generator=g) * 2 - 1
          ).contiguous(memory_format=CL)
    assert ops.conv_x6_ok(x, w, s, dgrad=True)
    dx = ops.conv_x6_dgrad(gp, w, s, (H, H))
    assert dx.is_contiguous(memory_format=CL)
    w64, gp64 = w.double().cpu(), gp.double().cpu()
    ref = torch.nn.grad.conv2d_input(x.shape, w64, gp64, stride=s)
    scale = torch.nn.grad.conv2d_input(x.shape, w64.abs(), gp64.abs(), stride=s)
    lib = torch.nn.grad.conv2d_input(x.shape, w, gp, stride=s)
    _check(dx, ref, scale, lib)
    assert torch.equal(dx, ops.conv_x6_dgrad(gp, w, s, (H, H)))


def test_config3_minibatch_shapes_are_taken():
    """Every layer of config 3's update (minibatch 8192) and rollout (256 envs) forward fits."""
    for B in (8192, 256):
        for name, (_, C, H, Cout, K, s) in LAYERS.items():
            x = torch.empty(B, C, H, H, device=DEV).contiguous(memory_format=CL)
            w = torch.empty(Cout, C, K, K, device=DEV).contiguous(memory_format=CL)
            assert ops.conv_x6_ok(x, w, s), (B, name)
            if B == 8192:
                assert ops.conv_x6_ok(x, w, s, wgrad=True, dgrad=name != "conv1"), name


def test_rejects_bad_shapes():
    x, w, b, s = _operands("conv2")
    with pytest.raises(ValueError):
        ops.conv_x6(x.contiguous(), w, b, s)  # NCHW x
    with pytest.raises(ValueError):
        ops.conv_x6(x[:3].contiguous(memory_format=CL), w, b, s)  # 243 rows: no tile divides


def _frames(R=40, seed=5):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randint(0, 256, (R, 4, 84, 84), device=DEV, generator=g, dtype=torch.uint8)


@pytest.mark.parametrize("relu", [True, False])
def test_u8_first_conv_forward(relu):
    """conv_x6_u8: NormalizeImg + the 8x8/4 convolution read from u8 frame stacks through a sample
    index, against f64 on the gathered, normalised observations."""
    src = _frames()
    _, w, b, s = _operands("conv1")
    idx = torch.randperm(src.shape[0], device=DEV)[:16]
    assert ops.conv_x6_u8_ok(src, w, s, 16, wgrad=True)
    y = ops.conv_x6_u8(src, idx, w, b, s, relu)
    assert y.is_contiguous(memory_format=CL)
    x = src[idx].float() / 255.0  # the reference's NormalizeImg (f32)
    x64, w64, b64 = x.double().cpu(), w.double().cpu(), b.double().cpu()
    ref = F.conv2d(x64, w64, b64, stride=s)
    scale = F.conv2d(x64.abs(), w64.abs(), b64.abs(), stride=s)
    lib = F.conv2d(x, w, b, stride=s)
    if relu:
        ref, lib = ref.clamp_min(0), lib.clamp_min(0)
    _check(y, ref, scale, lib)
    assert torch.equal(y, ops.conv_x6_u8(src, idx, w, b, s, relu))


def test_u8_first_conv_weight_gradient():
    src = _frames(seed=6)
    _, w, _, s = _operands("conv1", 7)
    idx = torch.randperm(src.shape[0], device=DEV)[:16]
    g = torch.Generator(device=DEV).manual_seed(8)
    gp = (torch.rand(16, 32, 20, 20, device=DEV, generator=g) * 2 - 1).contiguous(memory_format=CL)
    rows = gp.permute(0, 2, 3, 1).reshape(-1, 32)
    dw = ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s).view(w.shape)  # (c, ky, kx) order
    x = src[idx].float() / 255.0
    x64, gp64 = x.double().cpu(), gp.double().cpu()
    ref = torch.nn.grad.conv2d_weight(x64, w.shape, gp64, stride=s)
    scale = torch.nn.grad.conv2d_weight(x64.abs(), w.shape, gp64.abs(), stride=s)
    lib = torch.nn.grad.conv2d_weight(x.contiguous(memory_format=CL), w.shape, gp, stride=s)
    _check(dw, ref, scale, lib)
    assert torch.equal(dw, ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s).view(w.shape))


@pytest.mark.parametrize("name", ["conv2", "conv3"])
def test_data_gradient_takes_the_relu_backward_below(name):
    """relu_out: the layer below's ReLU backward in the data gradient's epilogue — bitwise the
    unfused dX masked where relu_out <= 0 — and its bias gradient from the masked sums (f64)."""
    x, w, _, s = _operands(name, 9)
    Cout, C, K, _ = w.shape
    H = x.shape[2]
    OH = (H - K) // s + 1
    g = torch.Generator(device=DEV).manual_seed(10)
    gp = (torch.rand(x.shape[0], Cout, OH, OH, device=DEV, generator=g) * 2 - 1
          ).contiguous(memory_format=CL)
    below = (torch.rand(x.shape, device=DEV, generator=g) - 0.4).clamp_min(0).contiguous(
        memory_format=CL)  # a ReLU output: ~40 % zeros
    assert ops.conv_x6_dgrad_fuses_relu(x.shape[0] * (H // s) ** 2, C, s)
    db = torch.empty(C, device=DEV)
    fused = ops.conv_x6_dgrad(gp, w, s, (H, H), relu_out=below, db=db)
    plain = ops.conv_x6_dgrad(gp, w, s, (H, H))
    want = torch.where(below > 0, plain, torch.zeros_like(plain))
    assert torch.equal(fused, want)
    ref = want.double().sum((0, 2, 3))
    assert torch.allclose(db.double(), ref, rtol=1e-6, atol=1e-6 * float(want.abs().sum()) / C)


def test_u8_weight_gradient_index_slice_ends_before_a_sentinel():
    """ADVICE r05 (the round-5 fault): the u8 weight-gradient loader walks each thread's K rows
    image by image and must not read the index one past the minibatch's last image. idx here is a
    slice of a longer int64 buffer whose next element is far out of range: a read of it would
    fault or change the result. Bitwise the same gradient as from a private copy of idx."""
    src = _frames(seed=11)
    _, w, _, s = _operands("conv1", 12)
    B = 16
    buf = torch.full((B + 1,), 1 << 40, dtype=torch.int64, device=DEV)
    buf[:B] = torch.randperm(src.shape[0], device=DEV)[:B]
    idx = buf[:B]
    g = torch.Generator(device=DEV).manual_seed(13)
    gp = (torch.rand(B, 32, 20, 20, device=DEV, generator=g) * 2 - 1).contiguous(memory_format=CL)
    rows = gp.permute(0, 2, 3, 1).reshape(-1, 32)
    dw = ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s)
    assert torch.equal(dw, ops.conv_x6_u8_wgrad(rows, src, idx.clone(), (8, 8), s))
    x = src[idx].float() / 255.0
    ref = torch.nn.grad.conv2d_weight(x.double().cpu(), w.shape, gp.double().cpu(), stride=s)
    assert float((dw.view(w.shape).double().cpu() - ref).abs().max()) <= 1e-6 * float(
        torch.nn.grad.conv2d_weight(x.double().cpu().abs(), w.shape, gp.double().cpu().abs(),
                                    stride=s).max())


@pytest.mark.skipif(not ops.X6_BOUNDS, reason="bounds-check build only (OCPPO_LIB=... "
                    "-DOCPPO_X6_BOUNDS, tools/run_bounds_check.sh)")
@pytest.mark.parametrize("form", ["image", "loop", "wgrad_image", "wgrad_loop"])
def test_bounds_build_records_an_out_of_range_stack_row(form):
    """Positive control of the bounds-check build: an index past the u8 stacks' rows is recorded
    (kind 3, the index, the limit) instead of being read (the load falls back to row 0), in the
    image-staged kernels (tiles 7 / 8) and the tile loop's gathers (tiles 0 / 1)."""
    src = _frames(R=20, seed=14)
    _, w, b, s = _operands("conv1", 15)
    idx = torch.arange(16, device=DEV)
    idx[5] = 20  # one past the last stack
    rec = ops.bounds_record(DEV)
    rec.zero_()
    if form.startswith("wgrad"):
        gp = torch.rand(16 * 400, 32, device=DEV)
        ops.conv_x6_u8_wgrad(gp, src, idx, (8, 8), s, tile=8 if form == "wgrad_image" else 1)
    else:
        ops.conv_x6_u8(src, idx, w, b, s, True, tile=7 if form == "image" else 0)
    torch.cuda.synchronize()
    r = rec.cpu().tolist()
    rec.zero_()
    assert r[0] > 0 and r[1] == 3 and r[2] == 20 and r[4] == 20, r


@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("B", [16, 600])
def test_u8_first_conv_image_staged_is_bitwise_the_tile_loop(relu, B):
    """ocppo_conv_x6_u8 tile 7 (each image's u8 stack staged in LDS once, the weight's pieces in
    registers, a persistent loop over images) against the tile loop (tile 0): the same products in
    the same order, so the same bits; B = 600 images exceeds the persistent grid (512 workgroups)."""
    src = _frames(R=B + 7, seed=16)
    _, w, b, s = _operands("conv1", 17)
    idx = torch.randperm(src.shape[0], device=DEV)[:B]
    assert ops._conv_u8_img_ok(src, w, s)
    staged = ops.conv_x6_u8(src, idx, w, b, s, relu, tile=7)
    loop = ops.conv_x6_u8(src, idx, w, b, s, relu, tile=0)
    assert torch.equal(staged, loop), float((staged - loop).abs().max())
    assert torch.equal(staged, ops.conv_x6_u8(src, idx, w, b, s, relu))  # the default routes to 7


@pytest.mark.parametrize("B", [16, 300])
def test_u8_first_conv_image_staged_weight_gradient(B):
    """ocppo_conv_x6_u8 tile 8 (each image's stack in LDS once, rewritten per channel as
    tap-column rows; K taken image by image, 4 wave partials per workgroup summed in order)
    against a float64 weight gradient, next to the tile loop (tile 1), and bitwise repeatable.
    B = 300 puts several images on some workgroups (one workgroup per CU at most)."""
    src = _frames(R=B + 5, seed=18)
    _, w, _, s = _operands("conv1", 19)
    idx = torch.randperm(src.shape[0], device=DEV)[:B]
    g = torch.Generator(device=DEV).manual_seed(20)
    gp = (torch.rand(B, 32, 20, 20, device=DEV, generator=g) * 2 - 1).contiguous(memory_format=CL)
    rows = gp.permute(0, 2, 3, 1).reshape(-1, 32)
    assert ops._conv_u8_img_wgrad_ok(src, (8, 8), s, 32)
    dw = ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s, tile=8).view(w.shape)
    loop = ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s, tile=1).view(w.shape)
    x = src[idx].float() / 255.0
    x64, gp64 = x.double().cpu(), gp.double().cpu()
    ref = torch.nn.grad.conv2d_weight(x64, w.shape, gp64, stride=s)
    scale = torch.nn.grad.conv2d_weight(x64.abs(), w.shape, gp64.abs(), stride=s)
    lib = torch.nn.grad.conv2d_weight(x.contiguous(memory_format=CL), w.shape, gp, stride=s)
    _check(dw, ref, scale, lib)
    _check(loop, ref, scale, lib)
    assert torch.equal(dw, ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s, tile=8).view(w.shape))
    assert torch.equal(dw, ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s).view(w.shape))


@pytest.mark.parametrize("B", [16, 304])
def test_u8_first_conv_relu_backward_fused_into_the_weight_gradient(B):
    """The forward's ReLU bitmask (tile 7, mbits) handed to the weight-gradient kernel (tile 8)
    with the UNMASKED output gradient: the kernel's ReLU backward gives bitwise the dW of the
    masked gradient (relu_bias_grad's threshold_backward first, as the unfused backward does),
    and its per-channel sums the bias gradient (against relu_bias_grad's and a float64 sum)."""
    src = _frames(R=B + 5, seed=21)
    _, w, b, s = _operands("conv1", 22)
    idx = torch.randperm(src.shape[0], device=DEV)[:B]
    mb = torch.full((B * 400,), -1, dtype=torch.int32, device=DEV)
    y = ops.conv_x6_u8(src, idx, w, b, s, True, mbits=mb)
    assert torch.equal(y, ops.conv_x6_u8(src, idx, w, b, s, True))
    yr = y.permute(0, 2, 3, 1).reshape(-1, 32)
    bits = torch.stack([(mb >> c) & 1 for c in range(32)], 1).bool()
    assert torch.equal(bits, yr > 0)
    g = torch.Generator(device=DEV).manual_seed(23)
    gu = (torch.rand(B, 32, 20, 20, device=DEV, generator=g) * 2 - 1).contiguous(memory_format=CL)
    rows = gu.permute(0, 2, 3, 1).reshape(-1, 32)
    db_ref = torch.empty(32, device=DEV)
    gp, _ = ops.relu_bias_grad(rows, yr.contiguous(), db=db_ref)
    dw_ref = ops.conv_x6_u8_wgrad(gp, src, idx, (8, 8), s, tile=8)
    db = torch.full((32,), float("nan"), device=DEV)
    dw = ops.conv_x6_u8_wgrad(rows, src, idx, (8, 8), s, mbits=mb, db=db)
    assert torch.equal(dw, dw_ref)
    db64 = torch.where(yr > 0, rows, 0).double().sum(0)
    scale = rows.abs().double().sum(0)
    assert float(((db.double() - db64).abs() / scale).max()) < 1e-6
    assert float(((db_ref.double() - db64).abs() / scale).max()) < 1e-6
    db2 = torch.empty(32, device=DEV)  # without the mask: the plain column sums
    ops.conv_x6_u8_wgrad(gp, src, idx, (8, 8), s, db=db2)
    assert float(((db2.double() - db64).abs() / scale).max()) < 1e-6
    with pytest.raises(ValueError):
        ops.conv_x6_u8(src, idx, w, b, s, False, mbits=mb)  # a mask needs the ReLU


@pytest.mark.parametrize("name,B", [("conv2", 256), ("conv3", 256), ("conv2", 1), ("conv3", 32)])
def test_forward_rows_tile_at_rollout_sizes(name, B, monkeypatch):
    """ocppo_conv_x6 tile 7 at the rollout's batch (256 envs: 20736 / 12544 rows) and at odd
    small batches: against float64, and against the tile loop (the update's form) to f32 level."""
    _, C, H, Cout, K, s = LAYERS[name]
    g = torch.Generator(device=DEV).manual_seed(31)
    x = torch.rand(B, C, H, H, device=DEV, generator=g).contiguous(memory_format=CL)
    w = ((torch.rand(Cout, C, K, K, device=DEV, generator=g) * 2 - 1) / (C * K * K) ** 0.5
         ).contiguous(memory_format=CL)
    b = (torch.rand(Cout, device=DEV, generator=g) * 2 - 1) * 0.1
    OH = (H - K) // s + 1
    if (B * OH * OH) % 32:
        pytest.skip("rows not a multiple of 32")
    y = ops.conv_x6(x, w, b, s, True)
    x64, w64, b64 = x.double().cpu(), w.double().cpu(), b.double().cpu()
    ref = F.conv2d(x64, w64, b64, stride=s).clamp_min(0)
    scale = F.conv2d(x64.abs(), w64.abs(), b64.abs(), stride=s)
    _check(y, ref, scale, F.conv2d(x, w, b, stride=s).clamp_min(0))
    assert torch.equal(y, ops.conv_x6(x, w, b, s, True))
    # the weight pre-split once (the rollout's form, agents._planes_infer): the same pieces, so
    # the same bits
    wm = w.permute(0, 2, 3, 1).reshape(Cout, -1)
    ops.WeightPlanes(fwd=(wm,)).refresh()
    assert torch.equal(y, ops.conv_x6(x, w, b, s, True, w_planes=wm._ocppo_planes["fwd"]))
    if ops.conv_x6_ok(x, w, s):
        monkeypatch.setattr(ops, "CONV_FWD_ROWS", False)
        loop = ops.conv_x6(x, w, b, s, True)
        assert float(((loop.double() - y.double()).abs().cpu() / scale.clamp_min(1e-300)).max()) < 1e-6


@pytest.mark.parametrize("name", ["conv2", "conv3"])
def test_pre_split_weight_planes_are_bitwise_the_in_kernel_split(name, monkeypatch):
    """The forward's weight and the data gradient's class weights pre-split into bf16 planes
    (ocppo_conv_x6 w_planes, ocppo_split_planes: the update's form) give the same bits as the
    tile loop splitting them in every workgroup."""
    monkeypatch.setattr(ops, "CONV_FWD_ROWS", False)
    x, w, b, s = _operands(name, 41)
    Cout = w.shape[0]
    wm = w.permute(0, 2, 3, 1).reshape(Cout, -1)
    ops.WeightPlanes(fwd=(wm,)).refresh()
    y = ops.conv_x6(x, w, b, s, True)
    assert torch.equal(y, ops.conv_x6(x, w, b, s, True, w_planes=wm._ocppo_planes["fwd"]))
    g = torch.Generator(device=DEV).manual_seed(42)
    gp = (torch.rand(y.shape, device=DEV, generator=g) * 2 - 1).contiguous(memory_format=CL)
    monkeypatch.setattr(ops, "CONV_DGRAD_PLANES", False)
    dx = ops.conv_x6_dgrad(gp, w, s, tuple(x.shape[2:]))
    monkeypatch.setattr(ops, "CONV_DGRAD_PLANES", True)
    assert torch.equal(dx, ops.conv_x6_dgrad(gp, w, s, tuple(x.shape[2:])))


@pytest.mark.parametrize("name", ["conv2", "conv3"])
def test_forward_relu_bitmask_feeds_relu_bias_grad(name, monkeypatch):
    """The tile loop's forward epilogue writes the ReLU mask row-major (ocppo_conv_x6
    mbits_rows): bit = output > 0; ocppo_relu_bias_grad_bits reading it gives bitwise the gp and
    db of ocppo_relu_bias_grad reading the f32 output."""
    monkeypatch.setattr(ops, "CONV_FWD_ROWS", False)
    x, w, b, s = _operands(name, 51)
    Cout = w.shape[0]
    y0 = ops.conv_x6(x, w, b, s, True)
    M = y0.numel() // Cout
    mb = torch.full((M * Cout // 32,), -1, dtype=torch.int32, device=DEV)
    y = ops.conv_x6(x, w, b, s, True, mbits=mb)
    assert torch.equal(y, y0)
    yr = y.permute(0, 2, 3, 1).reshape(-1, Cout)
    words = mb.view(M, Cout // 32)
    bits = torch.stack([(words[:, c // 32] >> (c % 32)) & 1 for c in range(Cout)], 1).bool()
    assert torch.equal(bits, yr > 0)
    g = torch.Generator(device=DEV).manual_seed(52)
    g2 = torch.rand(M, Cout, device=DEV, generator=g) * 2 - 1
    gp_ref, db_ref = ops.relu_bias_grad(g2, yr.contiguous())
    gp, db = ops.relu_bias_grad(g2, bits=mb)
    assert torch.equal(gp, gp_ref) and torch.equal(db, db_ref)
