"""Host-side choices of the update GEMM path (no GPU): which config-2 products run on
ocppo_gemm_x6, with which tile and row split (agents._x6 / _x6_dw / _x6_splits, ops.x6_tile), and
the bench's parsing of the gemm_x6 timer sites. The measurements behind the rules are
profiles/r03/exp_gemm_x6*.jsonl."""
import bench
from oc_cleanrl_amd import agents, ops

# config 2's update products per minibatch: encoder at the dedup capacity (11520 frames),
# decoder at the minibatch (4096); (M, N_out, K_in) of each Linear
LAYERS = {"L2": (11520, 512, 256), "L3": (11520, 1024, 512), "L4": (11520, 512, 1024),
          "dec": (4096, 512, 2048)}


def test_forward_and_dx_gating_matches_the_measurements():
    on = {k: agents._x6(M, N, K) for k, (M, N, K) in LAYERS.items()}
    # forward [M, N]: the decoder's 128 tiles of 128 x 128 stay on hipBLASLt (79 vs 62 us)
    assert on == {"L2": True, "L3": True, "L4": True, "dec": False}
    # dX [M, K] = g [M, N] W: the second layer's [11520 x 256] stays on hipBLASLt
    dx = {k: agents._x6(M, K, N) for k, (M, N, K) in LAYERS.items()}
    assert dx == {"L2": False, "L3": True, "L4": True, "dec": True}


def test_weight_grad_gating_and_split():
    dw = {k: agents._x6_dw(N, K, M) for k, (M, N, K) in LAYERS.items()}
    assert dw == {"L2": False, "L3": True, "L4": True, "dec": True}
    # 128 x 128 tiles (variant 24) with the fewest splits reaching two workgroups per CU
    assert agents._x6_splits(11520, 1024, 512) == (16, 24)
    assert agents._x6_splits(11520, 512, 1024) == (16, 24)
    assert agents._x6_splits(4096, 512, 2048) == (8, 24)
    assert agents._x6_splits(100, 512, 512) is None  # rows not a multiple of 32


def test_tile_choice():
    assert ops.X6_AUTO == 24 and ops.X6_TILES[24] == (128, 128)
    assert ops.x6_tile(11520, 1024) == 24  # 720 tiles
    assert ops.x6_tile(11520, 512) == ops.X6_MIXED == 56  # 360 tiles: 256 of 128 x 128 + 208 x 2
    assert ops.X6_TILES[56] == (64, 128) and ops.x6_tile(11520, 512, 2) == 24
    assert ops.x6_tile(4096, 512) == 25  # 128 tiles of 128 x 128 -> 64 x 128 (256)
    assert ops.x6_tile(96, 128) is None
    assert ops.x6_tile(512, 1024, 16) == 24
    assert ops.x6_tile(128, 128, 1, 3) == 3 and ops.x6_tile(96, 128, 1, 3) is None
    assert ops.x6_tile(128, 128, 1, 57) is None and ops.x6_tile(128, 128, 1, 64) is None
    for t in ops.X6_BUILT:
        assert 0 <= t < 64


def test_mbits_words():
    # one 64-bit word per thread and tile: 720 tiles x 256 threads at [11520 x 1024]
    assert ops.x6_mbits_words(11520, 1024, 24) == 720 * 256
    assert ops.x6_mbits_words(128, 128, 28) == 512  # 8-wave shape: 512 threads


def test_bench_parses_gemm_sites():
    assert bench.gemm_x6_shape("gemm_x6_11520x1024x512s1m") == (11520, 1024, 512, 1, "m")
    assert bench.gemm_x6_shape("gemm_x6_512x1024x11520s16") == (512, 1024, 11520, 16, "")
    assert bench.gemm_x6_shape("gemm_x6_11520x256x512s1w") == (11520, 256, 512, 1, "w")
    assert bench.gemm_x6_bytes("gemm_x6_11520x256x512s1w") == 4 * (
        11520 * 512 + 256 * 512 + 11520 * 256)
    M, N, K = 11520, 1024, 512
    assert bench.gemm_x6_bytes("gemm_x6_11520x1024x512s1") == 4 * (M * K + N * K + M * N)
    assert bench.gemm_x6_bytes("gemm_x6_11520x1024x512s1m") == (
        4 * (M * K + N * K + M * N) + M * N // 8 + 4 * N * (M // 128))


def test_update_gemm_route_is_per_agent():
    """Two agents in one process keep their own update-GEMM route (Args.x6_gemm per trainer):
    agents.set_update_gemm marks each Linear's weight, nothing process-wide changes."""
    import torch.nn as nn

    from oc_cleanrl_amd import agents

    a = agents.make_agent("PPO_OBJ", (4, 12), 6)
    b = agents.make_agent("PPO_OBJ", (4, 12), 6)
    agents.set_update_gemm(a, False)
    agents.set_update_gemm(b, True)
    lins_a = [m for m in a.modules() if isinstance(m, nn.Linear)]
    lins_b = [m for m in b.modules() if isinstance(m, nn.Linear)]
    assert lins_a and all(not agents.x6_route(m.weight) for m in lins_a)
    assert all(agents.x6_route(m.weight) for m in lins_b)
    assert agents.x6_route(nn.Linear(4, 4).weight) == agents.X6_GEMM_DEFAULT
    assert not hasattr(agents, "X6_GEMM") and not hasattr(agents, "X6_MASK_DX")


def test_split_planes_ref_is_exact():
    """The three round-to-nearest bf16 pieces of an f32 sum back to it exactly (the premise of
    gemm_x6 and of its pre-split weights)."""
    import torch

    from oc_cleanrl_amd import ops

    g = torch.Generator().manual_seed(0)
    x = torch.randn(4096, generator=g) * torch.exp(torch.randn(4096, generator=g) * 4)
    p = ops.split_planes_ref(x)
    assert p.shape == (3, 4096) and p.dtype == torch.bfloat16
    assert torch.equal(p[0].double() + p[1].double() + p[2].double(), x.double())
    # each piece is the nearest bf16 of what remains
    assert torch.equal(p[0], x.to(torch.bfloat16))
