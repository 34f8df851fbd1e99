"""Frame-deduplicated PPObj minibatch: host planner (oc_cleanrl_amd/frames.py) and the oracle's
restatement of the frame timeline (oracle/ocppo_oracle.py), on CPU.

The key property: for every sample b = t*N + n of a minibatch, the frames the plan gathers,
indexed through pos_of at the sample's slot timeline ids, ARE the stored observation obs[t, n]
that the reference feeds its encoder (ppo_atari_oc.py:566, b_obs[mb_inds]) -- bit for bit, for
rollouts with resets anywhere (including obs[0] and consecutive resets)."""
import numpy as np
import pytest

from oc_cleanrl_amd.frames import FramePlanner
from oracle import ocppo_oracle as O


def _rollout(T, N, W, F, p_done, rng, done0):
    """obs [T+1, N, W, F] and dones [T+1, N] built with the store rule of the trainer."""
    obs = np.zeros((T + 1, N, W, F), np.float32)
    dones = np.zeros((T + 1, N), np.float32)
    dones[0] = done0
    first = rng.integers(0, 200, (N, W, F)).astype(np.float32)
    for n in range(N):  # a reset stack when dones[0] says so
        if done0[n]:
            first[n, :] = first[n, -1]
    obs[0] = first
    for t in range(T):
        frame = rng.integers(0, 200, (N, F)).astype(np.float32)
        d = (rng.random(N) < p_done).astype(np.float32)
        obs[t + 1] = O.rollout_store(frame, d, obs[t])
        dones[t + 1] = d
    return obs, dones


def _plan(T, N, W, M, E, nmb, rng):
    pl = FramePlanner(T, N, W, M, E, nmb)
    B = T * N
    perm = np.concatenate([rng.permutation(B) for _ in range(E)]).astype(np.int64)
    used, inv = pl.plan(perm)
    cap = pl.cap_for(pl.counts)
    buf = np.zeros(pl.size(cap), np.int32)
    pl.fill(buf, cap, used, inv)
    return pl, perm, pl.views(buf, cap), cap


@pytest.mark.parametrize("T,N,W,M,E,nmb,p_done", [(16, 8, 4, 32, 2, 4, 0.2), (9, 5, 3, 15, 1, 3, 0.5),
                                                 (12, 4, 1, 12, 2, 4, 0.3), (20, 3, 6, 15, 1, 4, 0.4)])
def test_plan_matches_set_restatement(T, N, W, M, E, nmb, p_done):
    rng = np.random.default_rng(1)
    pl, perm, (uniq, pos_of, inv), cap = _plan(T, N, W, M, E, nmb, rng)
    B = T * N
    assert cap % pl.align == 0 or cap == M * W
    for j in range(E * nmb):
        mb = perm[j * M:(j + 1) * M]
        want = sorted({int((b // N + k) * N + b % N) for b in mb for k in range(W)})
        got = uniq[j][uniq[j] >= 0]
        assert list(got) == want and pl.counts[j] == len(want) <= cap
        assert np.all(uniq[j][len(want):] == -1)
        assert np.array_equal(pos_of[j][want], np.arange(len(want)))
    for e in range(E):
        assert np.array_equal(inv[e][perm[e * B:(e + 1) * B]], np.arange(B))


@pytest.mark.parametrize("p_done", [0.0, 0.15, 0.6])
def test_dedup_frames_are_the_stored_observation(p_done):
    T, N, W, F, M, E, nmb = 16, 6, 4, 5, 24, 2, 4
    rng = np.random.default_rng(7)
    obs, dones = _rollout(T, N, W, F, p_done, rng, (rng.random(N) < 0.5).astype(np.float32))
    pl, perm, (uniq, pos_of, inv), cap = _plan(T, N, W, M, E, nmb, rng)
    b_obs = obs[:T].reshape(T * N, W, F)
    for j in range(E * nmb):
        mb = perm[j * M:(j + 1) * M]
        ids = O.slot_frame_ids(mb, dones, N, W)
        assert np.isin(ids, uniq[j][uniq[j] >= 0]).all()  # reset-aware ids within the superset
        x = O.frames_gather(obs, uniq[j])
        h = O.frames_expand(x, pos_of[j], mb, dones, N, W)  # "encoder" = identity
        assert np.array_equal(h, b_obs[mb])


def test_scatter_is_the_adjoint_of_expand():
    """<expand(enc), dh> == <enc, scatter(dh)> on the used rows; padding rows get zeros."""
    T, N, W, F, M, E, nmb = 12, 5, 4, 3, 15, 1, 4
    rng = np.random.default_rng(3)
    _, dones = _rollout(T, N, W, F, 0.3, rng, np.zeros(N, np.float32))
    pl, perm, (uniq, pos_of, inv), cap = _plan(T, N, W, M, E, nmb, rng)
    for j in range(nmb):
        mb = perm[j * M:(j + 1) * M]
        enc = rng.standard_normal((cap, 7)).astype(np.float32)
        dh = rng.standard_normal((M, W, 7)).astype(np.float32)
        h = O.frames_expand(enc, pos_of[j], mb, dones, N, W)
        denc = O.frames_scatter(dh, uniq[j], inv[0], j, dones, T, N, W)
        np.testing.assert_allclose(np.vdot(h.astype(np.float64), dh), np.vdot(enc.astype(np.float64), denc),
                                   rtol=1e-5)
        assert np.all(denc[pl.counts[j]:] == 0)


@pytest.mark.parametrize("M,H,E,W,ok", [
    (4096, 512, 512, 4, True),    # config 2: the gathered decoder runs
    (6144, 512, 512, 3, False),   # a 3-frame stack: no 3-way split combine -> the expand path
    (6144, 512, 512, 2, True),
    (4096, 512, 512, 5, False),
])
def test_decode_gather_gate_only_takes_combinable_stack_widths(M, H, E, W, ok):
    """ocppo_sum_splits_act combines 1/2/4/8/16 splits and the gathered decoder forward runs one
    split per stack slot: any other buffer_window_size must take the _FramesExpand path instead
    of failing inside the update."""
    from oc_cleanrl_amd import frames

    assert frames.decode_gather_shape_ok(M, H, E, W) is ok
