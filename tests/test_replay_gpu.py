"""Config 5's HBM replay buffer (ops.ReplayBuffer: SB3 ReplayBuffer(optimize_memory_usage=True)
of dqn_atari_oc.py:317-325, add :369, sample :377).

* pinned to the reference-held restatement cleanrl_utils/buffers.py:379-431 (add / sample /
  _get_samples exec'd by tests/golden/gen_golden.py into replay_sb3.npz): the buffer after every
  add (wrap-around, full flag) bit for bit, every sampled transition equal to _get_samples of its
  slot, and the index support of sample() at a not-full and a full state;
* at the config's defining size, 1,000,000 transitions (u8 84x84x4 pixel stacks = 28.2 GB, and
  bf16 object vectors): the wrap of add at the end of the buffer, the (randint(1, size) + pos) %
  size law (never the slot being overwritten, uniform otherwise), [0, pos) before the buffer is
  full, next obs = the next slot's obs."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def test_replay_matches_reference_buffers_py(dev):
    from oc_cleanrl_amd import ops

    z = golden("replay_sb3.npz")
    size = int(z["size"])
    shape = z["in_obs"].shape[2:]
    rb = ops.ReplayBuffer(size, 1, shape, dev, obs_dtype=torch.uint8, seed=5)
    T = lambda a, dt=None: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    supports = {int(k.split("_")[1]): set(z[k].tolist()) for k in z if k.startswith("support_")}
    for t in range(len(z["in_obs"])):
        rb.add(T(z["in_obs"][t]), T(z["in_next_obs"][t]), T(z["in_action"][t].reshape(1)),
               T(z["in_reward"][t]), T(z["in_done"][t]))
        pos, full = rb.state.cpu().tolist()
        assert (pos, bool(full)) == (int(z["after_pos"][t]), bool(z["after_full"][t])), t
        assert np.array_equal(rb.obs.cpu().numpy(), z["after_observations"][t]), t
        assert np.array_equal(rb.actions.cpu().numpy(), z["after_actions"][t][..., 0]), t
        assert np.array_equal(rb.rewards.cpu().numpy(), z["after_rewards"][t]), t
        assert np.array_equal(rb.dones.cpu().numpy(), z["after_dones"][t]), t
        if t in supports:
            seen = set()
            for _ in range(40):
                d = rb.sample(512, with_indices=True)
                seen |= set(d["indices"][:, 0].cpu().tolist())
            assert seen == supports[t], (t, seen, supports[t])
    d = rb.sample(4096, with_indices=True)
    slots = d["indices"][:, 0].cpu().numpy()
    assert np.array_equal(d["indices"][:, 1].cpu().numpy(), np.zeros_like(slots))
    get = {k: z[f"get_{k}"] for k in ("observations", "next_observations", "actions", "rewards",
                                      "dones")}
    np.testing.assert_array_equal(d["observations"].cpu().numpy(),
                                  get["observations"][slots].astype(np.float32))
    np.testing.assert_array_equal(d["next_observations"].cpu().numpy(),
                                  get["next_observations"][slots].astype(np.float32))
    np.testing.assert_array_equal(d["actions"].cpu().numpy(), get["actions"][slots])
    np.testing.assert_array_equal(d["rewards"].cpu().numpy(), get["rewards"][slots])
    np.testing.assert_array_equal(d["dones"].cpu().numpy(), get["dones"][slots])


def _slot_code(i):
    """Three bytes identifying slot i (exact in u8 and bf16)."""
    return torch.stack([i & 255, (i >> 8) & 255, (i >> 16) & 255], 1)


@pytest.mark.parametrize("pixels", [True, False])
def test_replay_one_million_transitions(dev, pixels):
    from oc_cleanrl_amd import ops

    size = 1_000_000
    shape, dt = ((4, 84, 84), torch.uint8) if pixels else ((4, 12), torch.bfloat16)
    rb = ops.ReplayBuffer(size, 1, shape, dev, obs_dtype=dt, seed=11)
    D = rb.D
    assert rb.obs.numel() == size * D and (not pixels or rb.obs.numel() == 28_224_000_000)
    i = torch.arange(size, device=dev)
    flat = rb.obs.view(size, D)
    flat[:, :3] = _slot_code(i).to(dt)
    rb.actions[:, 0] = i % 6
    rb.rewards[:, 0] = (i % 1000).float()
    rb.dones[:, 0] = (i % 7 == 0).float()

    def check(d, pos, full):
        slot = d["indices"][:, 0]
        assert bool((d["indices"][:, 1] == 0).all())
        assert bool((slot >= 0).all()) and bool((slot < size).all())
        if full:
            assert not bool((slot == pos).any())  # the slot being overwritten is never drawn
        else:
            assert bool((slot < pos).all())
        code = d["observations"].flatten(1)[:, :3].long()
        assert torch.equal(code, _slot_code(slot))
        nxt = d["next_observations"].flatten(1)[:, :3].long()
        assert torch.equal(nxt, _slot_code((slot + 1) % size))  # next obs by index
        assert torch.equal(d["actions"][:, 0], slot % 6)
        assert torch.equal(d["rewards"][:, 0], (slot % 1000).float())
        assert torch.equal(d["dones"][:, 0], (slot % 7 == 0).float())
        return slot

    B = 2048 if pixels else 65536
    # not full yet: [0, pos)
    pos = size - 2
    rb.state.copy_(torch.tensor([pos, 0], device=dev))
    check(rb.sample(B, with_indices=True), pos, False)
    # add wraps at the end of the buffer: slot size-2 (obs) / size-1 (next), then size-1 / 0
    mk = lambda v: torch.full((1,) + shape, v, dtype=torch.float32, device=dev).to(  # noqa: E731
        torch.uint8 if pixels else torch.float32)
    one = lambda v, t=torch.float32: torch.tensor([v], dtype=t, device=dev)  # noqa: E731
    rb.add(mk(10), mk(11), one(3, torch.int64), one(0.5), one(0.0))
    assert rb.state.cpu().tolist() == [size - 1, 0]
    rb.add(mk(20), mk(21), one(4, torch.int64), one(-0.5), one(1.0))
    assert rb.state.cpu().tolist() == [0, 1]  # full, pos wrapped to 0
    assert bool((rb.obs[size - 2] == 10).all()) and bool((rb.obs[size - 1] == 20).all())
    assert bool((rb.obs[0] == 21).all())  # transition size-1's next obs lives in slot 0
    assert rb.actions[size - 1, 0].item() == 4 and rb.dones[size - 1, 0].item() == 1.0
    flat[:, :3] = _slot_code(i).to(dt)  # restore the slot codes the adds overwrote
    rb.actions[:, 0] = i % 6
    rb.rewards[:, 0] = (i % 1000).float()
    rb.dones[:, 0] = (i % 7 == 0).float()
    # full: (randint(1, size) + pos) % size, uniform over the other size-1 slots
    pos = 123_457
    rb.state.copy_(torch.tensor([pos, 1], device=dev))
    hist = torch.zeros(64, dtype=torch.int64, device=dev)
    n = 0
    for _ in range(64 if pixels else 4):
        slot = check(rb.sample(B, with_indices=True), pos, True)
        hist += torch.bincount(slot * 64 // size, minlength=64)
        n += B
    h = hist.cpu().numpy() / (n / 64)
    assert h.min() > 0.85 and h.max() < 1.15, h
    del rb
    torch.cuda.empty_cache()
