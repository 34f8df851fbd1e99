"""Data-parallel semantics of ppo_atari_multigpu.py:360-377 on CPU with gloo, world_size 2:
the flat-buffer gradient all-reduce (FlatGrads) leaves every rank with the mean gradient and
identical parameters after clip_grad_norm_ + Adam, equal to a single-process run on the mean."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    torch.manual_seed(0)  # identical init on every rank (ppo_atari_multigpu.py:210, 230)
    return nn.Sequential(nn.Linear(6, 16), nn.ReLU(), nn.Linear(16, 3))


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)  # rank-dependent rollout shard
    return torch.randn(32, 6, generator=g), torch.randn(32, 3, generator=g)


def _step(model, flat, x, y, world):
    from oc_cleanrl_amd.trainer import FlatGrads  # noqa: F401

    flat.zero()
    loss = ((model(x) - y) ** 2).mean()
    loss.backward()
    if world > 1:
        flat.allreduce_mean()
    nn.utils.clip_grad_norm_(model.parameters(), 0.5)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oc_cleanrl_amd.trainer import FlatGrads

    model = _model()
    flat = FlatGrads(model.parameters())
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, eps=1e-5)
    for it in range(3):
        x, y = _data(rank * 10 + it)
        _step(model, flat, x, y, world)
        opt.step()
    out[rank] = torch.cat([p.detach().flatten() for p in model.parameters()])
    dist.destroy_process_group()


def test_flat_grads_are_views():
    from oc_cleanrl_amd.trainer import FlatGrads

    m = _model()
    f = FlatGrads(m.parameters())
    from oc_cleanrl_amd.ops import FLAT_ALIGN, flat_offsets

    offs, n = flat_offsets(list(m.parameters()))
    assert f.numel == n and all(o % FLAT_ALIGN == 0 for o in offs)
    ((m(torch.randn(4, 6)) ** 2).sum()).backward()
    for p, o in zip(m.parameters(), offs):
        assert p.grad.data_ptr() == f.buf.data_ptr() + 4 * o
    live = sum(p.numel() for p in m.parameters())
    assert int((f.buf != 0).sum()) <= live  # padding stays zero
    f.zero()
    assert all(float(p.grad.abs().sum()) == 0 for p in m.parameters())


def test_two_rank_gloo_allreduce_matches_single_process():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    p0, p1 = out[0], out[1]
    assert torch.equal(p0, p1), "replicas diverged"
    # single-process reference: mean of the two ranks' grads each step
    from oc_cleanrl_amd.trainer import FlatGrads

    model = _model()
    flat = FlatGrads(model.parameters())
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, eps=1e-5)
    for it in range(3):
        gs = []
        for rank in range(2):
            flat.zero()
            x, y = _data(rank * 10 + it)
            ((model(x) - y) ** 2).mean().backward()
            gs.append(flat.buf.clone())
        flat.buf.copy_((gs[0] + gs[1]) / 2)
        nn.utils.clip_grad_norm_(model.parameters(), 0.5)
        opt.step()
    ref = torch.cat([p.detach().flatten() for p in model.parameters()])
    torch.testing.assert_close(p0, ref, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------------------------------------
# world size 4: the trainer's own exchange (trainer.GradExchange, rank_seeds) on CPU over gloo
# ---------------------------------------------------------------------------------------------
W4 = 4
ENC, DEC = (32, 64, 48), (64,)


def _ppobj_cpu(init_seed):
    from oc_cleanrl_amd.agents import make_agent

    torch.manual_seed(init_seed)
    return make_agent("PPO_OBJ", (4, 6), 6, "cpu", ENC, DEC)


def _tail_off(agent, params):
    """The trainer's cut (PPOTrainer.__init__): the flat offset of the last encoder layer."""
    from oc_cleanrl_amd.ops import flat_offsets

    split = 2 * (len(ENC) - 1)
    first_tail = agent.network[split].weight
    offs, _ = flat_offsets(params)
    return split, next(o for p, o in zip(params, offs) if p is first_tail)


def _shard(stream_seed, it, n=24):
    rng = np.random.RandomState(stream_seed * 100 + it)  # the rank's own env / sample stream
    x = torch.from_numpy(rng.randint(0, 160, (n, 4, 6)).astype(np.float32))
    a = torch.from_numpy(rng.randint(0, 6, n))
    return x, a


def _loss(agent, x, a, split):
    """A PPO-shaped scalar through the network cut at `split` (the trainer's two backward
    phases): returns (loss, low, low_detached)."""
    net = agent.network
    low = net[:split](x)
    low_d = low.detach().requires_grad_()
    h = net[split:](low_d)
    logits, v = agent.actor(h), agent.critic(h).view(-1)
    lp = torch.log_softmax(logits, -1).gather(1, a.view(-1, 1)).view(-1)
    return -(lp * 0.3).mean() + 0.5 * (v ** 2).mean() * 1e-4, low, low_d


def _w4_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oc_cleanrl_amd.trainer import FlatGrads, GradExchange, rank_seeds
    from oracle import ocppo_oracle as O

    init_seed, stream_seed = rank_seeds(42, rank)
    agent = _ppobj_cpu(init_seed)
    flat = FlatGrads(agent.parameters())
    params = flat.params
    split, tail = _tail_off(agent, params)
    out[f"init{rank}"] = torch.cat([p.detach().flatten() for p in params])

    # 1. bookkeeping, bit for bit: dyadic gradients (exact sums in any order) through the split
    #    exchange equal the whole-buffer exchange and the exact sum of every rank's values
    def dyadic(r):
        g = torch.Generator().manual_seed(1000 + r)
        return torch.randint(-512, 512, (flat.numel,), generator=g).float() / 256

    flat.buf.zero_()
    flat.buf[tail:] = dyadic(rank)[tail:]  # phase 1 wrote the tail

    def lower():  # phase 2 writes the head
        flat.buf[:tail] = dyadic(rank)[:tail]

    GradExchange(flat.buf, tail, world, scale_in_optimizer=True).split(lower)
    split_sum = flat.buf.clone()
    flat.buf.copy_(dyadic(rank))
    GradExchange(flat.buf, tail, world, scale_in_optimizer=True).whole()
    exact = sum(dyadic(r) for r in range(world))
    out[f"dyadic{rank}"] = (torch.equal(split_sum, flat.buf), torch.equal(split_sum, exact))
    flat.buf.copy_(dyadic(rank))
    GradExchange(flat.buf, tail, world, scale_in_optimizer=False).whole()
    out[f"mean{rank}"] = torch.equal(flat.buf, exact / world)

    # 2. three DP updates: split exchange, / world folded into clip + Adam (the oracle's
    #    restatement of ocppo_clip_adam_step, grad_scale = 1 / world)
    p = torch.cat([q.detach().flatten() for q in params]).numpy()
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    step = 0
    offs = []
    o = 0
    for q in params:
        offs.append(o)
        o += q.numel()
    from oc_cleanrl_amd.ops import flat_offsets

    foffs, _ = flat_offsets(params)
    for it in range(3):
        flat.zero()
        x, a = _shard(stream_seed, it)
        loss, low, low_d = _loss(agent, x, a, split)
        loss.backward()
        GradExchange(flat.buf, tail, world, scale_in_optimizer=True).split(
            lambda: torch.autograd.backward(low, low_d.grad))
        g = np.concatenate([flat.buf[fo:fo + q.numel()].numpy() for q, fo in zip(params, foffs)])
        p, m, v, step, _ = O.clip_adam_step(p, g, m, v, step, 2.5e-4, grad_scale=1.0 / world)
        with torch.no_grad():
            for q, so in zip(params, offs):
                q.copy_(torch.from_numpy(p[so:so + q.numel()]).view_as(q))
    out[f"params{rank}"] = torch.from_numpy(p.copy())
    dist.destroy_process_group()


def test_four_rank_trainer_exchange_gloo():
    """ppo_atari_multigpu.py:174-183, 208-212, 360-377 at world size 4 with the trainer's own
    GradExchange and rank_seeds: identical init on every rank; the split (tail async, then head)
    exchange equals one whole-buffer all-reduce and the exact sum bit for bit (dyadic values);
    three DP updates leave bit-identical replicas equal (to f32 order) to one process stepping
    on the mean of the four shards' gradients."""
    from oc_cleanrl_amd.trainer import FlatGrads, rank_seeds
    from oracle import ocppo_oracle as O

    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_w4_worker, args=(W4, port, out), nprocs=W4, join=True)
    for r in range(W4):
        assert torch.equal(out[f"init{r}"], out["init0"]), "init must not depend on the rank"
        assert out[f"dyadic{r}"] == (True, True), r
        assert out[f"mean{r}"], r
        assert torch.equal(out[f"params{r}"], out["params0"]), f"replica {r} diverged"
    # single process: the mean of the four shards' gradients, same oracle step
    agent = _ppobj_cpu(rank_seeds(42, 0)[0])
    flat = FlatGrads(agent.parameters())
    params = flat.params
    split, _ = _tail_off(agent, params)
    from oc_cleanrl_amd.ops import flat_offsets

    foffs, _ = flat_offsets(params)
    p = torch.cat([q.detach().flatten() for q in params]).numpy()
    m, v, step = np.zeros_like(p), np.zeros_like(p), 0
    for it in range(3):
        gs = []
        for r in range(W4):
            flat.zero()
            x, a = _shard(rank_seeds(42, r)[1], it)
            loss, low, low_d = _loss(agent, x, a, split)
            loss.backward()
            torch.autograd.backward(low, low_d.grad)
            gs.append(np.concatenate([flat.buf[fo:fo + q.numel()].numpy().astype(np.float64)
                                      for q, fo in zip(params, foffs)]))
        g = (sum(gs) / W4).astype(np.float32)
        p, m, v, step, _ = O.clip_adam_step(p, g, m, v, step, 2.5e-4)
        with torch.no_grad():
            so = 0
            for q in params:
                q.copy_(torch.from_numpy(p[so:so + q.numel()]).view_as(q))
                so += q.numel()
    np.testing.assert_allclose(out["params0"].numpy(), p, rtol=0, atol=0.01 * 2.5e-4)
