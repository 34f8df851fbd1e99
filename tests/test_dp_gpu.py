"""The data-parallel trainer path (ppo_atari_multigpu.py semantics) end to end on ONE GPU: two
ranks share cuda:0 and exchange gradients over gloo (RCCL needs distinct devices; the driver runs
the RCCL path at 2/4/8 GPUs). Checks: graphs per minibatch + all-reduce between replays work,
replicas stay bit-identical, and rank-dependent rollouts really differ."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# Config 2 per rank (ppo_atari_oc.py Pong obj, PPObj at the reference's default encoder (256, 512,
# 1024, 512) / decoder (512,), 128 envs x 128 steps, 4 x 4 minibatches of 4096): the network's
# real size, where the update's fused routes engage -- gemm_x6 with the ReLU backward in the next
# dX, the frame-dedup gather / scatter, the first layer's backward in the second layer's dX, the
# heads-loss finish in the decoder's combine. The toy dims reach none of them.
CONFIG2 = dict(num_envs=128, num_steps=128, num_minibatches=4, update_epochs=4,
               encoder_dims=(256, 512, 1024, 512), decoder_dims=(512,))
TOY2 = dict(num_envs=16, num_steps=16, num_minibatches=2, update_epochs=2, encoder_dims=(32, 64),
            decoder_dims=(64,))


def _dp_args(world, dims, **kw):
    from oc_cleanrl_amd.args import Args, finalize

    d = dict(dims)
    d["num_envs"] *= world
    return finalize(Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ",
                         total_timesteps=d["num_envs"] * d["num_steps"] * 10, save_model=False,
                         **d, **kw), world)


class GlooStandIn:
    """rccl.RcclComm's all_reduce_sum over the gloo process group, issued in `stream`'s order:
    drives rccl.RcclExchange's whole / split logic with two ranks holding different buffers."""

    def __init__(self):
        self.calls = []

    def all_reduce_sum(self, t, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        self.calls.append((t.data_ptr(), t.numel(), s == torch.cuda.current_stream(t.device)))
        with torch.cuda.stream(s):
            dist.all_reduce(t, op=dist.ReduceOp.SUM)


def _worker(rank, world, port, out, fused_opt, graphs, overlap=True, dims=None, standin=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oc_cleanrl_amd.trainer import PPOTrainer

    args = _dp_args(world, dims or TOY2, fused_optimizer=fused_opt, cuda_graphs=graphs,
                    dp_overlap=overlap)
    comm = GlooStandIn() if standin else None
    tr = PPOTrainer(args, torch.device("cuda:0"), rank, world, comm=comm)
    assert bool(tr.split) == overlap
    for _ in range(3):
        tr.train_iteration()
    if standin:
        # split form: per minibatch the tail on the side stream, then the head on the main one
        nmb = tr.E * tr.nmb * 3
        n = tr.grad_buf.numel()
        expect = ([(tr.grad_buf[tr.tail_off:].data_ptr(), n - tr.tail_off, False),
                   (tr.grad_buf.data_ptr(), tr.tail_off, True)] if overlap else
                  [(tr.grad_buf.data_ptr(), n, True)])
        assert comm.calls == expect * nmb, (comm.calls[:3], expect)
    torch.cuda.synchronize()
    out[rank] = (torch.cat([p.detach().flatten() for p in tr.agent.parameters()]).cpu(),
                 tr.actions.cpu())
    dist.destroy_process_group()


@pytest.mark.parametrize("fused_opt,graphs", [(True, True), (False, True), (True, False)])
def test_two_ranks_share_one_gpu_over_gloo(fused_opt, graphs):
    mgr = mp.Manager()
    out = mgr.dict()
    port = _port()
    mp.spawn(_worker, args=(2, port, out, fused_opt, graphs), nprocs=2, join=True)
    (p0, a0), (p1, a1) = out[0], out[1]
    assert torch.equal(p0, p1), "DP replicas diverged"
    assert not torch.equal(a0, a1), "ranks must roll out different env shards"


def test_overlapped_exchange_equals_the_whole_buffer_exchange():
    """The split exchange (the tail all-reduced while the lower layers' backward still runs)
    leaves the same parameters as one all-reduce after the whole backward: nothing the lower
    phase writes lies in the tail (a weight gradient deferred across the cut would race its
    all-reduce; encoder_dims (32, 64) puts the cut between the two encoder layers)."""
    res = []
    for overlap in (True, False):
        mgr = mp.Manager()
        out = mgr.dict()
        mp.spawn(_worker, args=(2, _port(), out, True, True, overlap), nprocs=2, join=True)
        res.append(out[0][0])
    assert torch.equal(res[0], res[1])



def _rccl_worker(rank, world, port, out, overlap, graphs, mode="rccl", dims=None, box=True):
    """The RCCL exchange path at world size 1: nccl (= RCCL) process group bound to cuda:0,
    against the plain single-GPU trainer in the same process. mode "rccl": the package's own
    communicator, each epoch's all-reduces captured in its graph (the tail's on a side stream
    during the lower backward); "torch": torch.distributed collectives between per-minibatch
    graphs (async tail all-reduce overlapped with the g_low replay, the head, g_opt);
    "torch-graph": torch's collectives captured with the epoch."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from oc_cleanrl_amd import frames
    from oc_cleanrl_amd.trainer import PPOTrainer

    frames.CUT_CARRIES_BOX = box
    toy = dict(num_envs=32, num_steps=16, num_minibatches=4, update_epochs=2,
               encoder_dims=(32, 64, 48), decoder_dims=(64,))

    def args(dp):
        return _dp_args(1, dims or toy, cuda_graphs=graphs, dp_overlap=overlap, dp_exchange=dp,
                        dp_collectives="rccl" if mode == "rccl" else "torch",
                        dp_graph_collectives=mode == "torch-graph")

    plain = PPOTrainer(args(False), dev)
    for _ in range(3):
        plain.train_iteration()
    torch.cuda.synchronize()
    assert not plain.dp
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    assert dist.get_backend() == "nccl"
    tr = PPOTrainer(args(True), dev)
    assert tr.dp and bool(tr.split) == overlap
    assert (tr.comm is not None) == (mode == "rccl")
    for _ in range(3):
        tr.train_iteration()
    torch.cuda.synchronize()
    if graphs and mode != "torch":
        assert tr.graphs_ready and len(tr.g_update) == tr.E and tr.g_opt is None
    elif graphs:
        assert tr.graphs_ready and len(tr.g_update) == tr.E * tr.nmb and tr.g_opt is not None
        assert len(tr.g_low) == (tr.E * tr.nmb if overlap else 0)
    flat = lambda t: torch.cat([p.detach().flatten() for p in t.agent.parameters()]).cpu()  # noqa
    out["plain"], out["dp"] = flat(plain), flat(tr)
    out["same_actions"] = bool(torch.equal(plain.actions, tr.actions))
    tr.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap,graphs,mode", [
    (True, True, "rccl"), (False, True, "rccl"), (True, False, "rccl"),
    (True, True, "torch"), (False, True, "torch"), (True, False, "torch"),
    (True, True, "torch-graph"), (False, True, "torch-graph")])
def test_rccl_exchange_one_rank_matches_single_gpu(overlap, graphs, mode):
    """ppo_atari_multigpu.py:174-183, 360-377 over RCCL on the one-GPU box: the DP flow with a
    1-rank nccl group leaves parameters bit-identical to the single-GPU trainer after 3
    iterations (SUM over one rank, /1 folded into Adam) -- through the package's own RCCL
    communicator with the all-reduces captured in each epoch's graph (the default), through
    torch's collectives between per-minibatch graphs, and through torch's collectives captured."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_worker, args=(1, _port(), out, overlap, graphs, mode), nprocs=1,
             join=True)
    assert out["same_actions"]
    assert torch.equal(out["plain"], out["dp"]), \
        float((out["plain"] - out["dp"]).abs().max())


@pytest.mark.parametrize("graphs", [True, False])
def test_overlapped_exchange_equals_single_allreduce(graphs):
    """dp_overlap (tail all-reduce during the lower layers' backward, then the head) gives the
    same parameters, bit for bit, as one all-reduce of the whole flat buffer."""
    res = []
    for overlap in (False, True):
        mgr = mp.Manager()
        out = mgr.dict()
        mp.spawn(_worker, args=(2, _port(), out, True, graphs, overlap), nprocs=2, join=True)
        res.append(out[0][0])
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("overlap,graphs,mode", [
    (True, True, "rccl"), (True, False, "rccl"), (True, True, "torch")])
def test_dp_exchange_one_rank_matches_single_gpu_at_config2(overlap, graphs, mode):
    """the N > 1 default (own RCCL communicator, overlap split, captured per
    epoch) at world 1 and config 2's real network size leaves the parameters bit-identical to the
    plain single-GPU trainer after 3 iterations. The cut before the last encoder layer hands the
    layer below its ReLU backward and bias-gradient partials through the box (frames._cut), so
    the split chain runs the same products in the same order as the uncut one."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_worker, args=(1, _port(), out, overlap, graphs, mode, CONFIG2), nprocs=1,
             join=True)
    assert out["same_actions"]
    assert torch.equal(out["plain"], out["dp"]), \
        float((out["plain"] - out["dp"]).abs().max())


@pytest.mark.parametrize("standin", [False, True])
def test_overlapped_exchange_equals_whole_at_config2(standin):
    """Two ranks sharing cuda:0 at config 2 per rank: the split exchange (the tail all-reduced on
    a side stream while the lower encoder layers' backward still runs, then the head) leaves the
    same parameters, bit for bit, as one all-reduce after the whole backward -- on the real x6 /
    frame-dedup routes, where a tail gradient written after its all-reduce was issued would show.
    standin: the exchange is rccl.RcclExchange itself (the N > 1 default's code) over a gloo
    stand-in communicator, so its whole() / split() reduce two different buffers; else torch's
    collectives (trainer.GradExchange)."""
    res = []
    for overlap in (False, True):
        mgr = mp.Manager()
        out = mgr.dict()
        mp.spawn(_worker, args=(2, _port(), out, True, not standin, overlap, CONFIG2, standin),
                 nprocs=2, join=True)
        (p0, a0), (p1, a1) = out[0], out[1]
        assert torch.equal(p0, p1), "DP replicas diverged"
        assert not torch.equal(a0, a1), "ranks must roll out different env shards"
        res.append(p0)
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())


def test_config2_cut_without_the_box_is_not_the_plain_chain():
    """Sensitivity of the test above: with the cut leaf NOT carrying the box (the round-5 form),
    the layer below the cut re-derives its ReLU backward and bias gradient with relu_bias_grad's
    row chunks -- another summation order -- and the config-2 parameters differ from the plain
    chain's after 3 iterations (round 5's checksums 0c39... vs 0ebad...)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_worker, args=(1, _port(), out, True, True, "rccl", CONFIG2, False), nprocs=1,
             join=True)
    assert not torch.equal(out["plain"], out["dp"])
