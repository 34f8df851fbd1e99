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


def _worker(rank, world, port, out, fused_opt, graphs, overlap=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oc_cleanrl_amd.args import Args, finalize
    from oc_cleanrl_amd.trainer import PPOTrainer

    args = finalize(Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ",
                         num_envs=16 * world, num_steps=16, num_minibatches=2, update_epochs=2,
                         total_timesteps=16 * world * 16 * 10, encoder_dims=(32, 64),
                         decoder_dims=(64,), save_model=False, fused_optimizer=fused_opt,
                         cuda_graphs=graphs, dp_overlap=overlap), world)
    tr = PPOTrainer(args, torch.device("cuda:0"), rank, world)
    assert bool(tr.split) == overlap
    for _ in range(3):
        tr.train_iteration()
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
