"""`python -m oc_cleanrl_amd [ppo_atari_oc.py flags]` — the training script.

Single GPU, or one process per GPU under torchrun (ppo_atari_multigpu.py:162-183 semantics:
LOCAL_RANK / WORLD_SIZE from the environment, RCCL via the torch `nccl` backend)."""
from __future__ import annotations

import torch
import torch.distributed as dist

from .args import env_rank, finalize, parse_args
from .trainer import run


def main(argv=None, defaults: dict | None = None):
    args = parse_args(argv, defaults)
    rank, local_rank, world = env_rank()
    args = finalize(args, world)
    if args.device_ids:
        if len(args.device_ids) != world:
            raise SystemExit("you must specify the same number of device ids as `--nproc_per_node`")
        device = torch.device(f"cuda:{args.device_ids[local_rank]}")
    else:
        device = torch.device(f"cuda:{local_rank}")
    torch.cuda.set_device(device)
    if world > 1:
        from datetime import timedelta

        dist.init_process_group(args.backend_dist, timeout=timedelta(seconds=args.dist_timeout),
                                **({"device_id": device} if args.backend_dist == "nccl" else {}))
    tr = None
    try:
        tr = run(args, device, rank, world)
        if rank == 0 and tr.last_metrics:
            print({k: round(v, 5) for k, v in tr.last_metrics.items()})
    finally:
        if tr is not None:
            tr.close()
        if world > 1:
            dist.destroy_process_group()
    return tr


if __name__ == "__main__":
    main()
