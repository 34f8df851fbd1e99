"""`Args` — the flag surface of cleanrl/ppo_atari_oc.py:63-190 (plus the DP fields of
cleanrl/ppo_atari_multigpu.py:55-102) with the same names and defaults, and a tyro-compatible
command line (tyro is not installed here): `--num-envs 8` and `--num_envs 8` both work, booleans
accept `--flag`, `--no-flag` and `--flag True|False`, tuples take several values.

Fields this build adds are grouped at the end and marked "[oc_cleanrl_amd]".
"""
from __future__ import annotations

import argparse
import dataclasses
import os
import sys
from dataclasses import dataclass, field
from typing import Optional

OBS_MODES = (
    "dqn", "obj", "masked_dqn_bin", "masked_dqn_pixels", "masked_dqn_planes",
    "masked_dqn_grayscale", "masked_dqn_pixel_planes", "masked_dqn_parallelplanes",
    "masked_dqn_bin+pixels", "masked_dqn_pixels+pixels", "masked_dqn_planes+pixels",
    "masked_dqn_grayscale+pixels", "masked_dqn_pixel_planes+pixels",
)

# ALE v5 minimal action-set sizes of the games the configs name
ACTION_COUNTS = {"ALE/Pong-v5": 6, "ALE/Breakout-v5": 4, "ALE/SpaceInvaders-v5": 6,
                 "CartPole-v1": 2}


@dataclass
class Args:
    # General (ppo_atari_oc.py:66-74)
    exp_name: str = "ppo_atari_oc"
    seed: int = 42
    torch_deterministic: bool = True
    cuda: bool = True

    # Environment (:77-96)
    env_id: str = "ALE/Pong-v5"
    obs_mode: str = "dqn"
    buffer_window_size: int = 4
    backend: str = "Synthetic"  # reference: OCAtari | HackAtari | Gym (ALE not available here)
    modifs: str = ""
    new_rf: str = ""
    frameskip: int = 4

    # Tracking (:99-116)
    track: bool = False
    wandb_project_name: str = "OCCAM"
    wandb_entity: str = "AIML_OC"
    wandb_dir: Optional[str] = None
    capture_video: bool = False
    ckpt: str = ""
    logging_level: int = 40
    author: str = "JB"
    checkpoint_interval: int = 1_000_000

    # Algorithm (:119-152)
    architecture: str = "PPO"
    total_timesteps: int = 10_000_000
    learning_rate: float = 2.5e-4
    num_envs: int = 10
    num_steps: int = 128
    anneal_lr: bool = True
    gamma: float = 0.99
    gae_lambda: float = 0.95
    num_minibatches: int = 4
    update_epochs: int = 4
    norm_adv: bool = True
    clip_coef: float = 0.1
    clip_vloss: bool = True
    ent_coef: float = 0.01
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    target_kl: Optional[float] = None

    # Transformer parameters (:155-162; those architectures are out of scope, kept for the CLI)
    emb_dim: int = 128
    num_heads: int = 64
    num_blocks: int = 1
    patch_size: int = 12

    # PPObj network (:165-168)
    encoder_dims: tuple = (256, 512, 1024, 512)
    decoder_dims: tuple = (512,)

    # HackAtari / imperfect detection / planes (:171-185)
    test_modifs: str = ""
    detection_failure_probability: float = 0.0
    mislabeling_probability: float = 0.0
    noise_std: float = 0.0
    extra_planes: int = 0
    v2: bool = False

    # runtime (:188-193)
    batch_size: int = 0
    minibatch_size: int = 0
    num_iterations: int = 0
    masked_wrapper: Optional[str] = None
    add_pixels: bool = False

    # data parallelism (ppo_atari_multigpu.py:55-102, 166-173)
    local_num_envs: int = 0  # 0 → num_envs // world_size
    backend_dist: str = "nccl"  # reference flag `--backend` (gloo|nccl|mpi) clashes with the env
    device_ids: tuple = ()      # backend above, hence the rename
    world_size: int = 1
    local_batch_size: int = 0
    local_minibatch_size: int = 0

    # [oc_cleanrl_amd] additions
    num_features: int = 12     # object-vector width F per frame of the synthetic obj env (unpinned
                               # upstream: OCAtari is un-vendored; 12 = x,y,w,h x 3 Pong objects)
    obs_storage: str = "auto"  # rollout obs dtype: auto | f32 | bf16 | u8 (auto = exact & compact)
    cuda_graphs: bool = True   # capture rollout and update into hipGraphs
    vecnorm_reward: bool = True  # VecNormalize(norm_reward=True) of ppo_atari_oc.py:414
    fused_optimizer: bool = True  # HIP clip_grad_norm_ + Adam over flat buffers (else torch's)
    log_dir: str = "runs"
    save_model: bool = True
    metrics_every: int = 1     # read the device-side metrics every N iterations
    rollout_frame_cache: bool = True  # PPO_OBJ rollout: encode only the newest frame per step
    rollout_fusion: bool = True  # PPO_OBJ rollout: store + first encoder layers in one launch,
                                 # cache shift in the last encoder layer's epilogue
    rollout_cache_ring: bool = True  # ... the cache as a ring the decoder reads rotated (no shift)
    update_frame_dedup: bool = True  # PPO_OBJ update: encode each distinct frame of a minibatch once
    prefetch_shuffle: bool = True  # shuffle (+ frame plan) of the next iteration while the GPU runs
    sampling_noise: str = "kernel"  # the rollout sampler's Exp(1) draws: "kernel" = the reference's
                                    # per-step stream (torch's [N, A] exponential_ per step, as
                                    # Categorical.sample draws it), all T steps' draws made by one
                                    # HIP launch at the rollout's start (ops.TorchExpStream.fill);
                                    # "head" = the same stream drawn inside the sampling kernel of
                                    # each step; "torch" = the same stream from torch's
                                    # exponential_ (a launch per step); "rollout" = one [T, N, A]
                                    # draw per rollout (not the reference's stream)
    fused_heads_loss: bool = True  # update: policy heads fwd + PPO loss + heads bwd in one HIP op
    dp_overlap: bool = True  # DP: all-reduce the decoder-side gradients during the encoder backward
    sample_records_min: int = 131072  # local batches of at least this many samples: GAE also
                                      # packs each sample's 16-B record and the minibatch gather
                                      # reads one record instead of five arrays (-1: never).
                                      # It pays at scale (1M samples: GAE + prepare 454 -> 427
                                      # us), not at config 2's 16K (+1-2 us), profiles/r04
    dp_collectives: str = "rccl"  # DP exchange: "rccl" = this package's own RCCL communicator
                                  # (oc_cleanrl_amd.rccl), its all-reduces captured with each
                                  # epoch's minibatches in one hipGraph; "torch" = torch.distributed
                                  # collectives (the only choice on gloo)
    dp_graph_collectives: bool = False  # DP, "torch" collectives: capture each epoch's minibatches
                                        # WITH their all-reduces in one hipGraph (else one graph
                                        # per phase, the collectives launched eagerly between them)
    dist_timeout: float = 300.0  # s: torch.distributed collectives / rendezvous of the DP ranks
    stall_timeout: float = 0.0  # s: > 0 ends a rank whose iteration makes no progress for this
                                # long, naming every rank's phase (oc_cleanrl_amd.watch); 0: off
    dp_exchange: bool = False  # run the DP exchange path (per-minibatch graphs + all-reduce) even
                               # at world size 1, over an initialised 1-rank process group
    conv_channels_last: bool = True  # pixel NatureCNN in NHWC (MIOpen NHWC kernels, no transposes)
    eval_episodes: int = 0  # after training: evaluate() episodes (the reference runs 10 when tracking)
    conv_benchmark: bool = False  # cudnn.benchmark (MIOpen Find) for the NatureCNN convolutions
    gemm_table: bool = True  # the shipped hipBLASLt solution table for the update GEMMs
    x6_gemm: bool = True  # update Linear GEMMs on the bf16 matrix cores as exact-split f32
                          # (ops.gemm_x6, f32 accuracy), ReLU backward fused into the next dX
    x6_weight_planes: bool = True  # ... with the weights split into bf16 planes once per
                                   # minibatch (ops.WeightPlanes; bitwise the same results)


def _flag_names(name: str) -> list[str]:
    names = [f"--{name}"]
    if "_" in name:
        names.append(f"--{name.replace('_', '-')}")
    return names


def _parse_bool(s: str) -> bool:
    if s.lower() in ("1", "true", "yes", "on"):
        return True
    if s.lower() in ("0", "false", "no", "off"):
        return False
    raise argparse.ArgumentTypeError(f"expected a boolean, got {s!r}")


def parse_dataclass(cls, argv=None, defaults: dict | None = None, description: str = ""):
    """tyro-like CLI over the dataclass `cls`. `defaults` overrides its defaults."""
    base = cls(**(defaults or {}))
    ap = argparse.ArgumentParser(description=description)
    tuples = []
    for f in dataclasses.fields(cls):
        cur = getattr(base, f.name)
        names = _flag_names(f.name)
        if isinstance(cur, bool):
            ap.add_argument(*names, dest=f.name, nargs="?", const=True, type=_parse_bool,
                            default=cur)
            ap.add_argument(*[n.replace("--", "--no-", 1) for n in names], dest=f.name,
                            action="store_false")
        elif isinstance(cur, tuple):
            tuples.append(f.name)
            ap.add_argument(*names, dest=f.name, nargs="*", type=int, default=cur)
        elif f.name in ("target_kl",):
            ap.add_argument(*names, dest=f.name, type=lambda s: None if s == "None" else float(s),
                            default=cur)
        elif cur is None:
            ap.add_argument(*names, dest=f.name, type=str, default=cur)
        else:
            ap.add_argument(*names, dest=f.name, type=type(cur), default=cur)
    ns = ap.parse_args(sys.argv[1:] if argv is None else argv)
    d = vars(ns)
    for k in tuples:
        d[k] = tuple(d[k])
    if "obs_mode" in d and d["obs_mode"] not in OBS_MODES:
        ap.error(f"--obs_mode must be one of {OBS_MODES}")
    return cls(**d)


def parse_args(argv=None, defaults: dict | None = None) -> Args:
    """tyro-like CLI over Args. `defaults` overrides dataclass defaults (e.g. per-script)."""
    return parse_dataclass(Args, argv, defaults, "oc_cleanrl_amd PPO (ppo_atari_oc.py surface)")


def finalize(args: Args, world_size: int = 1) -> Args:
    """Derived sizes (ppo_atari_oc.py:344-356; DP: ppo_atari_multigpu.py:166-173)."""
    args.world_size = world_size
    if world_size > 1 or args.local_num_envs:
        if not args.local_num_envs:
            if args.num_envs % world_size:
                raise ValueError(f"num_envs={args.num_envs} is not divisible by {world_size}")
            args.local_num_envs = args.num_envs // world_size
        args.num_envs = args.local_num_envs * world_size
    else:
        args.local_num_envs = args.num_envs
    args.local_batch_size = int(args.local_num_envs * args.num_steps)
    args.local_minibatch_size = int(args.local_batch_size // args.num_minibatches)
    args.batch_size = int(args.num_envs * args.num_steps)
    args.minibatch_size = int(args.batch_size // args.num_minibatches)
    args.num_iterations = args.total_timesteps // args.batch_size
    if "masked" in args.obs_mode:
        raise NotImplementedError("masked_* observation modes need the un-vendored ocatari_wrappers"
                                  " (out of scope); use obs_mode dqn or obj")
    if args.obs_mode == "obj" and args.architecture not in ("PPO_OBJ", "CARTPOLE_MLP"):
        raise AssertionError('"obj" observations only work with "PPO_OBJ" architecture!')
    if args.local_batch_size % args.num_minibatches:
        raise ValueError("local batch size must be divisible by num_minibatches")
    if args.sampling_noise not in ("kernel", "head", "torch", "rollout"):
        raise ValueError(f"sampling_noise must be kernel, head, torch or rollout, got "
                         f"{args.sampling_noise!r}")
    if args.dp_collectives not in ("rccl", "torch"):
        raise ValueError(f"dp_collectives must be rccl or torch, got {args.dp_collectives!r}")
    return args


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment."""
    return (int(os.getenv("RANK", "0")), int(os.getenv("LOCAL_RANK", "0")),
            int(os.getenv("WORLD_SIZE", "1")))
