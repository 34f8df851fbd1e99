"""The PPO actor-learner: cleanrl/ppo_atari_oc.py:339-729 (and its data-parallel twin
cleanrl/ppo_atari_multigpu.py:162-403) rebuilt around HBM-resident rollout storage, HIP kernels
for the memory-bound glue and hipGraph replay.

One PPO iteration on one GPU (rank):
  rollout graph  : T x [agent fwd (PyTorch GEMMs) → Exp(1) draw → HIP action head (writes
                   actions/logprobs/values rows) → HIP env step → HIP VecNormalize → HIP store
                   (frame stack + bf16/u8 rollout slot + f32 network input + reward/done rows)]
                   → bootstrap value → HIP GAE → HIP minibatch advantage stats
  update graph(s): per minibatch: HIP obs gather (PPObj: distinct frames only) → agent fwd →
                   HIP fused loss fwd+bwd (dlogits, dvalue) → autograd backward of the network
                   into a flat grad buffer → [RCCL all-reduce SUM of the flat buffer, / world;
                   PPObj: the decoder-side tail is reduced while the lower encoder layers run
                   their backward] → clip_grad_norm_ → Adam
One host sync per iteration (metrics), none per step or per minibatch.

Storage layout (step-major like the reference, :452-459): obs [T+1, N, W, ...] in the rollout
dtype (slot T is the next iteration's slot 0), actions [T, N] i64, logprobs/rewards [T, N] f32,
dones/values [T+1, N] f32 (row T = next_done / next_value, the bootstrap of :534).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

from . import agents, frames, gemm_table, ops, rccl
from .rccl import RcclComm, RcclExchange
from .agents import NormalizeImg, PPObj, fused_trunk, linear_relu, make_agent
from .args import Args
from .envs import HostVecEnv, make_device_env


def storage_dtype(args: Args, pixels: bool, integer_obs: bool = True) -> torch.dtype:
    """Rollout obs dtype. `auto` picks the narrowest EXACT type: u8 for ALE pixels, bf16 for the
    synthetic env's integer object coordinates (|x| <= 256), f32 when detection noise makes them
    fractional, for CartPole's state and for host envs, whose feature ranges nothing here pins
    (OCAtari is un-vendored): pass obs_storage="bf16" for a host env known to emit integers
    |x| <= 256."""
    choice = args.obs_storage
    if choice == "auto":
        if pixels:
            return torch.uint8
        return torch.bfloat16 if args.noise_std == 0.0 and integer_obs else torch.float32
    return {"f32": torch.float32, "bf16": torch.bfloat16, "u8": torch.uint8}[choice]


# The rollout's synthetic object-frame env step fused into the policy head's launch
# (ops.policy_head_env_step: bitwise the two-launch step; one launch fewer per env step).
FUSED_HEAD_ENV = True
# The weights' bf16 planes for the next minibatch's GEMMs written by the optimizer step itself
# (ops.FlatAdam.write_planes) instead of a split launch per minibatch. Off: at config 2 nearly
# every parameter has planes (W^T ones among them, scattered 2-B writes from the Adam lanes) and
# the step took 23.9 instead of 12.3 us against the 5.2 us split launch it replaces
# (profiles/r05/breakdown_config2.txt vs the round-4 trace)
ADAM_WRITES_PLANES = False
# The fused heads forward + loss + heads backward (ops.heads_loss_fwd_bwd) also for trunks that
# are not a Linear/ReLU stack (NatureCNN): the grad buffer is zeroed before it, as the unfused
# path does before its backward
FUSED_HEADS_LOSS_ANY_TRUNK = True
# The next iteration's shuffle / frame-plan host-to-device copies on a copy stream of their own
# (PPOTrainer._stage) instead of the compute stream between the update and the next rollout:
# measured slower at config 2 (1,002k vs 1,030k env steps/s in three interleaved pairs: the
# cross-stream event waits cost more than the ~60 us of copies they move off the compute
# stream; profiles/r06/c2_stage_stream/), so off
STAGE_ON_SIDE_STREAM = False
# Pixel trunks: the rollout's first convolution reads the u8 frame stacks of the rollout buffer's
# slot t (agents.trunk_frames: exact bf16 operands, NormalizeImg in the epilogue) instead of the
# f32 network copy the store writes
U8_ROLLOUT_CONV = True


class FlatGrads:
    """All parameter grads as views of ONE persistent f32 buffer: the DP all-reduce is a single
    in-place RCCL call (ppo_atari_multigpu.py:360-374 builds the same flat vector with torch.cat
    and copies it back every minibatch)."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        offs, n = ops.flat_offsets(self.params)
        dev = self.params[0].device
        self.buf = torch.zeros(n, dtype=torch.float32, device=dev)
        for p, off in zip(self.params, offs):
            p.grad = self.buf[off:off + p.numel()].as_strided(p.shape, p.stride())
        self.numel = n

    def zero(self):
        self.buf.zero_()

    def allreduce_mean(self, group=None):
        ws = dist.get_world_size(group)
        dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=group)
        self.buf.div_(ws)


class GradExchange:
    """The data-parallel gradient exchange of ppo_atari_multigpu.py:360-374 on ONE persistent flat
    grad buffer (every parameter's .grad is a view of it): all_reduce(SUM), then / world -- the
    division either here or folded into the optimizer step (FlatAdam's grad_scale), identical on
    every rank.

    split(): the buffer's tail [tail_off:] (the gradients the first backward phase has already
    written) is reduced asynchronously while `lower_backward()` fills the head [:tail_off], then
    the head is reduced and the tail's work awaited. The same SUM of the same bytes as
    whole(); ranks end with identical buffers."""

    def __init__(self, buf, tail_off: int, world: int, scale_in_optimizer: bool, group=None):
        self.buf, self.tail_off, self.world = buf, tail_off, world
        self.scale_in_optimizer, self.group = scale_in_optimizer, group

    def _finish(self):
        if not self.scale_in_optimizer:
            self.buf.div_(self.world)

    def whole(self):
        dist.all_reduce(self.buf, op=dist.ReduceOp.SUM, group=self.group)
        self._finish()

    def split(self, lower_backward):
        work = dist.all_reduce(self.buf[self.tail_off:], op=dist.ReduceOp.SUM, group=self.group,
                               async_op=True)
        lower_backward()
        dist.all_reduce(self.buf[:self.tail_off], op=dist.ReduceOp.SUM, group=self.group)
        work.wait()
        self._finish()


def rank_seeds(seed: int, rank: int) -> tuple[int, int]:
    """(init seed, stream seed) of ppo_atari_multigpu.py:208-212, 230-231: every rank builds the
    network from the same seed, then draws its env / sampling / shuffle streams from seed + rank."""
    return seed, seed + rank


_SCRUB: dict = {}


def l3_scrub(device, mib: int = 640):
    """A launch that streams `mib` MiB through the caches (a sum over a resident buffer, 2.5x the
    256 MiB Infinity Cache): whatever a kernel read before it is no longer cached after it."""
    key = (str(device), mib)
    if key not in _SCRUB:
        _SCRUB[key] = torch.ones(mib << 18, dtype=torch.float32, device=device)
    buf = _SCRUB[key]
    return lambda: buf.sum()


def replay_time_us(fn, reps: int = 64, rounds: int = 5, cold: bool = False) -> float:
    """Mean device time of one launch of the closure `fn`: `reps` back-to-back copies captured
    into one hipGraph, timed with HIP events over `rounds` replays (includes the ~1 us graph-node
    gap per launch). cold=True puts an L3 scrub (l3_scrub) before every copy and subtracts the
    same graph of scrubs alone (min over rounds of each), so every launch reads its operands
    from HBM: the figure an HBM roofline fraction may be quoted on."""
    def graph_of(body):
        g = torch.cuda.CUDAGraph()
        with _graph_capture(g):
            for _ in range(reps):
                body()
        g.replay()
        return g

    def timed(g):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    fn()
    torch.cuda.synchronize()
    if not cold:
        g = graph_of(fn)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(rounds):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        return 1e3 * a.elapsed_time(b) / (reps * rounds)
    scrub = l3_scrub(torch.device("cuda", torch.cuda.current_device()))

    def both():
        scrub()
        fn()

    g1, g0 = graph_of(both), graph_of(scrub)
    t1, t0 = [], []
    for _ in range(rounds):
        t1.append(timed(g1))
        t0.append(timed(g0))
    return 1e3 * max(min(t1) - min(t0), 0.0) / reps


class KernelTimer:
    """Per-launch device durations of this package's HIP kernels.

    On ROCm an event cannot be recorded inside a captured graph (torch rejects external events;
    hipEventRecordWithFlags(.., hipEventRecordExternal) returns hipErrorInvalidValue during
    capture), so the timed region itself cannot be bracketed per kernel. Instead every bracketed
    launch site keeps the closure of its first eager launch (same buffers, same stream) and
    `measure()` replays copies of exactly that launch (replay_time_us): warm (back to back, the
    operands cache-resident) for every site, and cold (an L3 scrub before every copy) for the
    sites named in `cold` -- the HBM-bound kernels, whose roofline fraction must not be quoted on
    Infinity-Cache hits. Cross-checked against rocprofv3 --kernel-trace in profiles/."""

    def __init__(self, enabled: bool):
        self.enabled = enabled
        self.sites: dict = {}
        self.per_iter: dict = {}
        self._counting = True
        self.mean_us: dict = {}
        self.cold_us: dict = {}

    def bracket(self, name, fn):
        if self.enabled and not (torch.cuda.is_available() and
                                 torch.cuda.is_current_stream_capturing()):
            self.sites.setdefault(name, fn)
            if self._counting:
                self.per_iter[name] = self.per_iter.get(name, 0) + 1
        return fn()

    def end_iteration(self):
        self._counting = False

    def measure(self, reps: int = 64, rounds: int = 5, cold=()) -> dict:
        for name, fn in self.sites.items():
            self.mean_us[name] = replay_time_us(fn, reps, rounds)
            if name in cold:
                self.cold_us[name] = replay_time_us(fn, 16, rounds, cold=True)
        return self.mean_us


def _quiesce_rccl():
    """Wait until the RCCL process group's watchdog holds no work of earlier eager collectives:
    a captured collective joins RCCL's stream into the capture, and the watchdog's hipEventQuery
    on an older work's event recorded on that stream then fails with hipErrorCapturedEvent and
    terminates the process (seen once at world 1 with the epoch's all-reduces captured,
    tests/test_dp_gpu.py). ProcessGroup._wait_for_pending_works is ProcessGroupNCCL's hook for
    exactly this; other backends have no watchdog events."""
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        dist.distributed_c10d._get_default_group()._wait_for_pending_works()


def _graph_capture(graph, pool=None, quiesce: bool = False):
    """hipGraph capture in thread-local mode: the RCCL process group's watchdog thread polls its
    work events (hipEventQuery) while this thread captures, which global-mode capture turns into
    hipErrorStreamCaptureUnsupported and a process abort (seen once in 3 runs of the 1-rank nccl
    test, tests/test_dp_gpu.py). Only this thread's calls are restricted, as they must be.
    quiesce: the capture will issue torch.distributed collectives (dp_collectives="torch" with
    dp_graph_collectives), which join the process group's stream: wait for its older work first
    (_quiesce_rccl). The package's own communicator (oc_cleanrl_amd.rccl) needs none of this."""
    if quiesce:
        _quiesce_rccl()
    return torch.cuda.graph(graph, pool=pool, capture_error_mode="thread_local")


class PPOTrainer:
    def __init__(self, args: Args, device, rank: int = 0, world_size: int = 1,
                 kernel_timing: bool = False, log: bool = True, envs=None, comm=None):
        """envs: optional host (CPU) gymnasium-style vector env of this rank's local_num_envs
        (envs.HostVecEnv documents the contract); None = the device-resident synthetic env.
        comm: the DP exchange's communicator in place of the package's own RCCL one -- any object
        with rccl.RcclComm's all_reduce_sum(t, stream) (tests drive rccl.RcclExchange's whole /
        split logic over several ranks with a gloo-backed stand-in; its collectives are not
        capturable, so such a trainer runs with cuda_graphs off)."""
        self.args = args
        self.dev = torch.device(device)
        self.rank, self.world = rank, world_size
        # the DP exchange path (per-minibatch graphs around an all-reduce of the flat grad buffer);
        # at world size 1 only on request (dp_exchange), over an initialised 1-rank group
        self.dp = world_size > 1 or (args.dp_exchange and dist.is_available()
                                     and dist.is_initialized())
        # the exchange's own RCCL communicator (oc_cleanrl_amd.rccl) over an nccl process group:
        # its all-reduces are captured with each epoch's minibatches; a side stream carries the
        # tail's all-reduce while the lower encoder layers run their backward
        self.comm = self.side = None
        self.dp_form = None  # the exchange actually in use (bench.py reports it)
        if self.dp and comm is not None:
            if args.cuda_graphs:
                raise ValueError("an injected DP communicator runs with cuda_graphs off")
            self.comm, self.dp_form = comm, f"rccl.RcclExchange over {type(comm).__name__}"
            self.side = torch.cuda.Stream(device)
        elif (self.dp and args.dp_collectives == "rccl" and torch.device(device).type == "cuda"
                and dist.get_backend() == "nccl"):
            torch.cuda.set_device(device)
            self.comm, self.dp_form = self._rccl_comm(rank, dist.get_world_size(), device)
            if self.comm is not None:
                self.side = torch.cuda.Stream(device)
        if self.dp and self.dp_form is None:
            self.dp_form = "torch collectives"
        self.log_enabled = log and rank == 0
        a = args
        if envs is None and a.backend != "Synthetic":
            raise NotImplementedError(f"env backend {a.backend!r} needs ALE/OCAtari (not available);"
                                      " use --backend Synthetic")
        torch.use_deterministic_algorithms(a.torch_deterministic)
        # deterministic mode also NaN-fills every torch.empty (a debugging aid: ~300 fill launches per
        # iteration here); nothing reads uninitialised memory, so results are unaffected
        torch.utils.deterministic.fill_uninitialized_memory = False
        torch.backends.cudnn.deterministic = a.torch_deterministic
        torch.backends.cudnn.benchmark = a.conv_benchmark
        self.gemm_table = a.gemm_table and gemm_table.use(device)

        # seeding as ppo_atari_multigpu.py:208-212, 230-231: identical init on every rank, then
        # rank-dependent sampling / env / shuffle streams
        init_seed, self.seed = rank_seeds(a.seed, rank)
        self.np_rng = np.random.RandomState(self.seed)  # np.random.shuffle stream of :561
        torch.manual_seed(init_seed)

        self.N = a.local_num_envs
        self.T = a.num_steps
        self.host_env = envs is not None
        if self.host_env:
            self.env = HostVecEnv(envs, a.env_id, a.obs_mode, self.N, self.seed, self.dev,
                                  a.buffer_window_size)
            self.env.reset()  # the obs shape comes from the env
        else:
            self.env = make_device_env(a.env_id, a.obs_mode, self.N, a.num_features, self.seed,
                                       self.dev, a.buffer_window_size)
        self.pixels = self.env.pixels
        # a host env's reset observations are its own stacks (envs.HostVecEnv): the stored obs no
        # longer follow the frame-stack fill rule the rollout frame cache and the update's frame
        # dedup rely on, so both use the plain (every slot encoded) path then
        self.reset_stacks = self.host_env and self.env.reset_stacks
        self.A = self.env.n_actions
        self.obs_shape = self.env.single_obs_shape
        self.agent = make_agent(a.architecture, self.obs_shape, self.A, self.dev, a.encoder_dims,
                                a.decoder_dims).to(self.dev)
        # this agent's update-GEMM route (gemm_x6 or hipBLASLt): per-agent state, not a global
        agents.set_update_gemm(self.agent, a.x6_gemm)
        # NatureCNN in channels_last: MIOpen runs its NHWC kernels without transposing every
        # activation; the HIP store/gather kernels write the network input in NHWC directly
        self.channels_last = (a.conv_channels_last and self.pixels and len(self.obs_shape) == 3
                              and any(isinstance(m, nn.Conv2d) for m in self.agent.modules()))
        self.net_format = torch.channels_last if self.channels_last else torch.contiguous_format
        if self.channels_last:
            self.agent = self.agent.to(memory_format=torch.channels_last)
        # ... and its NormalizeImg (x / 255) folded into those HIP writes
        net0 = self.agent.network[0] if isinstance(self.agent.network, nn.Sequential) else None
        self.prescale = self.channels_last and isinstance(net0, NormalizeImg)
        torch.manual_seed(self.seed)
        self.fused_head = isinstance(self.agent.actor, nn.Linear) and \
            isinstance(self.agent.critic, nn.Linear)
        self.H = self.agent.actor.in_features if self.fused_head else 0
        # PPObj's encoder sees one frame at a time: the rollout keeps the W frame encodings of
        # every env in a cache and encodes only the newest frame per step
        self.frame_cache = (a.rollout_frame_cache and self.fused_head and not self.reset_stacks and
                            isinstance(self.agent, PPObj) and len(a.encoder_dims) > 0)
        # every parameter's grad is written in place by agents._LinearAct (no zero-fill needed)
        # when the agent is a Linear/ReLU stack owned by the fused optimizer
        self.direct_grads = a.fused_optimizer and self.fused_head and all(
            isinstance(m, (nn.Linear, nn.ReLU, nn.Flatten)) for m in self.agent.network)
        if a.fused_optimizer:
            # every parameter becomes a view of one flat buffer; clip + Adam = 2 HIP launches
            self.optimizer = ops.FlatAdam(self.agent.parameters(), lr=a.learning_rate, eps=1e-5,
                                          max_grad_norm=a.max_grad_norm)
            self.params = self.optimizer.param_list
            self.grad_buf = self.optimizer.grads
            self.lr = self.optimizer.lr
        else:
            grads = FlatGrads(self.agent.parameters())
            self.params = grads.params
            self.grad_buf = grads.buf
            self.lr = torch.tensor(a.learning_rate, dtype=torch.float32, device=self.dev)
            self.optimizer = torch.optim.Adam(self.params, lr=self.lr, eps=1e-5, fused=True,
                                              capturable=True)

        T, N = self.T, self.N
        f32 = torch.float32
        dev = self.dev
        self.obs_dtype = storage_dtype(a, self.pixels, not self.host_env and
                                       getattr(self.env, "integer_obs", False))
        self.obs = torch.zeros((T + 1, N) + self.obs_shape, dtype=self.obs_dtype, device=dev)
        self.net_obs = torch.empty((N,) + self.obs_shape, dtype=f32, device=dev,
                                   memory_format=self.net_format).zero_()
        self.actions = torch.zeros((T, N), dtype=torch.int64, device=dev)
        self.logprobs = torch.zeros((T, N), dtype=f32, device=dev)
        self.rewards = torch.zeros((T, N), dtype=f32, device=dev)
        self.dones = torch.zeros((T + 1, N), dtype=f32, device=dev)
        self.values = torch.zeros((T + 1, N), dtype=f32, device=dev)
        self.advantages = torch.zeros((T, N), dtype=f32, device=dev)
        self.returns = torch.zeros((T, N), dtype=f32, device=dev)
        # the Exp(1) draws torch's Categorical.sample makes ([N, A] per step): by default the
        # rollout's T draws of the reference's stream drawn by one launch at its start as torch's
        # exponential_ would (ops.TorchExpStream.fill), or inside the sampling kernel step by step
        # ("head"); or torch's exponential_ per step / per rollout (Args.sampling_noise)
        self.noise = torch.zeros((T, N, self.A), dtype=f32, device=dev)
        self.exp_stream = (ops.TorchExpStream(N * self.A, dev)
                           if a.sampling_noise in ("kernel", "head") else None)
        self.enc_cache = (torch.zeros((N, self.obs_shape[0], self.agent.encoding_dim), dtype=f32,
                                      device=dev) if self.frame_cache else None)
        # frame cache + fusions: the store of step t-1 rides in the launch of step t's first two
        # encoder layers, the last encoder layer shifts the cache in its epilogue
        self.rollout_fusion = self.frame_cache and a.rollout_fusion and self._fusable_encoder()
        self.enc_pair = (torch.zeros((N, self.agent.network[2].out_features), dtype=f32, device=dev)
                         if self.rollout_fusion else None)
        # ... and the cache is a ring (no shift): step t writes the newest encoding over the oldest
        # (physical slot (t-1) mod W) and the decoder's first layer reads the slots rotated by
        # t mod W (ocppo_linear_cache_ring / ocppo_linear_act_ring), bit-identical to the shift
        self.cache_ring = self.rollout_fusion and a.rollout_cache_ring and self._ring_decoder()
        self.ret_state = torch.zeros(N, dtype=torch.float64, device=dev)
        self.rms_state = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=dev)

        # update-phase buffers
        self.B = a.local_batch_size
        self.M = a.local_minibatch_size
        self.E = a.update_epochs
        self.nmb = a.num_minibatches
        self.b_inds = np.arange(self.B)
        self.perm_host = torch.empty(self.E * self.B, dtype=torch.int64, pin_memory=True)
        self.perm_dev = torch.zeros(self.E * self.B, dtype=torch.int64, device=dev)
        # the next iteration's shuffle is drawn and copied while the GPU runs this one; it lands
        # in perm_stage and is moved into perm_dev (which the graphs read) at iteration start
        self.perm_stage = torch.zeros_like(self.perm_dev)
        self.staged = False
        self.staged_rng_state = self.current_rng_state = None
        self.executed_mb = self.E * self.nmb  # minibatches the last update ran (target_kl)
        # train_iteration(lag=True): the pending record and two pinned host vectors used in turn
        # (a new copy never lands in the vector the pending record still has to be read from)
        self._pending_metrics, self._metrics_host, self._metrics_turn = None, [None, None], 0
        self.perm_event = torch.cuda.Event()
        self.perm_event.record()
        # the staging copies (host -> perm_stage / plan_stage) on a stream of their own, so they
        # run beside this iteration's update instead of between it and the next rollout; they
        # wait for the previous iteration's reads of the stage (stage_read), and the next
        # iteration's moves out of the stage wait for them (perm_event)
        self.copy_stream = (torch.cuda.Stream(dev) if STAGE_ON_SIDE_STREAM and
                            torch.device(dev).type == "cuda" else None)
        self.stage_read = torch.cuda.Event()
        # PPObj update with every distinct frame of a minibatch encoded once (frames.py)
        W = self.obs_shape[0]
        self.frame_dedup = (a.update_frame_dedup and isinstance(self.agent, PPObj) and
                            not self.reset_stacks and
                            not self.pixels and len(self.obs_shape) == 2 and
                            len(a.encoder_dims) > 0 and 1 <= W <= 16)
        self.planner = (frames.FramePlanner(T, N, W, a.local_minibatch_size, a.update_epochs,
                                            a.num_minibatches) if self.frame_dedup else None)
        self.plan_host = self.plan_stage = self.plan_dev = self.plan = None
        # DP: cut the backward before the last encoder layer, so the all-reduce of the flat
        # buffer's tail (last encoder layer + decoder + heads, ~70 % of the bytes for PPObj)
        # overlaps the backward of the layers below (_exchange)
        self.split, self.tail_off, self.cuts = 0, 0, {}
        if self.dp and a.dp_overlap and self.frame_dedup and len(a.encoder_dims) >= 2:
            self.split = 2 * (len(a.encoder_dims) - 1)  # network[:split] = the layers below
            first_tail = self.agent.network[self.split].weight
            offs, _ = ops.flat_offsets(self.params)
            self.tail_off = next(o for p, o in zip(self.params, offs) if p is first_tail)
            assert self.grad_buf[self.tail_off:].data_ptr() == first_tail.grad.data_ptr()
        nmbt = self.E * self.nmb
        self.mb = {"actions": torch.zeros(nmbt * self.M, dtype=torch.int64, device=dev),
                   **{k: torch.zeros(nmbt * self.M, dtype=f32, device=dev)
                      for k in ("logprobs", "advantages", "returns", "values")},
                   "adv_stats": torch.zeros((nmbt, 2), dtype=f32, device=dev)}
        self.mb_obs = torch.empty((self.M,) + self.obs_shape, dtype=f32, device=dev,
                                  memory_format=self.net_format).zero_()
        self.dlogits = torch.zeros((self.M, self.A), dtype=f32, device=dev)
        self.dvalue = torch.zeros(self.M, dtype=f32, device=dev)
        self.stats = torch.zeros((self.E * self.nmb, len(ops.STAT_NAMES)), dtype=f32, device=dev)
        self.loss_ws = ops.LossWorkspace(self.M, self.A, dev)
        # heads forward + loss + heads backward fused on the decoder output (needs the in-place
        # grads of FlatAdam and the decoder's ReLU box; see _fused_tail)
        # (FlatAdam's in-place grads; a trunk that is not a Linear/ReLU stack, e.g. NatureCNN,
        # gets the grad buffer zeroed first, _fused_tail)
        self.fused_heads_loss = (a.fused_heads_loss and a.fused_optimizer and self.fused_head and
                                 self.H in ops.HEADS_LOSS_WIDTHS and self.A <= 7 and
                                 (self.direct_grads or FUSED_HEADS_LOSS_ANY_TRUNK))
        self.gp_tail = (torch.empty((self.M, self.H), dtype=f32, device=dev)
                        if self.fused_heads_loss else None)
        self.hl_finish = ops.DeferredFinish(dev) if self.fused_heads_loss else None
        self.b_obs = self.obs[:T].view((T * N,) + self.obs_shape)
        # pixel trunks: the update's first convolution reads the u8 frame stacks itself
        self.u8_first_conv = (not self.frame_dedup and self.b_obs.dtype == torch.uint8 and
                              self.prescale and hasattr(self.agent, "trunk_frames_ok") and
                              self.agent.trunk_frames_ok(self.b_obs, self.M))
        # ... and so does the rollout's, from slot t of the rollout buffer (no f32 stack read)
        self.u8_rollout = (U8_ROLLOUT_CONV and self.u8_first_conv and not self.frame_cache and
                           self.agent.trunk_frames_ok(self.obs[0], self.N))
        self.env_rows = torch.arange(self.N, dtype=torch.int64, device=dev)
        # the store's f32 network copy of the stacks: nothing reads it on the u8 rollout path
        self._store_net = None if self.u8_rollout else self.net_obs
        self.wplanes, self.wplanes_built = None, False  # built at the first minibatch
        self.planes_by_opt = False
        # GAE's per-sample records for the minibatch gather (ops.sample_records)
        self.records = (ops.sample_records(self.B, dev)
                        if 0 <= a.sample_records_min <= self.B else None)

        # Every update is captured, the NatureCNN's MIOpen convolutions included (round 1 ran that
        # one eagerly after a capture_end crash that no longer reproduces: tools/exp_c3_capture.py
        # captures and replays it at 16 and 256 envs, deterministic or not, NHWC or NCHW,
        # profiles/r02/c3_capture.log)
        self.graph_update = a.cuda_graphs
        # DP: the all-reduces inside the per-epoch update graphs (own communicator, or torch's
        # collectives captured on request), else eager between per-phase graphs
        self.captured_exchange = self.dp and (self.comm is not None or a.dp_graph_collectives)
        self.quiesce = self.dp and self.comm is None and a.dp_graph_collectives
        self.timer = KernelTimer(kernel_timing)
        if kernel_timing:
            ops.TIMER = self.timer  # launch sites inside autograd (relu_bias_grad, frames_*)
        self.graphs_ready = False
        self.g_rollout = None
        self.g_update: list = []
        self.g_low: list = []
        self.g_host: list = []
        self.g_opt = None
        self.iteration = 0
        self.global_step = 0
        self.last_metrics: dict = {}
        self._reset_env()

    def _weight_planes(self):
        """ops.WeightPlanes of the PPObj Linear weights whose update forward / dX run on gemm_x6
        where the pre-split B pays (measured at config 2, profiles/r04/planes_ab.txt): the mixed
        128 x 128 / 64 x 128 tiles and the 4096-row decoder dX gain 2-7 us per product, the
        720-tile [11520 x 1024] products lose 4-7 us (their extra B bytes per step), so those keep
        the in-kernel split. Built at the first minibatch (the frame-dedup capacity, the rows the
        encoder sees, is known by then); None when no product qualifies."""
        a, ag = self.args, self.agent
        if (a.x6_weight_planes and agents.CONV_X6_PLANES and self.dev.type == "cuda" and
                self.pixels and isinstance(getattr(ag, "network", None), nn.Sequential)):
            # NatureCNN: the convolutions after the first (which reads the u8 stacks) take their
            # weight's [Cout, KH KW C] matrix pre-split (ocppo_conv_x6 w_planes)
            views = []
            convs = [m for m in ag.network if isinstance(m, nn.Conv2d)]
            for m in convs[1:]:
                w = m.weight
                v = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
                if w.is_cuda and v.data_ptr() == w.data_ptr() and v.is_contiguous() and \
                        v.shape[1] % 8 == 0:
                    views.append((w, v))
            if not views:
                return None
            wp = ops.WeightPlanes(fwd=[v for _, v in views])
            for w, v in views:
                w._ocppo_planes = v._ocppo_planes
            return wp
        if not (a.x6_gemm and a.x6_weight_planes and isinstance(ag, PPObj) and self.dev.type == "cuda"):
            return None
        enc_rows = self.planner.cap if self.frame_dedup else self.M * self.obs_shape[0]

        def pays(rows, n, k):
            t = ops.x6_tile(rows, n)
            return (agents._x6(rows, n, k) and k % 32 == 0 and t is not None
                    and (t == ops.X6_MIXED or rows <= 4096))

        fwd, dx = [], []
        for i, m in enumerate(ag.network):
            if not isinstance(m, nn.Linear) or i == 0:
                continue
            rows = enc_rows if i < ag._flat else self.M
            if pays(rows, m.out_features, m.in_features) or (
                    agents.X6_FWD_SPLITK and m.in_features % 32 == 0 and
                    ops.x6_fwd_splits(rows, m.out_features, m.in_features) is not None):
                fwd.append(m.weight)
            # (the decoder's dX planes only where measured to pay: frames.DECODE_DX_PLANES)
            if pays(rows, m.in_features, m.out_features) and (i < ag._flat or
                                                              frames.DECODE_DX_PLANES):
                dx.append(m.weight)
        return ops.WeightPlanes(fwd, dx) if fwd or dx else None

    def _fusable_encoder(self) -> bool:
        """PPObj encoder shapes the fused rollout kernels take: >= 3 Linear+ReLU layers, the first
        two within ocppo_store_linear2's limits, f32 object frames, f32 / bf16 storage."""
        net = self.agent.network
        lins = [m for m in net[:self.agent._flat] if isinstance(m, nn.Linear)]
        if len(lins) < 3 or self.pixels or self.env.frame_dtype != torch.float32 or \
                self.obs_dtype not in (torch.float32, torch.bfloat16) or self.channels_last:
            return False
        acts = list(net[:self.agent._flat])
        if not all(isinstance(acts[i], nn.ReLU) for i in range(1, len(acts), 2)):
            return False
        l1, l2 = lins[0], lins[1]
        return (l1.in_features <= 64 and l1.out_features % 16 == 0 and l1.out_features <= 512
                and l2.weight.data_ptr() % 16 == 0 and all(m.bias is not None for m in lins))

    def _ring_decoder(self) -> bool:
        """The decoder's first layer (after the Flatten) is a biased Linear+ReLU that the ring
        kernel takes (K = W*E, E a power of two >= 32) at a batch where it runs on the HIP path
        anyway."""
        net, f = self.agent.network, self.agent._flat
        if len(net) < f + 3 or not isinstance(net[f + 1], nn.Linear) or \
                not isinstance(net[f + 2], nn.ReLU) or net[f + 1].bias is None:
            return False
        E, K = self.agent.encoding_dim, net[f + 1].in_features
        return (E >= 32 and E & (E - 1) == 0 and K == self.obs_shape[0] * E and self.N <= 128
                and K <= 2048)

    def _decode_cache(self, t: int):
        """Decoder output on the frame-encoding cache at rollout step t."""
        ag = self.agent
        if not self.cache_ring:
            return ag.decode(self.enc_cache)
        net, f = ag.network, ag._flat
        W, E = self.enc_cache.shape[1], self.enc_cache.shape[2]
        lin = net[f + 1]
        h = self.timer.bracket("decoder", lambda: ops.linear_act(
            self.enc_cache.view(self.N, W * E), lin.weight, lin.bias, True, ring=(E, t % W)))
        rest = net[f + 3:]
        return fused_trunk(rest, h) if len(rest) else h

    def cache_logical(self, t: int):
        """The cache in logical slot order (oldest .. newest) at rollout step t (tests)."""
        if not self.cache_ring:
            return self.enc_cache
        return torch.roll(self.enc_cache, -(t % self.enc_cache.shape[1]), dims=1)

    # ------------------------------------------------------------------------------------------
    def _reset_env(self):
        frame = self.env.frame if self.host_env else self.env.reset()
        if self.reset_stacks:  # the env's own initial stack (envs.HostVecEnv.reset)
            ones = torch.ones(self.N, dtype=torch.float32, device=self.dev)
            ops.rollout_store(frame, ones, ones, self.obs[0], self.obs[self.T], self._store_net,
                              scale255=self.prescale, reset_prev=self.env.reset_prev)
        else:
            ops.obs_reset(frame, self.obs[self.T], self._store_net, scale255=self.prescale)
        self.dones[self.T].zero_()

    def _policy_hidden(self, t: int):
        """Trunk output for net_obs at rollout step t (t == T: the bootstrap of :534). With the
        frame cache: step 0 encodes all W frames (the weights changed since the last rollout),
        later steps encode only the newest frame and shift the cache with done row t."""
        if not self.frame_cache:
            if self.u8_rollout:  # the first convolution reads slot t's u8 stacks itself
                return self.agent.trunk_frames(self.obs[t], self.env_rows)
            return self.agent.trunk(self.net_obs, self.prescale)
        self._policy_encode(t)
        return self._decode_cache(t)

    def _policy_encode(self, t: int):
        """The frame-encoding cache at rollout step t (see _policy_hidden)."""
        ag = self.agent
        if t == 0:
            self.enc_cache.copy_(ag.encode(self.net_obs))  # logical order: ring offset 0
        elif self.rollout_fusion:
            self._store_encode(t)
        else:
            fresh = ag.encode(self.net_obs[:, -1])
            self.timer.bracket("frame_cache", lambda: ops.frame_cache_shift(
                self.enc_cache, fresh, self.dones[t]))

    def _store_encode(self, t: int):
        """Store of step t-1 + encode of step t's newest frame into the cache, in 2 + (encoder
        depth - 3) launches (ops.store_linear2, middle layers, ops.linear_cache_shift)."""
        a, env, net = self.args, self.env, self.agent.network
        lins = [m for m in net[:self.agent._flat] if isinstance(m, nn.Linear)]
        vn = (self.ret_state, self.rms_state) if a.vecnorm_reward else None
        self.timer.bracket("store_encode", lambda: ops.store_linear2(
            env.frame, env.reward, env.done, self.obs[t - 1], self.obs[t], self.net_obs,
            self.dones[t], self.rewards[t - 1], lins[0].weight, lins[0].bias, lins[1].weight,
            lins[1].bias, self.enc_pair, vecnorm_state=vn))
        x = self.enc_pair
        for i, lin in enumerate(lins[2:-1]):
            x = self.timer.bracket("encoder_mid" if i == 0 else f"encoder_mid{i}",
                                   lambda x=x, lin=lin: linear_relu(x, lin))
        last = lins[-1]
        if self.cache_ring:
            W = self.enc_cache.shape[1]
            self.timer.bracket("cache_linear", lambda: ops.linear_cache_ring(
                x, last.weight, last.bias, self.enc_cache, (t - 1) % W, self.dones[t]))
        else:
            self.timer.bracket("cache_linear", lambda: ops.linear_cache_shift(
                x, last.weight, last.bias, self.enc_cache, self.dones[t]))

    def _rollout_step(self, t: int):
        """One env step of the rollout (:500-514): network trunk (PyTorch) → fused HIP policy
        head (actor+critic GEMVs + Categorical sample, writes actions/logprobs/values rows) →
        env → fused HIP store (+ VecNormalize) of the next obs slot and reward/done rows. With
        the synthetic object-frame env the env step rides in the head's launch
        (ops.policy_head_env_step)."""
        if not self._act(t, env_step=True):
            self.timer.bracket("env_step", lambda: self.env.step(self.actions[t], t))
        if not self.rollout_fusion:  # else the store rides in step t+1's encoder launch
            self._store(t)

    def _act(self, t: int, env_step: bool = False) -> bool:
        """Actions / log-probs / values of step t; True when the env step ran too."""
        ag = self.agent
        if self.args.sampling_noise == "torch":
            # the reference's stream: one Exp(1) draw of [N, A] per step (Categorical.sample at
            # ppo_atari_oc.py:506), from the same device generator
            self.noise[t].exponential_()
        px = self.exp_stream.philox(t) if self.args.sampling_noise == "head" else None
        if self.fused_head:
            hidden = self._policy_hidden(t)
            if env_step and FUSED_HEAD_ENV and ops.policy_head_env_ok(
                    hidden, ag.actor.weight, ag.critic.weight, self.env):
                self.timer.bracket("action_head_env", lambda: ops.policy_head_env_step(
                    hidden, ag.actor.weight, ag.actor.bias, ag.critic.weight, ag.critic.bias,
                    self.noise[t], self.actions[t], self.logprobs[t], self.values[t], self.env,
                    t, philox=px))
                return True
            self.timer.bracket("action_head", lambda: ops.policy_head_sample(
                hidden, ag.actor.weight, ag.actor.bias, ag.critic.weight, ag.critic.bias,
                self.noise[t], self.actions[t], self.logprobs[t], self.values[t], philox=px))
        else:
            logits, value = (ag.heads(ag.trunk_frames(self.obs[t], self.env_rows))
                             if self.u8_rollout else ag.logits_and_value(self.net_obs, self.prescale))
            self.timer.bracket("action_head", lambda: ops.categorical_sample(
                logits, self.noise[t], self.actions[t], self.logprobs[t], None, value.view(-1),
                self.values[t], philox=px))
        return False

    def _store(self, t: int):
        a = self.args
        rp = self.env.reset_prev if self.reset_stacks else None
        if a.vecnorm_reward:
            self.timer.bracket("rollout_store", lambda: ops.rollout_store_vecnorm(
                self.env.frame, self.env.reward, self.env.done, self.obs[t], self.obs[t + 1],
                self._store_net, self.dones[t + 1], self.ret_state, self.rms_state, self.rewards[t],
                scale255=self.prescale, reset_prev=rp))
        else:
            self.timer.bracket("rollout_store", lambda: ops.rollout_store(
                self.env.frame, self.env.reward, self.env.done, self.obs[t], self.obs[t + 1],
                self._store_net, self.rewards[t], self.dones[t + 1], scale255=self.prescale,
                reset_prev=rp))

    def _rollout_begin(self):
        T = self.T
        self.obs[0].copy_(self.obs[T])
        self.dones[0].copy_(self.dones[T])
        if self.args.sampling_noise == "rollout":
            self.noise.exponential_()  # the whole rollout's Exp(1) draws in one generator call
        elif self.args.sampling_noise == "kernel":
            # the reference's T per-step draws (the claimed generator range), one launch
            self.timer.bracket("noise_draws", lambda: self.exp_stream.fill(self.noise))

    def _rollout_end(self):
        """Bootstrap + GAE (:533-547) + minibatch adv stats (:577-579)."""
        a = self.args
        T = self.T
        if self.frame_cache:
            self.values[T].copy_(self.agent._head(self.agent.critic,
                                                  self._policy_hidden(T)).view(-1))
        elif self.u8_rollout:
            self.values[T].copy_(self.agent._head(
                self.agent.critic, self.agent.trunk_frames(self.obs[T], self.env_rows)).view(-1))
        else:
            self.values[T].copy_(self.agent.get_value(self.net_obs, self.prescale).view(-1))
        rec = self.records
        self.timer.bracket("gae", lambda: ops.gae(
            self.rewards, self.values[:T], self.dones[:T], self.values[T], self.dones[T],
            a.gamma, a.gae_lambda, self.advantages, self.returns, logprobs=self.logprobs,
            actions=self.actions, records=rec))
        self._prepare_minibatches(from_records=rec is not None)

    def _prepare_minibatches(self, from_records: bool = False):
        """Every minibatch's per-sample records in minibatch order + its adv (mean, std)
        (:566-579: b_*[mb_inds] and the minibatch advantage statistics). from_records: gather
        the 16-B sample records this iteration's GAE wrote (one gather per sample instead of
        five; bitwise the same outputs)."""
        T = self.T
        rec = self.records if from_records else None
        self.timer.bracket("mb_prepare", lambda: ops.minibatch_prepare(
            self.perm_dev, self.M, self.actions.view(-1), self.logprobs.view(-1),
            self.advantages.view(-1), self.returns.view(-1), self.values[:T].reshape(-1),
            out=self.mb, with_stats=self.args.norm_adv, records=rec))

    def _rollout(self):
        """Rollout (:500-530) + bootstrap + GAE (:533-547) + minibatch adv stats (:577-579)."""
        with torch.no_grad(), agents.rollout_inference():
            self._rollout_begin()
            for t in range(self.T):
                self._rollout_step(t)
            self.env.advance(self.T)
            self._rollout_end()

    def _host_part(self, k: int):
        """Device work between two host env steps (host env): part k uploads env step k-1's
        staging block and stores it, then acts for step k and queues its actions' D2H copy; part
        T ends the rollout. Each part is one hipGraph once captured."""
        with torch.no_grad():
            if k == 0:
                self._rollout_begin()
            else:
                self.env.upload()
                if not self.rollout_fusion:
                    self._store(k - 1)
            if k < self.T:
                self._act(k)
                self.env.fetch_actions(self.actions[k])
            else:
                self._rollout_end()

    def _rollout_host(self):
        for k in range(self.T + 1):
            if k > 0:  # eager, ordered before part k's store of step k-1
                self.env.upload_resets()
            if self.g_host:
                self.g_host[k].replay()
            else:
                self._host_part(k)
            if k < self.T:
                self.env.host_step()  # waits for part k's action copy, steps the CPU env

    def _forward_backward(self, j: int):
        """Minibatch j: gather, forward, fused loss, backward into the flat grad buffer (the
        weights' bf16 planes refreshed first: the previous minibatch's step changed them)."""
        if not self.wplanes_built:
            self.wplanes, self.wplanes_built = self._weight_planes(), True
            # the optimizer step writes the planes of the weights it just changed (FlatAdam plane
            # jobs): the split launch then runs once per iteration (weights changed outside the
            # optimizer between iterations -- checkpoint loads, tests -- are re-split there)
            self.planes_by_opt = (ADAM_WRITES_PLANES and self.wplanes is not None
                                  and self.args.fused_optimizer and len(self.wplanes.jobs) <= 8
                                  and all(w.is_contiguous() for w, _, _ in self.wplanes.jobs))
            if self.planes_by_opt:
                self.optimizer.write_planes(self.wplanes.jobs)
        if self.wplanes is None:
            return self._forward_backward_body(j)
        if j == 0 or not self.planes_by_opt:
            self.timer.bracket("split_planes", self.wplanes.refresh)
        with agents.weight_planes():
            return self._forward_backward_body(j)

    def _forward_backward_body(self, j: int):
        a = self.args
        idx = self.perm_dev[j * self.M:(j + 1) * self.M]
        ag = self.agent
        if self.frame_dedup:
            e, k = divmod(j, self.nmb)
            uniq, pos_of, inv = self.plan
            hidden = frames.minibatch_hidden(ag, self.obs, self.dones, uniq[j], pos_of[j], inv[e],
                                             idx, k, split=self.split)
            if self.split:
                hidden, self.cuts[j] = hidden
            if self._fused_tail(j, hidden):
                return
            logits, value = ag.heads(hidden)
        elif self.u8_first_conv:
            # the first convolution reads the u8 frame stacks through idx (no f32 minibatch copy)
            hidden = ag.trunk_frames(self.b_obs, idx)
            if self._fused_tail(j, hidden):
                return
            logits, value = ag.heads(hidden)
        else:
            self.timer.bracket("gather", lambda: ops.gather_rows(self.b_obs, idx, self.mb_obs,
                                                                 scale255=self.prescale))
            hidden = ag.trunk(self.mb_obs, self.prescale)
            if self._fused_tail(j, hidden):
                return
            logits, value = ag.heads(hidden)
        lg, vv = logits.detach(), value.detach().view(-1)  # the timer's closure must not hold
        sl = slice(j * self.M, (j + 1) * self.M)
        mb = self.mb
        self.timer.bracket("ppo_loss", lambda: ops.ppo_loss_fwd_bwd(  # the autograd graph
            lg, vv, mb["actions"][sl], mb["logprobs"][sl], mb["advantages"][sl],
            mb["returns"][sl], mb["values"][sl], mb_inds=None,
            adv_stats=mb["adv_stats"][j] if a.norm_adv else None, clip_coef=a.clip_coef,
            ent_coef=a.ent_coef, vf_coef=a.vf_coef, norm_adv=a.norm_adv,
            clip_vloss=a.clip_vloss, dlogits=self.dlogits, dvalue=self.dvalue,
            stats=self.stats[j], workspace=self.loss_ws))
        if not self.direct_grads:
            self.grad_buf.zero_()
        torch.autograd.backward([logits, value], [self.dlogits, self.dvalue.view(-1, 1)])

    def _fused_tail(self, j: int, hidden) -> bool:
        """Heads forward + fused loss + heads backward (with the decoder's ReLU mask and bias grad)
        as ONE HIP op on the decoder output (ops.heads_loss_fwd_bwd), then autograd from the
        decoder down. Taken when the head / decoder grads are written in place (FlatAdam)."""
        if hidden is None or not self.fused_heads_loss:
            return False
        box = getattr(hidden, "_ocppo_box", None)
        if box is None or not ops.heads_loss_ok(hidden, self.A):
            return False
        a, ag, mb = self.args, self.agent, self.mb
        sl = slice(j * self.M, (j + 1) * self.M)
        box["premasked"] = True  # the decoder's _LinearAct backward gets gp with its mask applied
        # the heads-loss finish (heads' and decoder-bias grads, loss statistics) rides in the
        # decoder's split-K weight-gradient combine (agents._weight_grad), or runs alone below
        box["finish"] = self.hl_finish
        if not self.direct_grads:
            self.grad_buf.zero_()  # before any of this minibatch's gradient writes
        h = hidden.detach()
        self.timer.bracket("heads_loss", lambda: ops.heads_loss_fwd_bwd(
            h, ag.actor.weight, ag.actor.bias, ag.critic.weight, ag.critic.bias,
            mb["actions"][sl], mb["logprobs"][sl], mb["advantages"][sl], mb["returns"][sl],
            mb["values"][sl], adv_stats=mb["adv_stats"][j] if a.norm_adv else None,
            clip_coef=a.clip_coef, ent_coef=a.ent_coef, vf_coef=a.vf_coef, norm_adv=a.norm_adv,
            clip_vloss=a.clip_vloss, gp=self.gp_tail, db_h=box["bias"].grad,
            dwa=ag.actor.weight.grad, dwc=ag.critic.weight.grad, dba=ag.actor.bias.grad,
            dbc=ag.critic.bias.grad, stats=self.stats[j], defer=self.hl_finish))
        torch.autograd.backward(hidden, self.gp_tail)
        self.hl_finish.run()  # no-op when the combine took it
        return True

    def _backward_low(self, j: int):
        """Second backward phase of a split minibatch: the encoder layers below the cut."""
        # popped: a cut kept alive past its backward would keep the autograd graph (and its
        # AccumulateGrad nodes, bound to the stream they were created on) alive into the next
        # capture, which then syncs with that stream and breaks
        low, low_d = self.cuts.pop(j)
        with agents.weight_planes():
            torch.autograd.backward(low, low_d.grad)

    def _exchange(self, j: int, replay: bool):
        """Minibatch j's gradients, all-reduced (GradExchange; the `/ world_size` is folded into
        the fused optimizer step). Split form: the first backward phase has filled the flat
        buffer's tail (the last encoder layer, decoder and heads); its all-reduce runs on RCCL's
        stream while the second phase (the encoder layers below the cut) runs on ours, then the
        head of the buffer follows."""
        if self.comm is not None:
            ex = RcclExchange(self.grad_buf, self.tail_off, self.world, self.args.fused_optimizer,
                              self.comm, self.side)
        else:
            ex = GradExchange(self.grad_buf, self.tail_off, self.world, self.args.fused_optimizer)
        if not self.split:
            ex.whole()
        elif replay:
            ex.split(self.g_low[j].replay)
        else:
            ex.split(lambda: self._backward_low(j))

    def _opt_step(self):
        if self.args.fused_optimizer:
            self.optimizer.step(grad_scale=1.0 / self.world)
        else:
            nn.utils.clip_grad_norm_(self.params, self.args.max_grad_norm)
            self.optimizer.step()

    def _update_epoch(self, epoch: int):
        for k in range(self.nmb):
            j = epoch * self.nmb + k
            self._forward_backward(j)
            if self.dp:
                self._exchange(j, replay=False)
            self._opt_step()

    # ------------------------------------------------------------------------------------------
    def _shuffle(self):
        """np.random.shuffle(b_inds) once per epoch (:561), all epochs up front, plus (frame
        dedup) the minibatches' frame plan; one async copy each into the staging buffers. Runs
        for iteration i+1 while the GPU executes iteration i (same RNG stream order)."""
        self.perm_event.synchronize()  # the previous async copies out of the host buffers are done
        out = self.perm_host.numpy()
        self.staged_rng_state = self.np_rng.get_state()
        self.b_inds = np.arange(self.B)  # b_inds = np.arange(batch_size) every iteration (:558)
        for e in range(self.E):
            self.np_rng.shuffle(self.b_inds)
            out[e * self.B:(e + 1) * self.B] = self.b_inds
        self._stage(out)

    def _stage(self, out: np.ndarray):
        """Stage the epochs' permutations `out` (a view of perm_host) and, with frame dedup,
        their frame plan: one async copy each into the staging buffers."""
        if self.frame_dedup:
            used, inv = self.planner.plan(out)
            cap = self.planner.cap
            if cap is None or int(self.planner.counts.max()) > cap:
                self._alloc_plan(self.planner.cap_for(self.planner.counts))
            self.planner.fill(self.plan_host.numpy(), self.planner.cap, used, inv)
        if self.copy_stream is not None:
            self.copy_stream.wait_event(self.stage_read)
            with torch.cuda.stream(self.copy_stream):
                if self.frame_dedup:
                    self.plan_stage.copy_(self.plan_host, non_blocking=True)
                self.perm_stage.copy_(self.perm_host, non_blocking=True)
                self.perm_event.record()
        else:
            if self.frame_dedup:
                self.plan_stage.copy_(self.plan_host, non_blocking=True)
            self.perm_stage.copy_(self.perm_host, non_blocking=True)
            self.perm_event.record()
        self.staged = True

    def load_permutation(self, perm) -> None:
        """Use `perm` [E*B] (the epochs' shuffles) as the current iteration's minibatch order,
        with its frame plan, in place of the np.random stream (tests: a reference fixture's
        permutation through the trainer's own update path)."""
        perm = np.asarray(perm, np.int64)
        if perm.shape != (self.E * self.B,):
            raise ValueError(f"perm must have {self.E * self.B} entries, got {perm.shape}")
        self.perm_event.synchronize()
        out = self.perm_host.numpy()
        out[:] = perm
        self.staged_rng_state = self.np_rng.get_state()
        self._stage(out)
        self._load_staged()

    def _rewind_shuffle(self, epochs: int):
        """target_kl stopped the update after `epochs` epochs: the reference drew only that many
        shuffles this iteration (:561), so put the np RNG where those draws leave it."""
        self.np_rng.set_state(self.current_rng_state)
        b = np.arange(self.B)
        for _ in range(epochs):
            self.np_rng.shuffle(b)

    def _alloc_plan(self, cap: int):
        """(Re)size the frame-plan buffers for `cap` distinct frames per minibatch. A resize
        after capture waits for the GPU and drops the graphs (they hold the old addresses)."""
        if self.plan_dev is not None:
            torch.cuda.synchronize(self.dev)
            self.graphs_ready = False
            self.g_rollout, self.g_update, self.g_opt, self.g_low = None, [], None, []
            self.g_host = []
        self.planner.cap = cap
        n = self.planner.size(cap)
        self.plan_host = torch.empty(n, dtype=torch.int32, pin_memory=True)
        self.plan_stage = torch.zeros(n, dtype=torch.int32, device=self.dev)
        self.plan_dev = torch.zeros(n, dtype=torch.int32, device=self.dev)
        self.plan = self.planner.views(self.plan_dev, cap)

    def _load_staged(self):
        """Move the staged shuffle / frame plan into the buffers the graphs read."""
        if not self.staged:
            self._shuffle()
        self.current_rng_state = self.staged_rng_state
        if self.copy_stream is not None:
            torch.cuda.current_stream(self.dev).wait_event(self.perm_event)
        self.perm_dev.copy_(self.perm_stage)
        if self.frame_dedup:
            self.plan_dev.copy_(self.plan_stage)
        self.stage_read.record()  # the next staging copies may overwrite the stage after this
        self.staged = False

    def _capture(self):
        """Capture the rollout and the update into hipGraphs (after one eager warm-up iteration,
        which has also created the Adam state)."""
        torch.cuda.synchronize(self.dev)
        self.g_rollout = None
        pool = None
        if not self.host_env:
            self.g_rollout = torch.cuda.CUDAGraph()
            with _graph_capture(self.g_rollout):
                self._rollout()
            pool = self.g_rollout.pool()
        else:  # a host env steps between the parts: one graph per part
            for k in range(self.T + 1):
                g = torch.cuda.CUDAGraph()
                with _graph_capture(g, pool):
                    self._host_part(k)
                pool = pool if pool is not None else g.pool()
                self.g_host.append(g)
        if not self.graph_update:
            pass
        elif not self.dp or self.captured_exchange:
            # (DP: the epoch's all-reduces captured with it -- the package's own communicator, or
            # torch's collectives, for which ProcessGroupNCCL records no watchdog work)
            for e in range(self.E):
                g = torch.cuda.CUDAGraph()
                with _graph_capture(g, pool, quiesce=self.quiesce):
                    self._update_epoch(e)
                self.g_update.append(g)
                pool = pool if pool is not None else g.pool()
        else:
            for j in range(self.E * self.nmb):
                g = torch.cuda.CUDAGraph()
                with _graph_capture(g, pool):
                    self._forward_backward(j)
                self.g_update.append(g)
                pool = pool if pool is not None else g.pool()
                if self.split:  # second backward phase: reads the cut tensors of graph j
                    g = torch.cuda.CUDAGraph()
                    with _graph_capture(g, pool):
                        self._backward_low(j)
                    self.g_low.append(g)
            self.g_opt = torch.cuda.CUDAGraph()
            with _graph_capture(self.g_opt, pool):
                self._opt_step()
        self.graphs_ready = True

    def _run_update(self):
        """update_epochs x num_minibatches updates (:560-617); with target_kl, the epoch loop
        stops after the first epoch whose last minibatch's approx_kl exceeds it (:616-617)."""
        a = self.args
        self.executed_mb = 0
        for e in range(self.E):
            if self.graphs_ready and self.graph_update:
                if not self.dp or self.captured_exchange:
                    self.g_update[e].replay()
                else:
                    for k in range(self.nmb):
                        j = e * self.nmb + k
                        self.g_update[j].replay()
                        self._exchange(j, replay=True)
                        self.g_opt.replay()
            else:
                self._update_epoch(e)
            self.executed_mb += self.nmb
            if a.target_kl is not None:
                kl = float(self.stats[e * self.nmb + self.nmb - 1, 5])
                if kl > a.target_kl:
                    if e + 1 < self.E:
                        self._rewind_shuffle(e + 1)
                    break

    # ------------------------------------------------------------------------------------------
    def train_iteration(self, collect_metrics: bool = True, lag: bool = False) -> dict:
        """One PPO iteration (:469-670). lag: the iteration's metric scalars are gathered on the
        device and copied to pinned host memory behind its work, and the PREVIOUS iteration's
        metrics are returned (flush_metrics() returns the last one): the host never waits for
        the GPU between iterations, so the next iteration's work is queued while the host turns
        this one's scalars into the dict (same scalars as lag=False, one iteration later)."""
        a = self.args
        self.iteration += 1
        if a.anneal_lr:
            frac = 1.0 - (self.iteration - 1.0) / max(a.num_iterations, 1)
            self.lr.fill_(frac * a.learning_rate)
        self._load_staged()
        use_graphs = a.cuda_graphs and self.iteration > 1
        if use_graphs and not self.graphs_ready:
            self._capture()
        if self.exp_stream is not None:
            # the rollout's T draws of the reference stream: the generator state they start at
            # (read by the sampling kernels, captured or not) and the generator advanced past them
            self.exp_stream.claim(self.T)
        if self.host_env:
            self._rollout_host()
        elif self.graphs_ready:
            self.g_rollout.replay()
        else:
            self._rollout()
        self._run_update()
        if a.prefetch_shuffle:
            self._shuffle()  # host work of the next iteration, overlapped with this one's GPU work
        self.timer.end_iteration()
        self.global_step += self.N * self.T * self.world
        m = {}
        if collect_metrics and lag and self._lag_ok():
            prev, self._pending_metrics = self._pending_metrics, self._metrics_device()
            if prev is not None:
                m = self._metrics_from(prev)
        elif collect_metrics:
            m = self.flush_metrics()
            m.update(self._metrics())
        return m

    def _lag_ok(self) -> bool:
        return self.args.target_kl is None and hasattr(self.env, "ep_state")

    def flush_metrics(self) -> dict:
        """The metrics of the last lagged iteration still pending ({} if none)."""
        prev, self._pending_metrics = self._pending_metrics, None
        return self._metrics_from(prev) if prev is not None else {}

    def _metrics_device(self):
        """_metrics' scalars gathered on the device and copied (non-blocking) into pinned host
        memory behind this iteration's work: (event, host vector, executed minibatches)."""
        y_true = self.returns.double().view(-1)
        y_pred = self.values[:self.T].double().reshape(-1)
        var_y = torch.var(y_true, unbiased=False)
        ev = 1 - torch.var(y_true - y_pred, unbiased=False) / var_y
        ep = self.env.ep_state[:, 2:5].sum(0, dtype=torch.float64)
        self.env.ep_state[:, 2:5].zero_()
        n = self.executed_mb
        vec = torch.cat([var_y.view(1), ev.view(1), self.lr.double().view(1), ep,
                         self.stats[:n].double().reshape(-1)])
        # the other vector than the one the still-pending record (the previous iteration's) reads
        k = self._metrics_turn
        self._metrics_turn ^= 1
        if self._metrics_host[k] is None or self._metrics_host[k].numel() < vec.numel():
            self._metrics_host[k] = torch.empty(vec.numel(), dtype=torch.float64, pin_memory=True)
        host = self._metrics_host[k][:vec.numel()]
        host.copy_(vec, non_blocking=True)
        done = torch.cuda.Event()
        done.record()
        return done, host, n

    def _metrics_from(self, pend) -> dict:
        done, host, n = pend
        done.synchronize()
        v = host.numpy().copy()
        var_y, ev, lr = float(v[0]), float(v[1]), float(v[2])
        ep_ret, ep_len, ep_n = (float(t) for t in v[3:6])
        stats = v[6:].reshape(n, -1)
        last = stats[-1]
        m = {
            "charts/learning_rate": lr,
            "losses/value_loss": float(last[2]),
            "losses/policy_loss": float(last[1]),
            "losses/entropy": float(last[3]),
            "losses/old_approx_kl": float(last[4]),
            "losses/approx_kl": float(last[5]),
            "losses/clipfrac": float(np.mean(stats[:, 6].astype(np.float32))),
            "losses/explained_variance": float("nan") if var_y == 0 else ev,
            "losses/loss": float(last[0]),
        }
        if ep_n > 0:
            m["charts/Episodic_Original_Reward"] = ep_ret / ep_n
            m["charts/Episodic_Length"] = ep_len / ep_n
        self.last_metrics = m
        return m

    def _metrics(self) -> dict:
        """Device-side scalars → host once (the reference syncs with .item() ~20 times)."""
        a = self.args
        y_true = self.returns.double().view(-1)
        y_pred = self.values[:self.T].double().reshape(-1)
        var_y = torch.var(y_true, unbiased=False)
        ev = 1 - torch.var(y_true - y_pred, unbiased=False) / var_y
        # rows of the minibatches this iteration executed (target_kl may stop early): the scalars
        # of the last executed one, clipfrac averaged over the executed ones (:616-638)
        stats = self.stats[:self.executed_mb].cpu().numpy()  # sync point
        ep_ret, ep_len, ep_n = self.env.pop_episode_stats()
        last = stats[-1]
        m = {
            "charts/learning_rate": float(self.lr),
            "losses/value_loss": float(last[2]),
            "losses/policy_loss": float(last[1]),
            "losses/entropy": float(last[3]),
            "losses/old_approx_kl": float(last[4]),
            "losses/approx_kl": float(last[5]),
            "losses/clipfrac": float(np.mean(stats[:, 6])),
            "losses/explained_variance": float("nan") if float(var_y) == 0 else float(ev),
            "losses/loss": float(last[0]),
        }
        if ep_n > 0:
            m["charts/Episodic_Original_Reward"] = ep_ret / ep_n
            m["charts/Episodic_Length"] = ep_len / ep_n
        self.last_metrics = m
        return m

    # ------------------------------------------------------------------------------------------
    def state_dict_checkpoint(self) -> dict:
        """The `.cleanrl_model` payload of ppo_atari_oc.py:486-490."""
        return {"model_weights": _own_tensors(self.agent.state_dict()), "args": asdict(self.args),
                "Timesteps": self.iteration * self.args.batch_size}

    def save(self, path):
        torch.save(self.state_dict_checkpoint(), path)

    @staticmethod
    def _rccl_comm(rank: int, world: int, device):
        """The package's RCCL communicator: (comm or None, the form in use). Two agreements
        through the process group, each an all-reduce every rank reaches: (1) before the
        collective init, that every rank loaded the library and rank 0 drew the unique id -- a
        refusal there falls back to torch's collectives on every rank; (2) after the init, one
        eager all-reduce on the communicator checked for the right sum. A rank whose
        ncclCommInitRank itself fails cannot take part in (2) (its peers wait inside their init):
        that case is bounded by the rank watchdog (watch.RankWatch, bench.py's stall limits), not
        recovered."""
        def agree(why):
            ok = torch.tensor([0 if why else 1], dtype=torch.int32, device=device)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            return int(ok.item()) == 1

        uid, why = None, ""
        try:
            if rank == 0:
                uid = rccl.unique_id()
            else:
                rccl._lib()
        except (OSError, RuntimeError) as e:
            why = str(e)
        if not agree(why):
            return None, f"torch collectives (RCCL library refused: {why or 'on a peer'})"
        comm = RcclComm(rank, world, uid=uid)  # collective; a failure here ends the rank
        try:
            t = torch.ones(1, dtype=torch.float32, device=device)
            comm.all_reduce_sum(t)
            torch.cuda.synchronize(device)
            if float(t.item()) != float(world):
                why = f"check all-reduce gave {float(t.item())} for {world} ranks"
        except RuntimeError as e:  # ncclResult of the check
            why = str(e)
        if agree(why):
            return comm, "rccl (own communicator, captured per epoch)"
        comm.close(abort=True)
        return None, f"torch collectives (own RCCL communicator refused: {why or 'on a peer'})"

    def close(self):
        """Release the exchange's RCCL communicator (before the process group is destroyed)."""
        if self.comm is not None:
            torch.cuda.synchronize(self.dev)
            self.comm.close()
            self.comm = None

    def param_checksum(self) -> int:
        """An exact, order-sensitive checksum of every parameter's f32 bit pattern (int64 sum of
        bits × (position mod 65521 + 1)). The DP replicas of ppo_atari_multigpu.py:360-377 start
        from one init and apply the same all-reduced step, so this is equal on every rank."""
        total = 0
        for p in self.params:
            bits = p.detach().contiguous().view(-1).view(torch.int32).to(torch.int64)
            w = torch.arange(bits.numel(), dtype=torch.int64, device=bits.device) % 65521 + 1
            total = (total * 1_000_003 + int((bits * w).sum())) % (1 << 61)
        return total


def _own_tensors(sd: dict) -> dict:
    """Parameters are views of the optimizer's flat buffer: save standalone copies so the
    checkpoint holds exactly the reference's tensors."""
    return {k: v.detach().clone() for k, v in sd.items()}


def run(args: Args, device=None, rank: int = 0, world_size: int = 1) -> PPOTrainer:
    """The script body: iterations, SPS, metrics JSONL, checkpoints (rank 0)."""
    if device is None:
        device = torch.device(f"cuda:{rank % max(torch.cuda.device_count(), 1)}")
    tr = PPOTrainer(args, device, rank, world_size)
    run_name = f"{args.env_id}__{args.exp_name}__{args.seed}__{int(time.time())}".replace("/", "_")
    run_dir = Path(args.log_dir) / run_name
    writer = None
    if rank == 0:
        run_dir.mkdir(parents=True, exist_ok=True)
        (run_dir / "args.json").write_text(json.dumps(asdict(args), indent=1, default=str))
        writer = open(run_dir / "metrics.jsonl", "w")
    watch = None
    if args.stall_timeout > 0:  # fail fast: a rank stuck in an iteration ends the run, with a record
        import sys

        from .watch import RankWatch

        port = os.environ.get("MASTER_PORT", str(os.getpid()))
        watch = RankWatch(rank, world_size, os.environ.get("OCPPO_WATCH_DIR",
                                                           f"/tmp/ocppo_watch_{port}"),
                          stall_s=args.stall_timeout,
                          on_fire=lambda rec: print(json.dumps(rec), file=sys.stderr, flush=True))
    start = time.time()
    for it in range(1, args.num_iterations + 1):
        if watch is not None:  # the first two iterations also capture the graphs
            watch.phase(f"iteration {it}", stall_s=args.stall_timeout * (3 if it <= 2 else 1))
        if it % args.checkpoint_interval == 0 and rank == 0 and args.save_model:
            tr.save(run_dir / f"{args.exp_name}_{it}.cleanrl_model")
        collect = (it % args.metrics_every == 0) or it == args.num_iterations
        m = tr.train_iteration(collect_metrics=collect)
        if writer and m:
            m["charts/SPS"] = int(tr.global_step / (time.time() - start))
            m["global_step"] = tr.global_step
            writer.write(json.dumps(m) + "\n")
            writer.flush()
    if rank == 0 and args.save_model:
        torch.save({"model_weights": _own_tensors(tr.agent.state_dict()), "args": asdict(args)},
                   run_dir / f"{args.exp_name}_final.cleanrl_model")
    if rank == 0 and args.eval_episodes > 0:  # ppo_atari_oc.py:687-695 (FinalReward_* summary)
        from .evals import evaluate, make_env

        rewards = evaluate(tr.agent, make_env, args.eval_episodes, tr.dev, env_id=args.env_id,
                           obs_mode=args.obs_mode, num_features=args.num_features,
                           seed=args.seed + 10_000)
        summ = {"eval/FinalReward_mean": float(np.mean(rewards)),
                "eval/FinalReward_median": float(np.median(rewards)),
                "eval/FinalReward_min": float(np.min(rewards)),
                "eval/FinalReward_max": float(np.max(rewards)), "eval/returns": rewards}
        tr.last_metrics.update({k: v for k, v in summ.items() if k != "eval/returns"})
        if writer:
            writer.write(json.dumps(summ) + "\n")
    if writer:
        writer.close()
    if watch is not None:
        watch.stop()
    return tr
