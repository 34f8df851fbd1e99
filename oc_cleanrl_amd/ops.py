"""torch-facing wrappers of the HIP kernels (libocppo_hip.so).

Every function takes CUDA (HIP) tensors, validates shapes/dtypes/devices on the host before any
launch, and launches on the current torch stream of the tensors' device, so everything here is
asynchronous and capturable into a torch.cuda.CUDAGraph (hipGraph). There is no CPU fallback: a
CPU tensor is an error.

Reference lines replaced are cited per function (paths relative to the reference checkout).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import OCPPO_BF16, OCPPO_F32, OCPPO_U8, STAT_NAMES, call

_DTYPE_CODE = {torch.float32: OCPPO_F32, torch.bfloat16: OCPPO_BF16, torch.uint8: OCPPO_U8}


def _check(t: torch.Tensor, name: str, dtype: torch.dtype | None = None, device=None,
           numel: int | None = None) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: HIP kernels need a GPU tensor, got device {t.device}")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if numel is not None and t.numel() != numel:
        raise ValueError(f"{name}: has {t.numel()} elements, expected {numel}")
    return t.data_ptr()


def _opt(t, *a, **k) -> int | None:
    return None if t is None else _check(t, *a, **k)


def _net_obs(net_obs, N: int, W: int, D: int, device):
    """(pointer, layout) of a rollout network-input buffer: a contiguous [N, W, ...] f32 tensor
    (layout 0) or a channels_last [N, W, H, X] one (layout 1: memory [N, H, X, W], the NHWC input
    of a channels_last NatureCNN)."""
    if net_obs is None:
        return None, 0
    if net_obs.is_contiguous():
        return _check(net_obs, "net_obs", torch.float32, device, N * W * D), 0
    if net_obs.dim() == 4 and net_obs.is_contiguous(memory_format=torch.channels_last) and \
            tuple(net_obs.shape[:2]) == (N, W) and net_obs[0, 0].numel() == D:
        if net_obs.dtype != torch.float32 or net_obs.device != device:
            raise ValueError(f"net_obs: expected float32 on {device}")
        return net_obs.data_ptr(), 1
    raise ValueError("net_obs must be contiguous [N, W, ...] or channels_last [N, W, H, X]")


# Optional per-launch timer for launch sites inside autograd (the trainer's KernelTimer when
# kernel timing is on): timed(name, fn) runs fn and lets the timer keep its first eager launch.
TIMER = None


def timed(name: str, fn):
    return TIMER.bracket(name, fn) if TIMER is not None else fn()


# gemm_x6 launches issued with pre-split weight planes, by (M, N, K): host-side bookkeeping at
# issue time (under capture: once per captured launch), so tests can see that the planes a
# WeightPlanes refresh writes are actually read
PLANE_USES: dict = {}


def _note_planes(b_planes, M: int, N: int, K: int):
    if b_planes is not None:
        PLANE_USES[(M, N, K)] = PLANE_USES.get((M, N, K), 0) + 1


def _stream(device: torch.device) -> int:
    if device.type != "cuda":
        raise ValueError(f"HIP kernels need GPU tensors, got device {device} (no CPU fallback)")
    return torch.cuda.current_stream(device).cuda_stream


# ---------------------------------------------------------------------------------------------
# GAE (ppo_atari_oc.py:533-547)
# ---------------------------------------------------------------------------------------------
def gae(rewards, values, dones, next_value, next_done, gamma: float, gae_lambda: float,
        advantages=None, returns=None, logprobs=None, actions=None, records=None):
    """Advantages and returns of one rollout; [T, N] f32 in, ([T, N], [T, N]) out.

    Bit-identical to the reference loop. `next_value` may be [N] or [1, N] (as produced by
    `agent.get_value(next_obs).reshape(1, -1)`). records (with logprobs [T, N] f32 and actions
    [T, N] i64 in [0, 2^31)): also write each sample's 16-B record (sample_records) for
    minibatch_prepare(records=...).
    """
    if rewards.dim() != 2:
        raise ValueError(f"rewards must be [T, N], got {tuple(rewards.shape)}")
    T, N = rewards.shape
    dev = rewards.device
    f = torch.float32
    if advantages is None:
        advantages = torch.empty_like(rewards)
    if returns is None:
        returns = torch.empty_like(rewards)
    args = (_check(rewards, "rewards", f, dev),
            _check(values, "values", f, dev, T * N), _check(dones, "dones", f, dev, T * N),
            _check(next_value, "next_value", f, dev, N), _check(next_done, "next_done", f, dev, N),
            T, N, float(gamma), float(gae_lambda), _check(advantages, "advantages", f, dev, T * N),
            _check(returns, "returns", f, dev, T * N))
    if records is None:
        call("ocppo_gae", _stream(dev), *args)
    else:
        call("ocppo_gae_records", _stream(dev), *args,
             _check(logprobs, "logprobs", f, dev, T * N),
             _check(actions, "actions", torch.int64, dev, T * N),
             _check(records, "records", torch.int32, dev, 4 * T * N))
    return advantages, returns


def sample_records(B: int, device):
    """[B] x 16-B per-sample records (ocppo.h OcppoSampleRecord) as an int32 [B, 4] tensor."""
    return torch.zeros((B, 4), dtype=torch.int32, device=device)


# ---------------------------------------------------------------------------------------------
# minibatch advantage statistics (ppo_atari_oc.py:577-579)
# ---------------------------------------------------------------------------------------------
def minibatch_adv_stats(b_advantages, perm, minibatch_size: int, out=None):
    """(mean, unbiased std) of b_advantages over each minibatch of `perm` → [num_mb, 2]."""
    dev = b_advantages.device
    if perm.numel() % minibatch_size:
        raise ValueError("perm length must be a multiple of minibatch_size")
    num_mb = perm.numel() // minibatch_size
    if out is None:
        out = torch.empty((num_mb, 2), dtype=torch.float32, device=dev)
    call("ocppo_minibatch_adv_stats", _stream(dev),
         _check(b_advantages, "b_advantages", torch.float32, dev),
         _check(perm, "perm", torch.int64, dev), minibatch_size, num_mb,
         _check(out, "out", torch.float32, dev, 2 * num_mb))
    return out


def minibatch_prepare(perm, minibatch_size: int, b_actions, b_logprobs, b_advantages, b_returns,
                      b_values, out: dict | None = None, with_stats: bool = True, records=None):
    """Gather every minibatch's per-sample arrays into minibatch order (+ adv stats).
    records: the 16-B per-sample records of gae(records=...) gathered instead of the five b_*
    arrays (then only their sizes are read; bitwise the same outputs).

    Returns dict(actions, logprobs, advantages, returns, values: [num_mb*M], adv_stats [num_mb,2])."""
    dev = perm.device
    M = minibatch_size
    n = perm.numel()
    if n % M:
        raise ValueError("perm length must be a multiple of minibatch_size")
    num_mb = n // M
    B = b_logprobs.numel()
    f = torch.float32
    if records is not None:
        if out is None:
            out = {"actions": torch.empty(n, dtype=torch.int64, device=dev),
                   **{k: torch.empty(n, dtype=f, device=dev)
                      for k in ("logprobs", "advantages", "returns", "values")},
                   "adv_stats": torch.empty((num_mb, 2), dtype=f, device=dev)}
        call("ocppo_minibatch_prepare_records", _stream(dev),
             _check(perm, "perm", torch.int64, dev), M, num_mb,
             _check(records, "records", torch.int32, dev, 4 * B),
             _check(out["actions"], "mb_actions", torch.int64, dev, n),
             _check(out["logprobs"], "mb_logprobs", f, dev, n),
             _check(out["advantages"], "mb_advantages", f, dev, n),
             _check(out["returns"], "mb_returns", f, dev, n),
             _check(out["values"], "mb_values", f, dev, n),
             _check(out["adv_stats"], "adv_stats", f, dev, 2 * num_mb) if with_stats else None)
        return out
    if out is None:
        out = {"actions": torch.empty(n, dtype=torch.int64, device=dev),
               **{k: torch.empty(n, dtype=f, device=dev)
                  for k in ("logprobs", "advantages", "returns", "values")},
               "adv_stats": torch.empty((num_mb, 2), dtype=f, device=dev)}
    call("ocppo_minibatch_prepare", _stream(dev), _check(perm, "perm", torch.int64, dev), M,
         num_mb, _check(b_actions, "b_actions", torch.int64, dev, B),
         _check(b_logprobs, "b_logprobs", f, dev, B), _check(b_advantages, "b_advantages", f, dev, B),
         _check(b_returns, "b_returns", f, dev, B), _check(b_values, "b_values", f, dev, B),
         _check(out["actions"], "mb_actions", torch.int64, dev, n),
         _check(out["logprobs"], "mb_logprobs", f, dev, n),
         _check(out["advantages"], "mb_advantages", f, dev, n),
         _check(out["returns"], "mb_returns", f, dev, n),
         _check(out["values"], "mb_values", f, dev, n),
         _check(out["adv_stats"], "adv_stats", f, dev, 2 * num_mb) if with_stats else None)
    return out


# ---------------------------------------------------------------------------------------------
# fused PPO loss (ppo_atari_oc.py:566-602 from the network outputs on)
# ---------------------------------------------------------------------------------------------
class LossWorkspace:
    """Device scratch for ppo_loss_fwd_bwd (zeroed once; the kernel re-arms its ticket)."""

    def __init__(self, M: int, A: int, device):
        n = _lib.LIB.ocppo_ppo_loss_workspace_bytes(M, A)
        self.nbytes = int(n)
        self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self.M, self.A = M, A


def ppo_loss_fwd_bwd(logits, new_value, b_actions, b_logprobs, b_advantages, b_returns, b_values,
                     *, mb_inds=None, adv_stats=None, clip_coef: float, ent_coef: float,
                     vf_coef: float, norm_adv: bool, clip_vloss: bool, dlogits=None, dvalue=None,
                     stats=None, workspace: LossWorkspace | None = None):
    """One launch: loss statistics [9] plus dLoss/dlogits [M, A] and dLoss/dvalue [M].

    `b_*` are the flattened batch arrays (b_actions int64); `mb_inds` selects the minibatch
    (None = the b_* arrays are already the minibatch). Returns (stats, dlogits, dvalue); stats
    layout = _lib.STAT_NAMES.
    """
    if logits.dim() != 2:
        raise ValueError(f"logits must be [M, A], got {tuple(logits.shape)}")
    M, A = logits.shape
    dev = logits.device
    f = torch.float32
    B = b_logprobs.numel()
    if mb_inds is None and B != M:
        raise ValueError("without mb_inds the batch arrays must have M elements")
    if mb_inds is not None and mb_inds.numel() != M:
        raise ValueError(f"mb_inds has {mb_inds.numel()} elements, logits has M={M} rows")
    if dlogits is None:
        dlogits = torch.empty_like(logits)
    if dvalue is None:
        dvalue = torch.empty(M, dtype=f, device=dev)
    if stats is None:
        stats = torch.empty(len(STAT_NAMES), dtype=f, device=dev)
    if workspace is None:
        workspace = LossWorkspace(M, A, dev)
    call("ocppo_ppo_loss_fwd_bwd", _stream(dev), _check(logits, "logits", f, dev),
         _check(new_value, "new_value", f, dev, M), M, A,
         _opt(mb_inds, "mb_inds", torch.int64, dev, M),
         _check(b_actions, "b_actions", torch.int64, dev, B),
         _check(b_logprobs, "b_logprobs", f, dev, B),
         _check(b_advantages, "b_advantages", f, dev, B), _check(b_returns, "b_returns", f, dev, B),
         _check(b_values, "b_values", f, dev, B),
         _opt(adv_stats, "adv_stats", f, dev, 2) if norm_adv else None,
         float(clip_coef), float(ent_coef), float(vf_coef), int(bool(norm_adv)),
         int(bool(clip_vloss)), _check(dlogits, "dlogits", f, dev, M * A),
         _check(dvalue, "dvalue", f, dev, M), _check(stats, "stats", f, dev, len(STAT_NAMES)),
         workspace.buf.data_ptr(), workspace.nbytes)
    return stats, dlogits, dvalue


_HL_WS: dict = {}


# decoder widths ocppo_heads_loss_fwd_bwd is instantiated for (H / 64 columns per lane: 1, 2, 4, 8)
HEADS_LOSS_WIDTHS = (64, 128, 256, 512)


def heads_loss_ok(h, A: int) -> bool:
    H = h.shape[-1]
    return (h.is_cuda and h.dtype == torch.float32 and h.dim() == 2 and h.is_contiguous() and
            H in HEADS_LOSS_WIDTHS and 1 <= A <= 7 and h.data_ptr() % 16 == 0)


class DeferredFinish:
    """The finish of ocppo_heads_loss_rows (the tree over the heads-loss records that writes the
    heads' and decoder-bias gradients and the loss statistics) or of ocppo_relu_bias_wgrad_rows
    (the first layer's dw / db), held as the C-ABI's host record until a later launch on the same
    stream runs it: sum_splits(..., finish=) / sum_splits_db(..., finish=) fold it into a split-K
    combine, run() launches it alone. It must run exactly once (pending: not yet)."""

    def __init__(self, device):
        self.device = device
        self.rec = (ctypes.c_uint64 * 64)()
        self.pending = False  # filled by a rows launch, not yet run
        self.filled = False   # holds a record (a timer replay may run it again: same writes)

    def ptr(self) -> int:
        return ctypes.addressof(self.rec)

    def run(self):
        if self.pending:
            self.pending = False
            call("ocppo_deferred_finish_run", _stream(self.device), self.ptr())


def heads_loss_fwd_bwd(h, wa, ba, wc, bc, mb_actions, mb_logprobs, mb_advantages, mb_returns,
                       mb_values, *, adv_stats, clip_coef, ent_coef, vf_coef, norm_adv: bool,
                       clip_vloss: bool, gp=None, db_h=None, dwa=None, dwc=None, dba=None,
                       dbc=None, stats=None, dlogits=None, dvalue=None, defer=None):
    """The policy heads' forward, the fused PPO loss and the heads' backward with the decoder's
    ReLU mask, from the decoder output h [M, H] (include/ocppo.h ocppo_heads_loss_fwd_bwd).
    mb_* are the minibatch's prepared records [M]. Returns (gp, db_h, dwa, dwc, dba, dbc, stats).
    defer = a DeferredFinish: only the rows kernel runs now (ocppo_heads_loss_rows); db_h, dwa,
    dwc, dba, dbc and stats are written when the caller runs the finish."""
    M, H = h.shape
    A = wa.shape[0]
    dev = h.device
    f = torch.float32
    gp = torch.empty_like(h) if gp is None else gp
    dwa = torch.empty(A, H, dtype=f, device=dev) if dwa is None else dwa
    dwc = torch.empty(1, H, dtype=f, device=dev) if dwc is None else dwc
    dba = torch.empty(A, dtype=f, device=dev) if dba is None else dba
    dbc = torch.empty(1, dtype=f, device=dev) if dbc is None else dbc
    stats = torch.empty(len(STAT_NAMES), dtype=f, device=dev) if stats is None else stats
    key = (dev, M, H, A)
    ws = _HL_WS.get(key)
    if ws is None:
        nb = int(_lib.LIB.ocppo_heads_loss_workspace_bytes(M, H, A))
        ws = _HL_WS[key] = torch.zeros(nb // 4, dtype=f, device=dev)
    call("ocppo_heads_loss_rows" if defer is not None else "ocppo_heads_loss_fwd_bwd",
         _stream(dev), _check(h, "h", f, dev, M * H), M, H,
         _check(wa, "wa", f, dev, A * H), _check(ba, "ba", f, dev, A), _check(wc, "wc", f, dev, H),
         _check(bc, "bc", f, dev, 1), A, _check(mb_actions, "mb_actions", torch.int64, dev, M),
         _check(mb_logprobs, "mb_logprobs", f, dev, M),
         _check(mb_advantages, "mb_advantages", f, dev, M),
         _check(mb_returns, "mb_returns", f, dev, M), _check(mb_values, "mb_values", f, dev, M),
         _opt(adv_stats, "adv_stats", f, dev, 2) if norm_adv else None, float(clip_coef),
         float(ent_coef), float(vf_coef), int(bool(norm_adv)), int(bool(clip_vloss)),
         _check(gp, "gp", f, dev, M * H), _opt(db_h, "db_h", f, dev, H),
         _check(dwa, "dwa", f, dev, A * H), _check(dwc, "dwc", f, dev, H),
         _check(dba, "dba", f, dev, A), _check(dbc, "dbc", f, dev, 1),
         _check(stats, "stats", f, dev, len(STAT_NAMES)), _opt(dlogits, "dlogits", f, dev, M * A),
         _opt(dvalue, "dvalue", f, dev, M), ws.data_ptr(), ws.numel() * 4,
         *((defer.ptr(),) if defer is not None else ()))
    if defer is not None:
        defer.pending = defer.filled = True
    return gp, db_h, dwa, dwc, dba, dbc, stats


class _PPOLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, new_value, b_actions, b_logprobs, b_advantages, b_returns, b_values,
                mb_inds, adv_stats, cfg):
        stats, dlogits, dvalue = ppo_loss_fwd_bwd(
            logits.detach().contiguous(), new_value.detach().reshape(-1).contiguous(), b_actions,
            b_logprobs, b_advantages, b_returns, b_values, mb_inds=mb_inds, adv_stats=adv_stats,
            **cfg)
        ctx.save_for_backward(dlogits, dvalue)
        ctx.value_shape = new_value.shape
        ctx.mark_non_differentiable(stats)
        loss = stats[0].clone()
        return loss, stats

    @staticmethod
    def backward(ctx, grad_loss, grad_stats):
        dlogits, dvalue = ctx.saved_tensors
        return (dlogits * grad_loss, (dvalue * grad_loss).view(ctx.value_shape), None, None, None,
                None, None, None, None, None)


def ppo_loss(logits, new_value, b_actions, b_logprobs, b_advantages, b_returns, b_values,
             mb_inds=None, adv_stats=None, *, clip_coef, ent_coef, vf_coef, norm_adv=True,
             clip_vloss=True):
    """Differentiable fused PPO loss: returns (loss, stats). Only `loss` carries gradient."""
    cfg = dict(clip_coef=clip_coef, ent_coef=ent_coef, vf_coef=vf_coef, norm_adv=norm_adv,
               clip_vloss=clip_vloss)
    return _PPOLoss.apply(logits, new_value, b_actions, b_logprobs, b_advantages, b_returns,
                          b_values, mb_inds, adv_stats, cfg)


# ---------------------------------------------------------------------------------------------
# Categorical action head (architectures/ppo.py:89-95)
# ---------------------------------------------------------------------------------------------
class TorchExpStream:
    """The reference's sampling stream for the sampling kernels to draw themselves: the Exp(1)
    values torch.empty(N, A).exponential_() would return on `device`'s default generator, one
    [N, A] draw per rollout step (Categorical.sample, architectures/ppo.py:92-94, called at
    ppo_atari_oc.py:505-506). `claim(steps)` (host, before the rollout, outside any graph) takes
    the generator's current (seed, philox offset), advances the generator past `steps` draws as
    `steps` exponential_ calls would, and writes both into the device `state` the captured
    kernels read; `philox(t)` is step t's (state, offset, stride) argument."""

    def __init__(self, numel: int, device):
        self.device = torch.device(device)
        torch.cuda.init()  # default_generators is empty until the runtime is initialised
        self.gen = torch.cuda.default_generators[self.device.index
                                                 if self.device.index is not None else 0]
        self.stride, self.increment = torch_exponential_geometry(numel, self.device)
        self.state = torch.zeros(2, dtype=torch.int64, device=self.device)
        self._seed = None

    def claim(self, steps: int):
        base = self.gen.get_offset()
        self.gen.set_offset(base + steps * self.increment)
        seed = self.gen.initial_seed()
        if seed != self._seed:
            self.state[0].fill_(seed if seed < 1 << 63 else seed - (1 << 64))
            self._seed = seed
        self.state[1].fill_(base)  # a fill launch with the value as argument: no host sync

    def philox(self, t: int):
        return self.state, t * self.increment, self.stride

    def fill(self, noise):
        """noise [T, ...] = the T claimed draws (one launch; graph-capturable)."""
        return philox_exponential_steps(noise, self.state, 0, self.increment, self.stride)


def torch_exponential_geometry(numel: int, device) -> tuple[int, int]:
    """(grid stride, philox-offset increment) of torch's exponential_ over `numel` elements on
    `device` (ocppo_torch_exponential_geometry)."""
    props = torch.cuda.get_device_properties(device)
    stride, inc = ctypes.c_int64(), ctypes.c_int64()
    call("ocppo_torch_exponential_geometry", numel, props.multi_processor_count,
         props.max_threads_per_multi_processor, ctypes.byref(stride), ctypes.byref(inc))
    return stride.value, inc.value


def philox_exponential(out, state, offset: int, stride: int):
    """out[:] = torch's exponential_ draws at generator state[0..1] + (0, offset)."""
    dev = out.device
    call("ocppo_philox_exponential", _stream(dev), _check(out, "out", torch.float32, dev),
         out.numel(), _check(state, "philox_state", torch.int64, dev, 2), int(offset), int(stride))
    return out


def philox_exponential_steps(out, state, offset: int, increment: int, stride: int):
    """out[t] = torch's exponential_ draw t of shape out[0] at generator state[0..1] + (0, offset +
    t * increment): a rollout's per-step draws in one launch (out [steps, ...])."""
    dev = out.device
    steps = out.shape[0]
    call("ocppo_philox_exponential_steps", _stream(dev), _check(out, "out", torch.float32, dev),
         out[0].numel(), steps, _check(state, "philox_state", torch.int64, dev, 2), int(offset),
         int(increment), int(stride))
    return out


def _noise_args(noise, philox, n, dev):
    """(noise pointer, philox state pointer, offset, stride) of a sampling entry: noise read, or
    philox = (state, offset, stride) drawn in the kernel (noise then optional, written)."""
    f = torch.float32
    if philox is None:
        return (_check(noise, "noise", f, dev, n), None, 0, 0)
    state, off, stride = philox
    return (_opt(noise, "noise", f, dev, n), _check(state, "philox_state", torch.int64, dev, 2),
            int(off), int(stride))


def categorical_sample(logits, noise, action_out=None, logprob_out=None, entropy_out=None,
                       value_in=None, value_out=None, philox=None):
    """argmax(softmax(logits) / noise) with log_prob and entropy; noise ~ Exp(1) [N, A] (or drawn
    in the kernel: philox = TorchExpStream.philox(t), noise then receives the draws if given)."""
    N, A = logits.shape
    dev = logits.device
    f = torch.float32
    if action_out is None:
        action_out = torch.empty(N, dtype=torch.int64, device=dev)
    if logprob_out is None:
        logprob_out = torch.empty(N, dtype=f, device=dev)
    if (value_in is None) != (value_out is None):
        raise ValueError("value_in and value_out go together")
    call("ocppo_categorical_sample", _stream(dev), _check(logits, "logits", f, dev),
         *_noise_args(noise, philox, N * A, dev), N, A,
         _check(action_out, "action_out", torch.int64, dev, N),
         _check(logprob_out, "logprob_out", f, dev, N), _opt(entropy_out, "entropy_out", f, dev, N),
         _opt(value_in, "value_in", f, dev, N), _opt(value_out, "value_out", f, dev, N))
    return action_out, logprob_out, entropy_out


def policy_head_sample(hidden, w_actor, b_actor, w_critic, b_critic, noise, action_out=None,
                       logprob_out=None, value_out=None, entropy_out=None, logits_out=None,
                       philox=None):
    """Fused actor/critic heads + Categorical sample for a rollout step (no autograd)."""
    N, H = hidden.shape
    A = w_actor.shape[0]
    dev = hidden.device
    f = torch.float32
    if tuple(w_actor.shape) != (A, H) or w_critic.numel() != H or b_actor.numel() != A:
        raise ValueError("head weights do not match hidden")
    if action_out is None:
        action_out = torch.empty(N, dtype=torch.int64, device=dev)
    if logprob_out is None:
        logprob_out = torch.empty(N, dtype=f, device=dev)
    if value_out is None:
        value_out = torch.empty(N, dtype=f, device=dev)
    call("ocppo_policy_head_sample", _stream(dev), _check(hidden, "hidden", f, dev), N, H,
         _check(w_actor, "w_actor", f, dev), _check(b_actor, "b_actor", f, dev, A),
         _check(w_critic, "w_critic", f, dev, H), _check(b_critic, "b_critic", f, dev, 1),
         *_noise_args(noise, philox, N * A, dev), A,
         _check(action_out, "action_out", torch.int64, dev, N),
         _check(logprob_out, "logprob_out", f, dev, N), _opt(entropy_out, "entropy_out", f, dev, N),
         _check(value_out, "value_out", f, dev, N), _opt(logits_out, "logits_out", f, dev, N * A))
    return action_out, logprob_out, value_out


def policy_head_env_ok(hidden, w_actor, w_critic, env) -> bool:
    """policy_head_env_step applies: the E = 1 head form and an object-frame synthetic env."""
    N, H = hidden.shape
    A = w_actor.shape[0]
    fr = getattr(env, "frame", None)
    return (getattr(env, "synthetic", False) and fr is not None and fr.dtype == torch.float32
            and fr.is_contiguous() and 1 <= fr.shape[1] <= 4096 and fr.shape[0] == N
            and 1 <= N <= (3072 if H <= 512 else 2048) and H % 256 == 0 and 256 <= H <= 1024
            and 1 <= A <= 7 and hidden.is_contiguous() and w_actor.is_contiguous()
            and w_critic.is_contiguous()
            and (hidden.data_ptr() | w_actor.data_ptr() | w_critic.data_ptr()) % 16 == 0)


def policy_head_env_step(hidden, w_actor, b_actor, w_critic, b_critic, noise, action_out,
                         logprob_out, value_out, env, step_offset: int, philox=None):
    """policy_head_sample + env.step(action_out, step_offset) in one launch
    (ocppo_policy_head_env_step; env a SyntheticAtariEnv with object frames)."""
    N, H = hidden.shape
    A = w_actor.shape[0]
    dev = hidden.device
    f = torch.float32
    if tuple(w_actor.shape) != (A, H) or w_critic.numel() != H or b_actor.numel() != A:
        raise ValueError("head weights do not match hidden")
    D = env.frame.shape[1]
    call("ocppo_policy_head_env_step", _stream(dev), _check(hidden, "hidden", f, dev), N, H,
         _check(w_actor, "w_actor", f, dev), _check(b_actor, "b_actor", f, dev, A),
         _check(w_critic, "w_critic", f, dev, H), _check(b_critic, "b_critic", f, dev, 1),
         *_noise_args(noise, philox, N * A, dev), A,
         _check(action_out, "action_out", torch.int64, dev, N),
         _check(logprob_out, "logprob_out", f, dev, N), _check(value_out, "value_out", f, dev, N),
         env.seed & 0xFFFFFFFFFFFFFFFF, _check(env.step_base, "step_base", torch.int64, dev, 1),
         int(step_offset), D, _check(env.frame, "frame", f, dev, N * D),
         _check(env.reward, "reward", f, dev, N), _check(env.done, "done", f, dev, N),
         _opt(env.ep_state, "ep_state", f, dev, N * 5))
    return action_out, logprob_out, value_out


class _CategoricalLogProbEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, actions):
        N, A = logits.shape
        dev = logits.device
        lp = torch.empty(N, dtype=torch.float32, device=dev)
        ent = torch.empty(N, dtype=torch.float32, device=dev)
        lg = logits.detach().contiguous()
        act = actions.detach().reshape(-1).long().contiguous()
        call("ocppo_categorical_logprob_entropy", _stream(dev),
             _check(lg, "logits", torch.float32, dev), _check(act, "actions", torch.int64, dev, N),
             N, A, lp.data_ptr(), ent.data_ptr())
        ctx.save_for_backward(lg, act)
        return lp, ent

    @staticmethod
    def backward(ctx, g_lp, g_ent):
        lg, act = ctx.saved_tensors
        N, A = lg.shape
        dev = lg.device
        dl = torch.empty_like(lg)
        g_lp = None if g_lp is None else g_lp.contiguous()
        g_ent = None if g_ent is None else g_ent.contiguous()
        call("ocppo_categorical_logprob_entropy_bwd", _stream(dev), lg.data_ptr(), act.data_ptr(),
             _opt(g_lp, "grad_logprob", torch.float32, dev, N),
             _opt(g_ent, "grad_entropy", torch.float32, dev, N), N, A, dl.data_ptr())
        return dl, None


def categorical_logprob_entropy(logits, actions):
    """(log_prob(actions), entropy()) of Categorical(logits=logits), differentiable in logits."""
    return _CategoricalLogProbEntropy.apply(logits, actions)


# ---------------------------------------------------------------------------------------------
# rollout store / reset (ppo_atari_oc.py:502-503, 512-514), minibatch gather (:566-567)
# ---------------------------------------------------------------------------------------------
def _reset_prev(reset_prev, frame, N: int, W: int, D: int, dev):
    if reset_prev is None:
        return None
    if reset_prev.dtype != frame.dtype:
        raise ValueError(f"reset_prev dtype {reset_prev.dtype} != frame dtype {frame.dtype}")
    return _check(reset_prev, "reset_prev", None, dev, N * (W - 1) * D)


def rollout_store(frame, reward, done, prev_obs, obs_out, net_obs=None, reward_out=None,
                  done_out=None, scale255: bool = False, reset_prev=None):
    """obs_out = stack(prev_obs[:, 1:], frame) (reset-filled where done), plus reward/done rows.

    frame [N, D] f32|u8; prev_obs/obs_out [N, W, D] f32|bf16|u8; net_obs [N, W, D] f32, or a
    channels_last [N, W, H, X] f32 tensor (written in NHWC order). scale255: net_obs holds
    value / 255 exactly as the NatureCNN's NormalizeImg computes it on the GPU. reset_prev
    [N, W-1, D] (frame dtype): the older frames of the env's own reset observation for done rows
    (None: FrameStack's fill with the newest frame).
    """
    N, D = frame.shape[0], frame[0].numel()
    W = obs_out.shape[1]
    dev = frame.device
    if tuple(obs_out.shape[:2]) != (N, W) or obs_out[0, 0].numel() != D:
        raise ValueError(f"obs_out {tuple(obs_out.shape)} does not match frame {tuple(frame.shape)}")
    if prev_obs.shape != obs_out.shape or prev_obs.dtype != obs_out.dtype:
        raise ValueError("prev_obs and obs_out must have the same shape and dtype")
    if frame.dtype not in (torch.float32, torch.uint8) or obs_out.dtype not in _DTYPE_CODE:
        raise ValueError(f"unsupported dtypes frame={frame.dtype} obs={obs_out.dtype}")
    f = torch.float32
    net, layout = _net_obs(net_obs, N, W, D, dev)
    call("ocppo_rollout_store", _stream(dev), _check(frame, "frame", None, dev),
         _DTYPE_CODE[frame.dtype], _check(reward, "reward", f, dev, N),
         _check(done, "done", f, dev, N), N, W, D, _check(prev_obs, "prev_obs", None, dev),
         _check(obs_out, "obs_out", None, dev), _DTYPE_CODE[obs_out.dtype], net,
         _opt(reward_out, "reward_out", f, dev, N), _opt(done_out, "done_out", f, dev, N),
         layout | (2 if scale255 else 0), _reset_prev(reset_prev, frame, N, W, D, dev))


def rollout_store_vecnorm(frame, reward, done, prev_obs, obs_out, net_obs, done_out, ret_state,
                          rms_state, reward_out, gamma=0.99, epsilon=1e-8, clip_reward=10.0,
                          scale255: bool = False, reset_prev=None):
    """rollout_store + vecnorm_reward in one launch (reward_out gets the normalised reward)."""
    N, D = frame.shape[0], frame[0].numel()
    W = obs_out.shape[1]
    dev = frame.device
    if prev_obs.shape != obs_out.shape or prev_obs.dtype != obs_out.dtype:
        raise ValueError("prev_obs and obs_out must have the same shape and dtype")
    if tuple(obs_out.shape[:2]) != (N, W) or obs_out[0, 0].numel() != D:
        raise ValueError(f"obs_out {tuple(obs_out.shape)} does not match frame {tuple(frame.shape)}")
    f = torch.float32
    net, layout = _net_obs(net_obs, N, W, D, dev)
    call("ocppo_rollout_store_vecnorm", _stream(dev), _check(frame, "frame", None, dev),
         _DTYPE_CODE[frame.dtype], _check(reward, "reward", f, dev, N),
         _check(done, "done", f, dev, N), N, W, D, _check(prev_obs, "prev_obs", None, dev),
         _check(obs_out, "obs_out", None, dev), _DTYPE_CODE[obs_out.dtype], net,
         _opt(done_out, "done_out", f, dev, N),
         float(gamma), float(epsilon), float(clip_reward),
         _check(ret_state, "ret_state", torch.float64, dev, N),
         _check(rms_state, "rms_state", torch.float64, dev, 3),
         _check(reward_out, "reward_out", f, dev, N), layout | (2 if scale255 else 0),
         _reset_prev(reset_prev, frame, N, W, D, dev))


def obs_reset(frame, obs_out, net_obs=None, scale255: bool = False):
    N, D = frame.shape[0], frame[0].numel()
    W = obs_out.shape[1]
    dev = frame.device
    if obs_out.numel() != N * W * D:
        raise ValueError("obs_out does not match frame")
    net, layout = _net_obs(net_obs, N, W, D, dev)
    call("ocppo_obs_reset", _stream(dev), _check(frame, "frame", None, dev),
         _DTYPE_CODE[frame.dtype], N, W, D, _check(obs_out, "obs_out", None, dev),
         _DTYPE_CODE[obs_out.dtype], net, layout | (2 if scale255 else 0))


def linear_act(x, weight, bias=None, relu: bool = False, out=None, ring=None):
    """y = act(x @ weight.T + bias) on the f32 matrix cores, for rollout-sized batches (no
    autograd). x [M, K] f32 with unit column stride (row stride may exceed K, e.g. a frame slice
    of the stacked obs); weight [N, K] contiguous (nn.Linear.weight); bias [N] or None.
    ring = (seg, rot): x's rows are K / seg segments stored rotated, logical segment s at
    physical (s + rot) mod (K / seg) (the frame-encoding ring, ocppo_linear_act_ring)."""
    if x.dim() != 2 or weight.dim() != 2:
        raise ValueError(f"x must be [M, K] and weight [N, K], got {tuple(x.shape)}, "
                         f"{tuple(weight.shape)}")
    M, K = x.shape
    N = weight.shape[0]
    dev = x.device
    if weight.shape[1] != K:
        raise ValueError(f"weight is {tuple(weight.shape)}, x has K={K}")
    if x.dtype != torch.float32 or (M > 1 and x.stride(1) != 1) or x.device.type != "cuda":
        raise ValueError("x must be an f32 GPU tensor with unit column stride")
    ldx = x.stride(0) if M > 1 else K
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=dev)
    if tuple(out.shape) != (M, N) or (M > 1 and out.stride(1) != 1) or out.dtype != torch.float32:
        raise ValueError("out must be an f32 [M, N] tensor with unit column stride")
    ldy = out.stride(0) if M > 1 else N
    if ring is not None:
        seg, rot = (int(v) for v in ring)
        call("ocppo_linear_act_ring", _stream(dev), x.data_ptr(), ldx,
             _check(weight, "weight", torch.float32, dev), _opt(bias, "bias", torch.float32, dev, N),
             out.data_ptr(), ldy, M, N, K, seg, rot, 1 if relu else 0)
        return out
    call("ocppo_linear_act", _stream(dev), x.data_ptr(), ldx,
         _check(weight, "weight", torch.float32, dev), _opt(bias, "bias", torch.float32, dev, N),
         out.data_ptr(), ldy, M, N, K, 1 if relu else 0)
    return out


def conv2d_act(x, weight, bias=None, stride: int = 1, relu: bool = True, out=None):
    """act(conv2d(x, weight, bias, stride)) on the f32 matrix cores (ocppo_conv2d_act) for
    channels_last tensors: x [B, Cin, H, W] and weight [Cout, Cin, KH, KW] both in
    torch.channels_last memory format; no padding / dilation / groups. Returns [B, Cout, OH, OW]
    in channels_last (no autograd: the rollout forward)."""
    B, Cin, H, W = x.shape
    Cout, Cw, KH, KW = weight.shape
    dev = x.device
    f = torch.float32
    cl = torch.channels_last
    if Cw != Cin or x.dtype != f or weight.dtype != f or x.device.type != "cuda":
        raise ValueError("conv2d_act: f32 GPU x [B, Cin, H, W] and weight [Cout, Cin, KH, KW]")
    if not (x.is_contiguous(memory_format=cl) and weight.is_contiguous(memory_format=cl)):
        raise ValueError("conv2d_act: x and weight must be channels_last")
    OH, OW = (H - KH) // stride + 1, (W - KW) // stride + 1
    if out is None:
        out = torch.empty((B, Cout, OH, OW), dtype=f, device=dev, memory_format=cl)
    if tuple(out.shape) != (B, Cout, OH, OW) or not out.is_contiguous(memory_format=cl):
        raise ValueError("conv2d_act: out must be a channels_last [B, Cout, OH, OW] tensor")
    call("ocppo_conv2d_act", _stream(dev), x.data_ptr(), B, H, W, Cin, weight.data_ptr(),
         _opt(bias, "bias", f, dev, Cout), Cout, KH, KW, stride, out.data_ptr(), int(bool(relu)))
    return out


# ---- NHWC convolutions as implicit GEMMs on the x6 products (ocppo_conv_x6) ---------------------
# The NatureCNN trunk (architectures/ppo.py:20-31) without MIOpen: forward, weight gradient and
# data gradient, deterministic (split-K partials summed in split order), f32-level products.
_CONV_TILES = {0: (128, 32), 1: (32, 128), 2: (128, 64), 3: (64, 64), 4: (64, 128), 5: (128, 128),
               6: (32, 64)}


CONV_FWD_MIN_UNITS = 512


def _conv_fwd_tile(M: int, N: int) -> int | None:
    """The largest tile giving >= CONV_FWD_MIN_UNITS workgroups (two per CU), else the one giving
    the most."""
    best, units = None, 0
    for t in ((0,) if N == 32 else (2, 3, 6) if N == 64 else (5, 2, 3, 6)):
        bm, bn = _CONV_TILES[t]
        if M % bm == 0 and N % bn == 0:
            u = (M // bm) * (N // bn)
            if u >= CONV_FWD_MIN_UNITS:
                return t
            if u > units:
                best, units = t, u
    return best


def _conv_wgrad_tile(M: int, N: int) -> int | None:
    for t in ((1,) if M == 32 else (4, 3) if M == 64 else (5, 4, 3)):
        bm, bn = _CONV_TILES[t]
        if M % bm == 0 and N % bn == 0:
            return t
    return None


def conv_x6_ok(x, weight, stride: int, wgrad: bool = False, dgrad: bool = False) -> bool:
    """Shapes ocppo_conv_x6 takes: channels_last f32 x [B, C, H, W] and weight [Cout, C, KH, KW]
    (square stride, no padding), C % 4 == 0, kernel rows of KW C % 32 == 0 taps, row counts the
    tiles divide; wgrad / dgrad: also the weight gradient / the data gradient's stride classes."""
    if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and weight.dim() == 4 and weight.dtype == torch.float32):
        return False
    cl = torch.channels_last
    if not (x.is_contiguous(memory_format=cl) and weight.is_contiguous(memory_format=cl)):
        return False
    B, C, H, W = x.shape
    Cout, Cw, KH, KW = weight.shape
    s = int(stride)
    if Cw != C or C % 4 or (KW * C) % 32 or H < KH or W < KW or (H - KH) % s or (W - KW) % s:
        return False
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    rows = B * OH * OW
    if rows >= 1 << 24 or _conv_fwd_tile(rows, Cout) is None:
        return False
    if wgrad and (OH * OW > 1024 or rows % 32 or _conv_wgrad_tile(Cout, KH * KW * C) is None):
        return False
    if dgrad:
        if KH % s or KW % s or H % s or W % s or Cout % 4 or ((KW // s) * Cout) % 32:
            return False
        qrows = B * (H // s) * (W // s)
        return qrows < 1 << 24 and _conv_fwd_tile(qrows, s * s * C) is not None
    return True


_CONV_PARTS: dict = {}
# weight gradients: K splits for about this many workgroups (each split's partial [Cout, N] summed
# in split order by the same launch's sum_parts), per tile; measured at config 3's minibatch of
# 8192 (profiles/r05/ab_conv_wgrad_units.txt): 32 x 128 (the first layer) and 64 x 128 best at
# 1024, 64 x 64 at 4096. None: the per-tile table; an int: one target for every tile
CONV_WGRAD_UNITS = None
_WGRAD_UNITS = {1: 1024, 4: 1024, 3: 4096}


def _wgrad_units(tile: int) -> int:
    return CONV_WGRAD_UNITS if CONV_WGRAD_UNITS else _WGRAD_UNITS.get(tile, 2048)


def _geom(*v):
    return (ctypes.c_int64 * len(v))(*[int(t) for t in v])


# Bounds-check builds of the library (`python tools/build_variant.py OUT.so -DOCPPO_X6_BOUNDS`,
# loaded with OCPPO_LIB=OUT.so; never the product): before every convolution launch the library
# is handed the extents of the sources its gathers read, from the pointers it is passed, and a
# device record of the first out-of-range index (tests/test_conv_bounds_gpu.py reads it).
X6_BOUNDS = hasattr(_lib.LIB, "ocppo_x6_probe_set_bounds")
_BOUNDS_REC: dict = {}
BOUND_KINDS = {1: "f32 source offset", 2: "image index", 3: "u8 stack row", 4: "u8 byte offset"}


def _tail(t) -> int:
    """Elements of t's storage from t's first element on."""
    return t.untyped_storage().nbytes() // t.element_size() - t.storage_offset()


def bounds_record(dev) -> torch.Tensor:
    """The bounds-check build's violation record on `dev` (int32 [count, first kind, first index
    lo, hi, its limit lo, hi, 0, 0])."""
    key = str(dev)
    if key not in _BOUNDS_REC:
        _BOUNDS_REC[key] = torch.zeros(8, dtype=torch.int32, device=dev)
    return _BOUNDS_REC[key]


def _bounds(dev, x=None, u8=None):
    if X6_BOUNDS:
        _lib.LIB.ocppo_x6_probe_set_bounds.argtypes = [ctypes.c_void_p, ctypes.c_int64,
                                                       ctypes.c_int64, ctypes.c_int64]
        _lib.LIB.ocppo_x6_probe_set_bounds(
            bounds_record(dev).data_ptr(), _tail(x) if x is not None else 0,
            _tail(u8) if u8 is not None else 0, u8.shape[0] if u8 is not None else 0)


def _conv_rows_form(M: int, Cout: int) -> bool:
    """conv_x6 takes the few-rows form (ocppo_conv_x6 tile 7) for this product."""
    return CONV_FWD_ROWS and M <= CONV_FWD_ROWS_MAX and Cout in (32, 64) and M % 32 == 0


def _conv_planes_ptr(w_planes, N: int, K: int, dev):
    if w_planes is None:
        return None
    if w_planes.dtype != torch.bfloat16 or tuple(w_planes.shape) != (3, N, K) or \
            not w_planes.is_contiguous():
        raise ValueError(f"conv_x6: w_planes must be contiguous bf16 [3, {N}, {K}]")
    return _check(w_planes, "w_planes", torch.bfloat16, dev)


def conv_x6(x, weight, bias=None, stride: int = 1, relu: bool = True, out=None, w_planes=None,
            mbits=None):
    """act(conv2d(x, weight) + bias) (architectures/ppo.py:20-31's Conv2d + ReLU) on ocppo_conv_x6:
    channels_last f32 x [B, C, H, W], weight [Cout, C, KH, KW] -> channels_last [B, Cout, OH, OW]
    (no autograd; agents._ConvX6 is the autograd form). w_planes: the weight's [Cout, KH KW C]
    matrix pre-split into bf16 [3, Cout, KH KW C] (ocppo_split_planes: the same pieces as the
    in-kernel split, so the same bits). mbits: an int32 [B OH OW Cout / 32] tensor the tile loop's
    epilogue fills with the output's ReLU mask, row-major (relu_bias_grad's bits= form); the
    few-rows form (no autograd) takes none."""
    if not conv_x6_ok(x, weight, stride):
        raise ValueError(f"conv_x6: unsupported shapes x {tuple(x.shape)}, weight "
                         f"{tuple(weight.shape)}, stride {stride} (conv_x6_ok)")
    B, C, H, W = x.shape
    Cout, _, KH, KW = weight.shape
    s = int(stride)
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    dev, f = x.device, torch.float32
    K = KH * KW * C
    M = B * OH * OW
    wm = weight.permute(0, 2, 3, 1).reshape(Cout, K)  # a view: [Cout, KH, KW, C] in memory
    if out is None:
        out = torch.empty((B, Cout, OH, OW), dtype=f, device=dev, memory_format=torch.channels_last)
    if tuple(out.shape) != (B, Cout, OH, OW) or not out.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv_x6: out must be a channels_last [B, Cout, OH, OW] tensor")
    geom = _geom(OH, OW, H * W * C, s * W * C, s * C, W * C, KW * C)
    if _conv_rows_form(M, Cout):
        # few rows (the rollout's batch): K steps split over the waves of a workgroup
        if mbits is not None:
            raise ValueError("conv_x6: the few-rows form writes no ReLU bitmask")
        _bounds(dev, x)
        call("ocppo_conv_x6", _stream(dev), 0, x.data_ptr(), geom, wm.data_ptr(), K,
             out.data_ptr(), Cout, M, Cout, K, 1, _opt(bias, "bias", f, dev, Cout),
             int(bool(relu)), None, 7, None, None, None, None,
             _conv_planes_ptr(w_planes, Cout, K, dev), None)
        return out
    tile = _conv_fwd_tile(M, Cout)
    bm, bn = _CONV_TILES[tile]
    S = _conv_fwd_splits((M // bm) * (Cout // bn), K // 32)
    _bounds(dev, x)
    wpp = _conv_planes_ptr(w_planes, Cout, K, dev)
    if mbits is not None and (S != 1 or not relu or Cout % 32):
        raise ValueError("conv_x6: mbits needs one product with relu, 32 | Cout")
    if S == 1:
        call("ocppo_conv_x6", _stream(dev), 0, x.data_ptr(), geom, wm.data_ptr(), K,
             out.data_ptr(), Cout, M, Cout, K, 1, _opt(bias, "bias", f, dev, Cout),
             int(bool(relu)), None, tile, None, None, None, None, wpp,
             _opt(mbits, "mbits", torch.int32, dev, M * Cout // 32))
        return out
    # few rows (the rollout's batch): K-split partials, then bias + ReLU on their ordered sum
    key = ("fwd", str(dev), S, M, Cout)
    if key not in _CONV_PARTS:
        _CONV_PARTS[key] = torch.empty((S, M, Cout), dtype=f, device=dev)
    part = _CONV_PARTS[key]
    call("ocppo_conv_x6", _stream(dev), 0, x.data_ptr(), geom, wm.data_ptr(), K, part.data_ptr(),
         Cout, M, Cout, K, S, None, 0, None, tile, None, None, None, None, wpp, None)
    call("ocppo_sum_splits_act", _stream(dev), part.data_ptr(), S, M, Cout,
         _opt(bias, "bias", f, dev, Cout), int(bool(relu)), out.data_ptr())
    return out


# Forward products of at most CONV_FWD_ROWS_MAX rows (the rollout's batch: 20736 / 12544 rows for
# NatureCNN's second / third layer at 256 envs) on ocppo_conv_x6 tile 7: a 32-row tile per
# workgroup, its K steps split over 8 waves and summed through LDS in wave order, instead of the
# tile loop's chain of 16-18 dependent K steps on 2 waves
CONV_FWD_ROWS = True
CONV_FWD_ROWS_MAX = 65536


# K splits for a forward product of few workgroups (< 512; the rollout's image batch): measured
# no faster at 256 envs (conv + ordered sum 23.8 / 24.6 / 25.4 us vs 23.5 / 24.5 / 25.1 us in one
# launch), so off by default
CONV_FWD_SPLITS = False


def _conv_fwd_splits(units: int, steps: int) -> int:
    if not CONV_FWD_SPLITS or units >= 512:
        return 1
    S = 1
    for c in (2, 4, 8):
        if steps // c < 3:
            break
        S = c
        if units * c >= 1024:
            break
    return S


def conv_x6_wgrad(gp, x, kernel: tuple, stride: int, out=None):
    """dW of a convolution (channels_last weight layout [Cout, KH, KW, C] as a [Cout, KH KW C]
    matrix): sum over the output pixels r of gp[r, co] x(r, (ky, kx, c)); gp [B OH OW, Cout] the
    output gradient's NHWC rows, x the channels_last input. Split-K partials summed in order."""
    B, C, H, W = x.shape
    KH, KW = kernel
    s = int(stride)
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    rows, Cout = gp.shape
    dev, f = x.device, torch.float32
    if rows != B * OH * OW or not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv_x6_wgrad: gp must be [B OH OW, Cout], x channels_last")
    N = KH * KW * C
    tile = _conv_wgrad_tile(Cout, N)
    if tile is None or rows % 32:
        raise ValueError(f"conv_x6_wgrad: no tile for [{Cout} x {N}] over {rows} rows")
    bm, bn = _CONV_TILES[tile]
    tiles = (Cout // bm) * (N // bn)
    S = max(1, min(rows // 32 // 32, _wgrad_units(tile) // tiles))
    key = ("wgrad", str(dev), S, Cout, N)
    if key not in _CONV_PARTS:
        _CONV_PARTS[key] = torch.empty((S, Cout, N), dtype=f, device=dev)
    part = _CONV_PARTS[key]
    if out is None:
        out = torch.empty((Cout, N), dtype=f, device=dev)
    if out.numel() != Cout * N or not out.is_contiguous(memory_format=torch.channels_last
                                                        if out.dim() == 4 else torch.contiguous_format):
        raise ValueError("conv_x6_wgrad: out must hold [Cout, KH KW C] contiguously")
    _bounds(dev, x)
    call("ocppo_conv_x6", _stream(dev), 1, x.data_ptr(),
         _geom(OH, OW, H * W * C, s * W * C, s * C, W * C, KW * C),
         _check(gp, "gp", f, dev), Cout, part.data_ptr(), N, Cout, N, rows, S, None, 0, None, tile,
         out.data_ptr(), None, None, None, None, None)
    return out


def conv_x6_dgrad_fuses_relu(M: int, C: int, stride: int) -> bool:
    """conv_x6_dgrad can take the layer below's ReLU backward (the bounded loader's tiles)."""
    return not CONV_DGRAD_PAD_COPY and _conv_fwd_tile(M, stride * stride * C) in (2, 3, 5, 6)


def conv_x6_dgrad(gp, weight, stride: int, in_hw: tuple, out=None, relu_out=None, db=None):
    """dX of a convolution: gp channels_last [B, Cout, OH, OW] (the output gradient), weight
    [Cout, C, KH, KW] -> channels_last [B, C, H, W]. Per stride class (py, px) a forward-form
    product over gp zero-padded by KH / s - 1 with that class's taps flipped; each input pixel
    gets its <= (KH / s)^2 taps in one fixed order (deterministic). relu_out: the layer below's
    ReLU output (channels_last [B, C, H, W]): its ReLU backward in the epilogue (dX masked where
    relu_out <= 0) and its bias gradient (the masked dX's per-channel sums, row tiles and classes
    added in order in f64) into db [C]."""
    B, Cout, OH, OW = gp.shape
    _, C, KH, KW = weight.shape
    H, W = in_hw
    s = int(stride)
    T, TW = KH // s, KW // s
    dev, f = gp.device, torch.float32
    g = gp.permute(0, 2, 3, 1)  # NHWC view
    if not g.is_contiguous():
        g = g.contiguous()
    Hp, Wp = OH + 2 * (T - 1), OW + 2 * (TW - 1)
    QH, QW = H // s, W // s
    M, K = B * QH * QW, T * TW * Cout
    N = s * s * C  # every stride class's C channels: the classes read the same gradient rows
    tile = _conv_fwd_tile(M, N)
    if CONV_DGRAD_TILE and M % _CONV_TILES[CONV_DGRAD_TILE][0] == 0 and \
            N % _CONV_TILES[CONV_DGRAD_TILE][1] == 0:
        tile = CONV_DGRAD_TILE
    if out is None:
        out = torch.empty((B, C, H, W), dtype=f, device=dev, memory_format=torch.channels_last)
    if tuple(out.shape) != (B, C, H, W) or not out.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv_x6_dgrad: out must be a channels_last [B, C, H, W] tensor")
    # class (py, px)'s taps ky = py + s t, flipped (t' = T - 1 - t), as [C, T, TW, Cout] rows;
    # the classes stacked class-major: B = [s s C, K] -- one gather through a cached index into
    # the weight's memory (its [Cout, KH, KW, C] order when channels_last) instead of s^2 flips,
    # a stack and a layout copy per call
    wc, wcp = _dgrad_weight(weight, s, planes=CONV_DGRAD_PLANES and
                            (tile != 5 or CONV_DGRAD_PLANES_128))
    wpp = None if wcp is None else wcp.data_ptr()
    og = None if s == 1 else _geom(H * W * C, s * W * C, s * C, 0, C, s, W * C, C)
    if CONV_DGRAD_PAD_COPY or tile not in (2, 3, 5, 6):
        gpad = torch.nn.functional.pad(g, (0, 0, TW - 1, TW - 1, T - 1, T - 1))
        if relu_out is not None:
            raise ValueError("conv_x6_dgrad: the ReLU epilogue needs the bounded loader")
        _bounds(dev, gpad)
        call("ocppo_conv_x6", _stream(dev), 0, gpad.data_ptr(),
             _geom(QH, QW, Hp * Wp * Cout, Wp * Cout, Cout, Wp * Cout, TW * Cout), wc.data_ptr(),
             K, out.data_ptr(), C, M, N, K, 1, None, 0, og, tile, None, None, None, None, wpp, None)
        return out
    # the padding as bounds in the loader: taps outside the gradient read as zeros
    mask = dbp = None
    if relu_out is not None:
        if tuple(relu_out.shape) != (B, C, H, W) or not relu_out.is_contiguous(
                memory_format=torch.channels_last) or db is None:
            raise ValueError("conv_x6_dgrad: relu_out must be channels_last [B, C, H, W], with db")
        mask = relu_out
        dbp = torch.empty((M // _CONV_TILES[tile][0], N), dtype=f, device=dev)
    _bounds(dev, g)
    call("ocppo_conv_x6", _stream(dev), 0, g.data_ptr(),
         _geom(QH, QW, 0, 0, 0, 0, TW * Cout), wc.data_ptr(), K, out.data_ptr(), C, M, N, K, 1,
         None, 0, og, tile, None, _geom(T - 1, TW - 1, OH, OW, Cout),
         None if mask is None else mask.data_ptr(), None if dbp is None else dbp.data_ptr(), wpp, None)
    if dbp is not None:
        # row tiles, then stride classes, in order (f64, one rounding)
        db.copy_(dbp.view(-1, s * s, C).double().sum(0).sum(0))
    return out


_DG_IDX: dict = {}
_DG_BUF: dict = {}
# the data gradients' B operand (the stride classes' flipped weights) pre-split into bf16 planes
# once per call (ocppo_split_planes) instead of in every workgroup of the product
CONV_DGRAD_PLANES = True
# ... also on the 128 x 128 tile (the conv2 data gradient's 4 x 32 class columns), whose pre-split
# instance spills (experiments: A/B)
CONV_DGRAD_PLANES_128 = True


def _dgrad_weight(weight, s: int, planes: bool = False):
    """(wc, its bf16 planes or None): conv_x6_dgrad's B operand [s s C, T TW Cout], row (py, px,
    c), column (t, tw, co) = weight[co, c, py + s (T - 1 - t), px + s (TW - 1 - tw)], gathered in
    one launch into a buffer kept per weight (and split into planes by one more)."""
    Cout, C, KH, KW = weight.shape
    mem = weight.permute(0, 2, 3, 1)  # a view of the memory when channels_last
    key = (str(weight.device), Cout, C, KH, KW, s)
    idx = _DG_IDX.get(key)
    if idx is None:
        ar = torch.arange(Cout * KH * KW * C).view(Cout, KH, KW, C).permute(0, 3, 1, 2)
        idx = torch.stack([ar[:, :, py::s, px::s].flip(2, 3).permute(1, 2, 3, 0)
                           for py in range(s) for px in range(s)])
        idx = idx.reshape(s * s * C, -1).to(weight.device)
        _DG_IDX[key] = idx
    bkey = key + (weight.data_ptr(),)
    ent = _DG_BUF.get(bkey)
    if ent is None:
        buf = torch.empty(idx.shape, dtype=torch.float32, device=weight.device)
        ent = [buf, None]
        _DG_BUF[bkey] = ent
    buf = ent[0]
    with torch.no_grad():  # (the kernel timer replays this outside autograd's backward)
        torch.index_select(mem.reshape(-1), 0, idx.view(-1), out=buf.view(-1))
    if not planes or buf.shape[1] % 8:
        return buf, None
    if ent[1] is None:
        ent[1] = WeightPlanes(fwd=(buf,))
    ent[1].refresh()
    return buf, buf._ocppo_planes["fwd"]


# an explicit tile for the data gradients (0: _conv_fwd_tile's choice; experiments)
CONV_DGRAD_TILE = 0


# the data gradient over a zero-padded copy of the output gradient (F.pad: a fill and a copy per
# layer) instead of the bounded loader
CONV_DGRAD_PAD_COPY = False


def conv_x6_u8_ok(src, weight, stride: int, B: int, wgrad: bool = False) -> bool:
    """The first convolution straight from u8 frame stacks src [R, C, H, W] (ocppo_conv_x6_u8):
    KW, W and the stride multiples of 4, no padding, B samples' rows a tile divides."""
    if not (isinstance(src, torch.Tensor) and src.is_cuda and src.dtype == torch.uint8 and
            src.dim() == 4 and src.is_contiguous() and weight.dim() == 4):
        return False
    _, C, H, W = src.shape
    Cout, Cw, KH, KW = weight.shape
    s = int(stride)
    if Cw != C or KW % 4 or W % 4 or s % 4 or H < KH or W < KW or (H - KH) % s or (W - KW) % s:
        return False
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    rows, taps = B * OH * OW, C * KH * KW
    if rows >= 1 << 24 or taps % 32 or taps // 4 > 1024 or _conv_u8_tile(rows, Cout, 0) is None:
        return False
    return not wgrad or (OH * OW <= 1024 and rows % 32 == 0 and
                         _conv_u8_tile(Cout, taps, 1) is not None)


def _conv_u8_tile(M: int, N: int, mode: int) -> int | None:
    for t in (((0,) if N == 32 else (2,) if N == 64 else ()) if mode == 0 else
              ((1,) if M == 32 else (4,) if M == 64 else ())):
        bm, bn = _CONV_TILES[t]
        if M % bm == 0 and N % bn == 0:
            return t
    return None


# The first convolution's forward with each image's u8 stack staged in LDS once (ocppo_conv_x6_u8
# tile 7, conv_u8_img_kernel: bitwise the tile loop's output) where the geometry is NatureCNN's
# first layer (4 x 84 x 84 stacks, 8 x 8 taps, stride 4, 32 channels)
CONV_U8_IMG = True


def _conv_u8_img_ok(src, weight, stride: int) -> bool:
    _, C, H, W = src.shape
    Cout, _, KH, KW = weight.shape
    OH, OW = (H - KH) // stride + 1, (W - KW) // stride + 1
    return (CONV_U8_IMG and C == 4 and KH == 8 and KW == 8 and stride == 4 and Cout == 32 and
            (OH * OW) % 16 == 0 and (C * H * W) % 16 == 0 and 2 * C * H * W <= 65536 and
            src.data_ptr() % 16 == 0)


def conv_x6_u8(src, idx, weight, bias=None, stride: int = 4, relu: bool = True,
               divisor: float = 255.0, out=None, tile: int | None = None, mbits=None,
               wn=None):
    """act(conv2d(src[idx] / divisor, weight) + bias) with the u8 frame stacks read in place
    (ocppo_conv_x6_u8): src [R, C, H, W] u8, idx [B] int64 -> channels_last [B, Cout, OH, OW].
    tile: None = the image-staged kernel where it applies (CONV_U8_IMG), else the tile loop's;
    an explicit ocppo_conv_x6_u8 tile forces that form (tests). mbits: an int32 [B OH OW] tensor
    the image-staged kernel fills with the output's ReLU mask (bit co of row r = out > 0), for
    conv_x6_u8_wgrad's fused ReLU backward. wn: the weight already in nn.Conv2d's contiguous
    (c, ky, kx) tap order (a cached copy of a channels_last weight), else made here."""
    B = idx.numel()
    if not conv_x6_u8_ok(src, weight, stride, B):
        raise ValueError(f"conv_x6_u8: unsupported src {tuple(src.shape)} / weight "
                         f"{tuple(weight.shape)} / stride {stride} / {B} samples")
    _, C, H, W = src.shape
    Cout, _, KH, KW = weight.shape
    s = int(stride)
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    dev, f = src.device, torch.float32
    K, M = C * KH * KW, B * OH * OW
    if wn is None:
        wn = weight.contiguous()  # nn.Conv2d's (c, ky, kx) tap order
    elif tuple(wn.shape) != tuple(weight.shape) or not wn.is_contiguous():
        raise ValueError("conv_x6_u8: wn must be the weight as a contiguous tensor")
    if out is None:
        out = torch.empty((B, Cout, OH, OW), dtype=f, device=dev, memory_format=torch.channels_last)
    if tuple(out.shape) != (B, Cout, OH, OW) or not out.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv_x6_u8: out must be a channels_last [B, Cout, OH, OW] tensor")
    _bounds(dev, u8=src)
    if tile is None:
        tile = 7 if _conv_u8_img_ok(src, weight, s) else _conv_u8_tile(M, Cout, 0)
    if mbits is not None and (tile != 7 or not relu):
        raise ValueError("conv_x6_u8: mbits needs the image-staged kernel (tile 7) and relu")
    call("ocppo_conv_x6_u8", _stream(dev), 0, src.data_ptr(), _check(idx, "idx", torch.int64, dev, B),
         C, H, W, KH, KW, s, wn.data_ptr(), K, out.data_ptr(), M, Cout, K, 1,
         _opt(bias, "bias", f, dev, Cout), int(bool(relu)), float(divisor), tile, None,
         _opt(mbits, "mbits", torch.int32, dev, M), None, None)
    return out


# ... and its weight gradient (ocppo_conv_x6_u8 tile 8, conv_u8_wgrad_img_kernel: each image's
# stack in LDS once, rewritten per channel as tap-column rows; 4 partials per workgroup summed in
# order) for NatureCNN's first layer on 4 x 84 x 84 stacks
CONV_U8_IMG_WGRAD = True
_CUS: dict = {}


def _cus(dev) -> int:
    if str(dev) not in _CUS:
        _CUS[str(dev)] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CUS[str(dev)]


def _conv_u8_img_wgrad_ok(src, kernel, stride: int, Cout: int) -> bool:
    _, C, H, W = src.shape
    return (CONV_U8_IMG_WGRAD and C == 4 and H == 84 and W == 84 and tuple(kernel) == (8, 8) and
            stride == 4 and Cout == 32 and src.data_ptr() % 16 == 0)


def conv_x6_u8_wgrad(gp, src, idx, kernel: tuple, stride: int = 4, divisor: float = 255.0,
                     out=None, tile: int | None = None, mbits=None, db=None):
    """dW [Cout, C KH KW] (nn.Conv2d's tap order) of conv_x6_u8: sum over the output pixels r of
    gp[r, co] src[idx[b], c, s oy + ky, s ox + kx] / divisor; split partials summed in order.
    tile: None = the image-staged kernel where it applies (CONV_U8_IMG_WGRAD), else the tile
    loop's; an explicit ocppo_conv_x6_u8 tile forces that form (tests). Image-staged kernel only:
    mbits (conv_x6_u8's ReLU mask) makes gp the UNMASKED output gradient, masked in the kernel
    (relu_bias_grad's ReLU backward); db [Cout] receives the masked gradient's column sums (the
    bias gradient)."""
    B = idx.numel()
    _, C, H, W = src.shape
    KH, KW = kernel
    s = int(stride)
    OH, OW = (H - KH) // s + 1, (W - KW) // s + 1
    rows, Cout = gp.shape
    dev, f = src.device, torch.float32
    N = C * KH * KW
    if tile is None and _conv_u8_img_wgrad_ok(src, kernel, s, Cout):
        tile = 8
    if (mbits is not None or db is not None) and tile != 8:
        raise ValueError("conv_x6_u8_wgrad: mbits / db need the image-staged kernel (tile 8)")
    if tile == 8:
        if rows != B * OH * OW:
            raise ValueError("conv_x6_u8_wgrad: gp must be [B OH OW, Cout]")
        S = 4 * min(_cus(dev), B)  # 4 wave partials per workgroup, <= one workgroup per image
        key = ("wgrad_img", str(dev), S, Cout, N)
        if key not in _CONV_PARTS:
            _CONV_PARTS[key] = torch.empty((S, Cout, N), dtype=f, device=dev)
        part = _CONV_PARTS[key]
        if out is None:
            out = torch.empty((Cout, N), dtype=f, device=dev)
        dbp = None
        if db is not None:
            dkey = ("wgrad_img_db", str(dev), S, Cout)
            if dkey not in _CONV_PARTS:
                _CONV_PARTS[dkey] = torch.empty((S, Cout), dtype=f, device=dev)
            dbp = _CONV_PARTS[dkey].data_ptr()
        _bounds(dev, u8=src)
        call("ocppo_conv_x6_u8", _stream(dev), 1, src.data_ptr(),
             _check(idx, "idx", torch.int64, dev, B), C, H, W, KH, KW, s,
             _check(gp, "gp", f, dev), Cout, part.data_ptr(), Cout, N, rows, S, None, 0,
             float(divisor), 8, _check(out, "out", f, dev, Cout * N),
             _opt(mbits, "mbits", torch.int32, dev, rows), dbp, _opt(db, "db", f, dev, Cout))
        return out
    tile = _conv_u8_tile(Cout, N, 1) if tile is None else tile
    if rows != B * OH * OW or tile is None or rows % 32:
        raise ValueError("conv_x6_u8_wgrad: gp must be [B OH OW, Cout] with a tile for it")
    bm, bn = _CONV_TILES[tile]
    S = max(1, min(rows // 32 // 32, _wgrad_units(tile) // ((Cout // bm) * (N // bn))))
    key = ("wgrad", str(dev), S, Cout, N)
    if key not in _CONV_PARTS:
        _CONV_PARTS[key] = torch.empty((S, Cout, N), dtype=f, device=dev)
    part = _CONV_PARTS[key]
    if out is None:
        out = torch.empty((Cout, N), dtype=f, device=dev)
    _bounds(dev, u8=src)
    call("ocppo_conv_x6_u8", _stream(dev), 1, src.data_ptr(), _check(idx, "idx", torch.int64, dev, B),
         C, H, W, KH, KW, s, _check(gp, "gp", f, dev), Cout, part.data_ptr(), Cout, N, rows, S,
         None, 0, float(divisor), tile, _check(out, "out", f, dev, Cout * N), None, None, None)
    return out


def linear2_act(x, w1, b1, w2, b2, relu1: bool = True, relu2: bool = True, out=None):
    """y = act2(act1(x @ w1.T + b1) @ w2.T + b2) in ONE launch for rollout-sized batches (no
    autograd): x [M, K1] f32 (unit column stride, K1 <= 64), w1 [N1, K1], w2 [N2, N1]
    (N1 % 16 == 0, N1 <= 512)."""
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("x must be [M, K1] with unit column stride")
    M, K1 = x.shape
    N1, N2 = w1.shape[0], w2.shape[0]
    if w1.shape[1] != K1 or w2.shape[1] != N1:
        raise ValueError(f"shapes: x {tuple(x.shape)}, w1 {tuple(w1.shape)}, w2 {tuple(w2.shape)}")
    dev = x.device
    f = torch.float32
    if out is None:
        out = torch.empty((M, N2), dtype=f, device=dev)
    if x.dtype != f or x.device.type != "cuda":
        raise ValueError("x must be a float32 GPU tensor")
    call("ocppo_linear2_act", _stream(dev), x.data_ptr(), x.stride(0) if M > 1 else K1,
         _check(w1, "w1", f, dev), _opt(b1, "b1", f, dev, N1), _check(w2, "w2", f, dev),
         _opt(b2, "b2", f, dev, N2), _check(out, "out", f, dev, M * N2), N2, M, N1, N2, K1,
         int(bool(relu1)), int(bool(relu2)))
    return out


def linear_cache_shift(x, weight, bias, enc, done=None, relu: bool = True):
    """The rollout's last encoder layer and the frame-encoding cache shift in one launch:
    fresh = act(x @ weight.T + bias) (x [M, K] f32, unit column stride; weight [E, K]) shifts
    enc [M, W, E] like ops.frame_cache_shift(enc, fresh, done) without storing fresh."""
    if x.dim() != 2 or weight.dim() != 2 or enc.dim() != 3:
        raise ValueError(f"x [M, K], weight [E, K], enc [M, W, E] expected, got {tuple(x.shape)}, "
                         f"{tuple(weight.shape)}, {tuple(enc.shape)}")
    M, K = x.shape
    E = weight.shape[0]
    dev = x.device
    if weight.shape[1] != K or enc.shape[0] != M or enc.shape[2] != E:
        raise ValueError(f"shapes: x {tuple(x.shape)}, weight {tuple(weight.shape)}, "
                         f"enc {tuple(enc.shape)}")
    if x.dtype != torch.float32 or (M > 1 and x.stride(1) != 1) or x.device.type != "cuda":
        raise ValueError("x must be an f32 GPU tensor with unit column stride")
    call("ocppo_linear_cache_shift", _stream(dev), x.data_ptr(), x.stride(0) if M > 1 else K,
         _check(weight, "weight", torch.float32, dev), _opt(bias, "bias", torch.float32, dev, E),
         _check(enc, "enc", torch.float32, dev), _opt(done, "done", torch.float32, dev, M), M, E,
         K, enc.shape[1], 1 if relu else 0)
    return enc


def linear_cache_ring(x, weight, bias, enc, slot: int, done=None, relu: bool = True):
    """The rollout's last encoder layer writing the frame-encoding RING: fresh = act(x @ weight.T
    + bias) overwrites physical slot `slot` of enc [M, W, E] (every slot of an env with
    done != 0); nothing is shifted (ocppo_linear_cache_ring; read back with
    linear_act(..., ring=(E, rot)))."""
    if x.dim() != 2 or weight.dim() != 2 or enc.dim() != 3:
        raise ValueError(f"x [M, K], weight [E, K], enc [M, W, E] expected, got {tuple(x.shape)}, "
                         f"{tuple(weight.shape)}, {tuple(enc.shape)}")
    M, K = x.shape
    E = weight.shape[0]
    dev = x.device
    if weight.shape[1] != K or enc.shape[0] != M or enc.shape[2] != E:
        raise ValueError(f"shapes: x {tuple(x.shape)}, weight {tuple(weight.shape)}, "
                         f"enc {tuple(enc.shape)}")
    if x.dtype != torch.float32 or (M > 1 and x.stride(1) != 1) or x.device.type != "cuda":
        raise ValueError("x must be an f32 GPU tensor with unit column stride")
    call("ocppo_linear_cache_ring", _stream(dev), x.data_ptr(), x.stride(0) if M > 1 else K,
         _check(weight, "weight", torch.float32, dev), _opt(bias, "bias", torch.float32, dev, E),
         _check(enc, "enc", torch.float32, dev), _opt(done, "done", torch.float32, dev, M), M, E,
         K, enc.shape[1], int(slot), 1 if relu else 0)
    return enc


def store_linear2(frame, reward, done, prev_obs, obs_out, net_obs, done_out, reward_out, w1, b1,
                  w2, b2, y, vecnorm_state=None, gamma=0.99, epsilon=1e-8, clip_reward=10.0):
    """ONE launch: the rollout store of the previous step (ops.rollout_store, or
    ops.rollout_store_vecnorm when vecnorm_state = (ret_state, rms_state)) and
    y = relu(relu(f @ w1.T + b1) @ w2.T + b2) of the newest frames f (frame seen through the
    storage dtype of obs_out, f32 or bf16). frame [N, D] f32, obs [N, W, D], net_obs [N, W, D]
    f32, y [N, N2] f32 (row stride may exceed N2)."""
    N, D = frame.shape
    W = obs_out.shape[1]
    dev = frame.device
    f = torch.float32
    if frame.dtype != f:
        raise ValueError("store_linear2: object frames only (f32)")
    if prev_obs.shape != obs_out.shape or prev_obs.dtype != obs_out.dtype or \
            tuple(obs_out.shape) != (N, W, D) or obs_out.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError(f"obs slots must be [N, W, D] f32|bf16, got {tuple(obs_out.shape)} "
                         f"{obs_out.dtype}")
    N1, N2 = w1.shape[0], w2.shape[0]
    if tuple(w1.shape) != (N1, D) or tuple(w2.shape) != (N2, N1) or y.shape[0] != N or \
            y.shape[1] != N2 or y.stride(1) != 1 or y.dtype != f:
        raise ValueError(f"shapes: frame {tuple(frame.shape)}, w1 {tuple(w1.shape)}, "
                         f"w2 {tuple(w2.shape)}, y {tuple(y.shape)}")
    vn = vecnorm_state is not None
    ret, rms = vecnorm_state if vn else (None, None)
    call("ocppo_store_linear2", _stream(dev), _check(frame, "frame", f, dev),
         _check(reward, "reward", f, dev, N), _check(done, "done", f, dev, N), N, W, D,
         _check(prev_obs, "prev_obs", None, dev), _check(obs_out, "obs_out", None, dev),
         _DTYPE_CODE[obs_out.dtype], _opt(net_obs, "net_obs", f, dev, N * W * D),
         _check(reward_out, "reward_out", f, dev, N), _opt(done_out, "done_out", f, dev, N),
         int(vn), float(gamma), float(epsilon), float(clip_reward),
         _opt(ret, "ret_state", torch.float64, dev, N), _opt(rms, "rms_state", torch.float64, dev, 3),
         _check(w1, "w1", f, dev), _opt(b1, "b1", f, dev, N1), _check(w2, "w2", f, dev),
         _opt(b2, "b2", f, dev, N2), y.data_ptr(), y.stride(0) if N > 1 else N2, N1, N2)
    return y


# ---------------------------------------------------------------------------------------------
# Linear(+ReLU) backward, elementwise part: threshold_backward + bias sum in one pass
# (autograd of architectures/ppo.py:60-84 inside ppo_atari_oc.py:605)
# ---------------------------------------------------------------------------------------------
_RB_WS: dict = {}


def _relu_bias_ws(R: int, N: int, dev):
    """Per-shape workspace (tickets zeroed once, then self re-arming); never reallocated, so
    captured graphs keep valid pointers."""
    key = (dev, R, N)
    ws = _RB_WS.get(key)
    if ws is None:
        nb = int(_lib.LIB.ocppo_relu_bias_grad_workspace_bytes(R, N))
        ws = _RB_WS[key] = torch.zeros(nb, dtype=torch.uint8, device=dev)
    return ws


def relu_bias_grad_ok(g) -> bool:
    return (g.is_cuda and g.dtype == torch.float32 and g.dim() == 2 and g.shape[1] % 4 == 0
            and 4 <= g.shape[1] <= 16384 and g.is_contiguous() and g.data_ptr() % 16 == 0)


def relu_bias_grad(g, out=None, db=None, gp=None, bits=None):
    """(gp, db): gp = threshold_backward(g, out, 0) (g itself when out is None), db = gp.sum(0),
    in one pass over g [R, N] f32 (N % 4 == 0). Deterministic. bits: the ReLU mask as the
    forward epilogue's row-major bitmask (int32 [R N / 32], conv_x6(..., mbits=)) instead of out."""
    if g.dim() != 2:
        raise ValueError(f"g must be [R, N], got {tuple(g.shape)}")
    R, N = g.shape
    dev = g.device
    f = torch.float32
    if db is None:
        db = torch.empty(N, dtype=f, device=dev)
    if bits is not None:
        gp = torch.empty_like(g) if gp is None else gp
        ws = _relu_bias_ws(R, N, dev)
        call("ocppo_relu_bias_grad_bits", _stream(dev), _check(g, "g", f, dev),
             _check(bits, "bits", torch.int32, dev, R * N // 32), _check(gp, "gp", f, dev, R * N),
             _check(db, "db", f, dev, N), R, N, ws.data_ptr(), ws.numel())
        return gp, db
    if out is not None and gp is None:
        gp = torch.empty_like(g)
    ws = _relu_bias_ws(R, N, dev)
    call("ocppo_relu_bias_grad", _stream(dev), _check(g, "g", f, dev),
         _opt(out, "out", f, dev, R * N), _opt(gp, "gp", f, dev, R * N),
         _check(db, "db", f, dev, N), R, N, ws.data_ptr(), ws.numel())
    return (gp if out is not None else g), db


_RB_PART: dict = {}


def relu_bias_grad_partial(g, out=None, gp=None):
    """(gp, (partials, chunks)): relu_bias_grad with the bias-gradient chunk sums left for
    sum_splits_db (deferred to the launch that combines the layer's split-K weight gradient).
    partials [chunks, N] f32 is a per-shape persistent buffer (graph-safe)."""
    R, N = g.shape
    dev = g.device
    f = torch.float32
    if out is not None and gp is None:
        gp = torch.empty_like(g)
    key = (dev, R, N)
    buf = _RB_PART.get(key)
    if buf is None:
        chunks = int(_lib.LIB.ocppo_relu_bias_grad_chunks(R, N))
        buf = _RB_PART[key] = (torch.zeros((chunks, N), dtype=f, device=dev), chunks)
    call("ocppo_relu_bias_grad_partial", _stream(dev), _check(g, "g", f, dev),
         _opt(out, "out", f, dev, R * N), _opt(gp, "gp", f, dev, R * N), buf[0].data_ptr(), R, N)
    return (gp if out is not None else g), buf


def sum_splits_db(part, out, db_part, db, finish=None):
    """sum_splits(part, out) and db = db_part.sum(0) in a fixed order, one launch
    (db_part = the (partials, chunks) of relu_bias_grad_partial). finish = a filled
    DeferredFinish of relu_bias_wgrad(..., defer=): run by extra workgroups of the same launch
    (ocppo_sum_splits_db_finish; out / db bitwise the same)."""
    S = part.shape[0]
    dev = part.device
    f = torch.float32
    parts, chunks = db_part
    N = parts.shape[1]
    n = part[0].numel()
    args = (_check(part, "part", f, dev), S, n, _check(out, "out", f, dev, n),
            _check(parts, "db_partials", f, dev, chunks * N), chunks, N,
            _check(db, "db", f, dev, N))
    if finish is not None and finish.filled:
        finish.pending = False
        call("ocppo_sum_splits_db_finish", _stream(dev), *args, finish.ptr())
    else:
        call("ocppo_sum_splits_db", _stream(dev), *args)
    return out, db


def relu_bias_wgrad_ok(g, x) -> bool:
    return (relu_bias_grad_ok(g) and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
            and 1 <= x.shape[1] <= 16 and x.shape[0] == g.shape[0] and x.stride(1) == 1)


def relu_bias_wgrad(g, out, x, dw=None, db=None, defer=None):
    """(dw, db) of a Linear(+ReLU) layer whose input needs no gradient, in one pass:
    gp = threshold_backward(g, out, 0) (g when out is None, never materialised),
    db = gp.sum(0), dw = gp^T x. g [R, N] f32 (N % 4 == 0), x [R, K] f32 (K <= 16).
    defer = a DeferredFinish (R >= 1): only the rows launch runs now (ocppo_relu_bias_wgrad_rows);
    dw and db are written when the caller runs the finish (sum_splits_db(..., finish=) or run())."""
    if g.dim() != 2 or x.dim() != 2 or x.shape[0] != g.shape[0]:
        raise ValueError(f"g [R, N] and x [R, K] expected, got {tuple(g.shape)}, {tuple(x.shape)}")
    R, N = g.shape
    K = x.shape[1]
    dev = g.device
    f = torch.float32
    if x.stride(1) != 1 and R > 0:
        raise ValueError("x must have unit column stride")
    ldx = x.stride(0) if R > 1 else K
    if dw is None:
        dw = torch.empty((N, K), dtype=f, device=dev)
    if db is None:
        db = torch.empty(N, dtype=f, device=dev)
    if tuple(dw.shape) != (N, K) or not dw.is_contiguous():
        raise ValueError(f"dw must be a contiguous [{N}, {K}] tensor")
    key = (dev, "wg", R, N, K)
    ws = _RB_WS.get(key)
    if ws is None:
        nb = int(_lib.LIB.ocppo_relu_bias_wgrad_workspace_bytes(R, N, K))
        ws = _RB_WS[key] = torch.zeros(nb, dtype=torch.uint8, device=dev)
    call("ocppo_relu_bias_wgrad_rows" if defer is not None else "ocppo_relu_bias_wgrad",
         _stream(dev), _check(g, "g", f, dev),
         _opt(out, "out", f, dev, R * N),
         _check(x, "x", f, dev) if x.is_contiguous() else x.data_ptr(), ldx,
         _check(dw, "dw", f, dev, N * K), _check(db, "db", f, dev, N), R, N, K, ws.data_ptr(),
         ws.numel(), *((defer.ptr(),) if defer is not None else ()))
    if defer is not None:
        defer.pending = defer.filled = True
    return dw, db


def heads_bwd_ok(h, A: int) -> bool:
    return (h.is_cuda and h.dtype == torch.float32 and h.dim() == 2 and h.shape[0] >= 1 and
            h.shape[1] % 4 == 0 and 4 <= h.shape[1] <= 16384 and 1 <= A <= 7 and
            h.is_contiguous() and h.data_ptr() % 16 == 0)


def heads_bwd(h, dlogits, dvalue, wa, wc, relu: bool = True, gp=None, db_h=None, dwa=None,
              dwc=None, dba=None, dbc=None):
    """Actor/critic heads' backward + the producing layer's ReLU backward in one pass (see
    include/ocppo.h). h [M, H] (the heads' input = decoder ReLU output), dlogits [M, A],
    dvalue [M]; returns (gp, db_h, dwa, dwc, dba, dbc); db_h None skips the decoder bias.
    dvalue = wc = None: a single head (dwc, dbc returned as None)."""
    M, H = h.shape
    A = dlogits.shape[1]
    dev = h.device
    f = torch.float32
    critic = wc is not None
    if critic != (dvalue is not None):
        raise ValueError("dvalue and wc: both or neither")
    gp = torch.empty_like(h) if gp is None else gp
    dwa = torch.empty(A, H, dtype=f, device=dev) if dwa is None else dwa
    dba = torch.empty(A, dtype=f, device=dev) if dba is None else dba
    if critic:
        dwc = torch.empty(1, H, dtype=f, device=dev) if dwc is None else dwc
        dbc = torch.empty(1, dtype=f, device=dev) if dbc is None else dbc
    else:
        dwc = dbc = None
    key = (dev, "hb", M, H, A)
    ws = _RB_WS.get(key)
    if ws is None:
        nb = int(_lib.LIB.ocppo_heads_bwd_workspace_bytes(M, H, A))
        ws = _RB_WS[key] = torch.zeros(nb, dtype=torch.uint8, device=dev)
    call("ocppo_heads_bwd", _stream(dev), _check(h, "h", f, dev, M * H),
         _check(dlogits, "dlogits", f, dev, M * A), _opt(dvalue, "dvalue", f, dev, M),
         _check(wa, "wa", f, dev, A * H), _opt(wc, "wc", f, dev, H),
         _check(gp, "gp", f, dev, M * H), _opt(db_h, "db_h", f, dev, H),
         _check(dwa, "dwa", f, dev, A * H), _opt(dwc, "dwc", f, dev, H),
         _check(dba, "dba", f, dev, A), _opt(dbc, "dbc", f, dev, 1), M, H, A,
         1 if relu else 0, ws.data_ptr(), ws.numel())
    return gp, db_h, dwa, dwc, dba, dbc


def bias_act(y, b, relu: bool = True):
    """In place: y = act(y + b) over the rows of y [R, N] f32 (N % 4 == 0): the bias add + ReLU
    after a bias-less convolution (NHWC output viewed [B*H*W, C]) in one pass."""
    if y.dim() != 2:
        raise ValueError(f"y must be [R, N], got {tuple(y.shape)}")
    R, N = y.shape
    dev = y.device
    call("ocppo_bias_act", _stream(dev), _check(y, "y", torch.float32, dev),
         _check(b, "b", torch.float32, dev, N), R, N, int(bool(relu)))
    return y


def bias_act_nchw(y, b, relu: bool = True, out=None):
    """act(y + b) of a channels_last conv output y [B, C, H, W] (bias-less), returned as an
    NCHW-contiguous tensor (so an nn.Flatten after it is a view): one pass, layout copy included."""
    if y.dim() != 4 or not y.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("y must be a channels_last [B, C, H, W] tensor")
    B, C, H, W = y.shape
    dev = y.device
    f = torch.float32
    if out is None:
        out = torch.empty((B, C, H, W), dtype=f, device=dev)
    if not out.is_contiguous() or tuple(out.shape) != (B, C, H, W):
        raise ValueError("out must be a contiguous (NCHW) [B, C, H, W] tensor")
    call("ocppo_bias_act_nchw", _stream(dev), _check(y.permute(0, 2, 3, 1), "y", f, dev),
         _check(b, "b", f, dev, C),
         B, H * W, C, int(bool(relu)), _check(out, "out", f, dev, B * C * H * W))
    return out


def sum_splits_ok(part, out) -> bool:
    return (part.is_cuda and part.dtype == torch.float32 and part.is_contiguous() and
            out.is_contiguous() and out.dtype == torch.float32 and part.shape[0] in (1, 2, 4, 8, 16)
            and part[0].numel() % 4 == 0 and part.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0)


def sum_splits(part, out=None, finish=None):
    """out = part.sum(0) over the S split-K partial blocks of a weight gradient, in split order
    (added in f64, rounded once), in one streaming pass (part [S, ...] f32 contiguous, S in {1, 2, 4, 8, 16}).
    finish = a filled DeferredFinish: run by extra workgroups of the same launch
    (ocppo_sum_splits_finish; out bitwise the same)."""
    S = part.shape[0]
    dev = part.device
    if out is None:
        out = torch.empty(part.shape[1:], dtype=torch.float32, device=dev)
    n = part[0].numel()
    if finish is not None and finish.filled:
        finish.pending = False
        call("ocppo_sum_splits_finish", _stream(dev), _check(part, "part", torch.float32, dev), S,
             n, _check(out, "out", torch.float32, dev, n), finish.ptr())
        return out
    call("ocppo_sum_splits", _stream(dev), _check(part, "part", torch.float32, dev), S, n,
         _check(out, "out", torch.float32, dev, n))
    return out


# ---------------------------------------------------------------------------------------------
# Update-phase f32 GEMMs on the bf16 matrix cores (ocppo_gemm_x6; ppo_atari_oc.py:566-606)
# ---------------------------------------------------------------------------------------------
# (rows, columns) of variant & 7 (0-3: 4 waves, 4-7: 8 waves); variant & 8: loads two K steps
# ahead; variant & 16: one accumulator (built: every shape with both, shapes 0-3 with neither or
# only the latter). Variant 56: mixed tiles — rows [0, mbig) in 128 x 128 tiles dispatched first,
# the rest in 64 x 128 (mbig chosen in the library, include/ocppo.h); it divides, and counts its
# dbp rows and mask words, like 64 x 128
X6_TILES = ((128, 128), (64, 128), (128, 64), (64, 64),
            (128, 128), (64, 128), (128, 128), (128, 64)) * 7 + ((64, 128),) + (
    (256, 128), (128, 256), (128, 128), (128, 128)) + ((0, 0),) * 3
# workgroup threads of each variant (the ReLU bitmask holds one 64-bit word per thread and tile)
X6_THREADS = (256,) * 4 + (512,) * 4
X6_BUILT = tuple(range(4)) + tuple(range(16, 20)) + tuple(range(24, 32)) + (56, 57, 58, 59, 60)
X6_MIXED = 56
# the pipelined family (ocppo_gemm.hip gemm_x6p_kernel): two LDS stages, one barrier per K step
X6_PIPE = (57, 58, 59, 60)
X6_PIPE_THREADS = {57: 512, 58: 512, 59: 256, 60: 512}


X6_AUTO = 24  # the variant family x6_tile picks from (two K steps of loads in flight, one
# accumulator: fastest at every config-2 update shape, tools/exp_gemm_x6.py; error vs f64 at or
# below hipBLASLt's f32 GEMM, tests/test_gemm_gpu.py)


def x6_tile(M: int, N: int, splits: int = 1, tile: int | None = None) -> int | None:
    """Tile for an M x N (x splits) product: the largest tile that divides it and still gives
    >= 256 workgroups (one per CU; 128 x 128 is the fastest at every config-2 shape that has
    that many, tools/exp_gemm_x6.py), else the one giving the most; None if none divides."""
    if tile is not None:
        if tile not in X6_BUILT:
            return None  # no such variant in the library
        bm, bn = X6_TILES[tile]
        if tile == X6_MIXED and splits != 1:
            return None
        return tile if M % bm == 0 and N % bn == 0 else None
    # 256 < tiles of 128 x 128 <= 384 (more than one per CU, fewer than two): the mixed variant,
    # one 128 x 128 tile per CU and the rest in 64 x 128 tiles beside them (tools/exp_gemm_x6.py
    # --mbig; the split itself is chosen in the library)
    t128 = (M // 128) * (N // 128)
    if (splits == 1 and M % 128 == 0 and N % 128 == 0 and 256 < t128 <= 384
            and 256 % (N // 128) == 0):
        return X6_MIXED
    best, best_units = None, -1
    for i, (bm, bn) in enumerate(X6_TILES[:4]):
        i += X6_AUTO
        if M % bm or N % bn:
            continue
        units = splits * (M // bm) * (N // bn)
        if units >= 256:
            return i
        if units > best_units:
            best, best_units = i, units
    return best


def _x6_operand_ok(t) -> bool:
    return (t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.data_ptr() % 16 == 0
            and t.stride(1) == 1 and t.stride(0) % 4 == 0)


_SK_WS: dict = {}


def x6_sk_workspace(tile: int, device):
    """The stream-K workspace of a pipelined tile on `device` (zeroed once; every launch leaves
    its flags at zero again). Shared by the launches of one stream: they run one after another."""
    key = (tile, str(device))
    if key not in _SK_WS:
        n = _lib.LIB.ocppo_gemm_x6_sk_workspace_bytes(tile)
        if n == 0:
            raise ValueError(f"gemm_x6: tile {tile} has no stream-K form")
        _SK_WS[key] = torch.zeros(n, dtype=torch.uint8, device=device)
    return _SK_WS[key]


def x6_mbits_words(M: int, N: int, tile: int) -> int:
    """64-bit words of a gemm_x6 ReLU bitmask over an [M, N] output with `tile`."""
    bm, bn = X6_TILES[tile]
    nt = X6_PIPE_THREADS[tile] if tile in X6_PIPE_THREADS else X6_THREADS[tile & 7]
    return (M // bm) * (N // bn) * nt


def gemm_x6(a, sam, sak, b, sbn, sbk, c, ldc, M, N, K, splits=1, split_c=0, bias=None,
            relu=False, mask=None, dbp=None, tile=None, mbits_out=None, mbits_in=None, mbig=None,
            b_planes=None, stream_k=False, mbits_rows=False):
    """Raw ocppo_gemm_x6 call on tensors a, b, c (their data pointers; strides as given).
    mbig: rows in 128 x 128 tiles for the mixed variant (None: the library's choice).
    b_planes: B pre-split, bf16 [3, N, K] (split_planes of B); b may then be None.
    stream_k: a pipelined tile (57 / 58) as a persistent stream-K launch (x6_sk_workspace)."""
    t = x6_tile(M, N, splits, tile)
    if t is None:
        raise ValueError(f"gemm_x6: no tile divides {M} x {N}")
    dev = c.device
    if b_planes is not None:
        if (b_planes.dtype != torch.bfloat16 or tuple(b_planes.shape) != (3, N, K)
                or not b_planes.is_contiguous() or b_planes.device != dev or sak != 1
                or K % 8 or not (X6_AUTO <= t < X6_AUTO + 4 or t in (X6_MIXED, 57, 58))):
            raise ValueError("gemm_x6: b_planes must be a contiguous bf16 [3, N, K] on the "
                             "output's device, with a k-contiguous A and a tile of the x6 family")
    if mask is not None:
        if (mask.dim() != 2 or tuple(mask.shape) != (M, N) or mask.stride(1) != 1
                or mask.dtype != torch.float32 or dbp is None):
            raise ValueError("gemm_x6: mask must be an f32 [M, N] row-major view, with dbp")
    if mask is not None or mbits_in is not None:
        _check(dbp, "dbp", torch.float32, dev, (M // X6_TILES[t][0]) * N)
    if mbits_rows:
        if not relu or mbits_out is None:
            raise ValueError("gemm_x6: the row-major bitmask needs relu and mbits_out")
        _check(mbits_out, "mbits", torch.int32, dev, M * N // 32)
    for mb in ((mbits_in,) if mbits_rows else (mbits_out, mbits_in)):
        if mb is not None:
            _check(mb, "mbits", torch.int64, dev, x6_mbits_words(M, N, t))
    bp = None if bias is None else _check(bias, "bias", torch.float32, dev, N)
    args = (a.data_ptr(), sam, sak, None if b is None else b.data_ptr(), sbn, sbk, c.data_ptr(),
            ldc, M, N, K, splits,
            split_c, bp, int(bool(relu)) | (_lib.OCPPO_X6_MBITS_ROWS if mbits_rows else 0),
            None if mask is None else mask.data_ptr(),
            0 if mask is None else mask.stride(0), None if dbp is None else dbp.data_ptr(),
            None if mbits_out is None else mbits_out.data_ptr(),
            None if mbits_in is None else mbits_in.data_ptr(), t, -1 if mbig is None else int(mbig),
            None if b_planes is None else b_planes.data_ptr(), K, N * K,
            *((x6_sk_workspace(t, dev).data_ptr(), x6_sk_workspace(t, dev).numel())
              if stream_k else (None, 0)))
    # timer site name: the product's shape (bench.py's gemm_x6 roofline parses it); the closure
    # keeps the operand tensors alive for the timer's replays
    masked = mask is not None or mbits_in is not None
    name = f"gemm_x6_{M}x{N}x{K}s{splits}{'m' if masked else ''}"
    keep = (a, b, c, bias, mask, dbp, mbits_out, mbits_in, b_planes)
    _note_planes(b_planes, M, N, K)
    timed(name, lambda: call("ocppo_gemm_x6", _stream(dev), *args) or keep)
    return c


def linear_x6_ok(x, w) -> bool:
    """y = x W^T on gemm_x6: x [M, K], W [N, K] row-major f32, K % 32 == 0, a tile divides M x N."""
    return (_x6_operand_ok(x) and _x6_operand_ok(w) and x.shape[1] == w.shape[1]
            and x.shape[1] % 32 == 0 and x6_tile(x.shape[0], w.shape[0]) is not None)


def linear_x6(x, w, b=None, relu=False, out=None, mbits=False, planes=None):
    """act(x W^T + b) (torch._addmm_activation's order: sum, + bias, then ReLU). mbits=True
    (with relu) also returns the output's ReLU bitmask (tensor, tile) for dx_x6_relu; mbits="rows"
    the row-major one (int32 [M, N / 32] words, "rows") for frames_scatter_relu. planes: W's
    pre-split bf16 [3, N, K] (WeightPlanes; bitwise the same result)."""
    M, K = x.shape
    N = w.shape[0]
    out = torch.empty((M, N), dtype=torch.float32, device=x.device) if out is None else out
    if not mbits:
        return gemm_x6(x, x.stride(0), 1, w, w.stride(0), 1, out, out.stride(0), M, N, K, bias=b,
                       relu=relu, b_planes=planes)
    if mbits == "rows":
        if not relu or N % 32:
            raise ValueError("linear_x6: the row-major bitmask needs relu and N % 32 == 0")
        bits = torch.empty((M, N // 32), dtype=torch.int32, device=x.device)
        gemm_x6(x, x.stride(0), 1, w, w.stride(0), 1, out, out.stride(0), M, N, K, bias=b,
                relu=relu, mbits_out=bits, mbits_rows=True, b_planes=planes)
        return out, (bits, "rows")
    t = x6_tile(M, N)
    bits = torch.empty(x6_mbits_words(M, N, t), dtype=torch.int64, device=x.device)
    gemm_x6(x, x.stride(0), 1, w, w.stride(0), 1, out, out.stride(0), M, N, K, bias=b,
            relu=relu, tile=t, mbits_out=bits, b_planes=planes)
    return out, (bits, t)


def x6_fwd_splits(M: int, N: int, K: int):
    """K splits for a forward product too small for one wave of 128 x 128 tiles (< 256 of them):
    the fewest splits reaching >= 512 workgroups (two per CU) with >= 256 k per split, on the
    128 x 128 tile; None when it does not apply. ([4096 x 512] from K = 2048, the decoder: 4
    splits, 56.8 vs 71.9 us for hipBLASLt's f32 GEMM + epilogue, tools/exp_decoder_fwd.py.)"""
    if M % 128 or N % 128 or K % 32:
        return None
    tiles = (M // 128) * (N // 128)
    if tiles >= 256 or tiles < 32:
        return None
    for S in (2, 4, 8, 16):
        if K % (32 * S) == 0 and K // S >= 256 and S * tiles >= 512:
            return S
    return None


def gemm_x6_gather(a, sam, sak, b, sbn, sbk, c, ldc, M, N, K, gidx, gw, gseg, mode, splits=1,
                   split_c=0, bias=None, relu=False, b_planes=None):
    """ocppo_gemm_x6_gather: gemm_x6 on the 128 x 128 tile with one operand's rows read through
    the row table gidx [rows, gw] (mode 1: A(m, k) = a[gidx[m, k // gseg] * sam + k % gseg];
    mode 2: B(n, k) = b[gidx[k, n // gseg] * sbk + n % gseg]). Same products as gemm_x6 on the
    materialised operand, bitwise."""
    dev = c.device
    f = torch.float32
    args = (a.data_ptr(), sam, sak, None if b_planes is not None else b.data_ptr(), sbn, sbk,
            c.data_ptr(), ldc, M, N, K, splits, split_c, _opt(bias, "bias", f, dev),
            int(bool(relu)), None if b_planes is None else b_planes.data_ptr(),
            _check(gidx, "gidx", torch.int32, dev), gw, gseg, int(mode))
    keep = (a, b, c, bias, b_planes, gidx)
    _note_planes(b_planes, M, N, K)
    timed(f"gemm_x6_{M}x{N}x{K}s{splits}",
          lambda: call("ocppo_gemm_x6_gather", _stream(dev), *args) or keep)
    return c


def linear_x6_split(x, w, b, relu, splits, out=None, planes=None, gather=None):
    """act(x W^T + b) as `splits` K-split gemm_x6 partials + ocppo_sum_splits_act (the partials
    added in split order in f64, then + bias, then ReLU). gather = (idx [M, W], E): x is the
    [C, E] row source and the product's input row m is the concatenation of x[idx[m, 0..W)]
    (frames_expand never materialised; one split per stack slot, splits == W)."""
    if gather is None:
        M, K = x.shape
    else:
        idx, E = gather
        M, K = idx.shape[0], idx.shape[1] * E
    N = w.shape[0]
    dev = x.device
    part = torch.empty((splits, M, N), dtype=torch.float32, device=dev)
    if gather is None:
        gemm_x6(x, x.stride(0), 1, w, w.stride(0), 1, part, N, M, N, K, splits=splits,
                split_c=M * N, tile=X6_AUTO, b_planes=planes)
    else:
        gemm_x6_gather(x, x.stride(0), 1, w, w.stride(0), 1, part, N, M, N, K, idx, idx.shape[1],
                       E, 1, splits=splits, split_c=M * N, b_planes=planes)
    out = torch.empty((M, N), dtype=torch.float32, device=dev) if out is None else out
    f = torch.float32
    args = (part.data_ptr(), splits, M, N, _opt(b, "bias", f, dev, N), int(bool(relu)),
            _check(out, "out", f, dev, M * N))
    keep = (part, out, b)
    timed(f"sum_splits_act_{splits}x{M}x{N}",
          lambda: call("ocppo_sum_splits_act", _stream(dev), *args) or keep)
    return out


def dx_x6_ok(g, w) -> bool:
    """dX = g W on gemm_x6: g [M, N] (N % 32 == 0), W [N, K]."""
    return (_x6_operand_ok(g) and _x6_operand_ok(w) and g.shape[1] == w.shape[0]
            and g.shape[1] % 32 == 0 and x6_tile(g.shape[0], w.shape[1]) is not None)


def dx_x6(g, w, out=None, planes=None, tile=None):
    """g W; planes: W^T's pre-split bf16 [3, K, N] (WeightPlanes); tile: None = x6_tile's."""
    M, N = g.shape
    K = w.shape[1]
    out = torch.empty((M, K), dtype=torch.float32, device=g.device) if out is None else out
    return gemm_x6(g, g.stride(0), 1, w, 1, w.stride(0), out, out.stride(0), M, K, N,
                   b_planes=planes, tile=tile)


_WG_REC = {}


def dx_x6_wgrad_ok(g, w, mask, x) -> bool:
    """dX = g W with the lower layer's backward in the epilogue (dx_x6_wgrad) applies."""
    M, N = g.shape
    K = w.shape[1]
    return (_x6_operand_ok(g) and w.is_cuda and w.dtype == torch.float32 and w.dim() == 2
            and w.stride(1) == 1 and w.stride(0) % 4 == 0 and w.data_ptr() % 16 == 0
            and w.shape[0] == N and N % 32 == 0 and M % 64 == 0 and K % 64 == 0
            and mask.is_cuda and mask.dtype == torch.float32 and mask.shape == (M, K)
            and mask.stride(1) == 1 and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
            and x.shape[0] == M and 1 <= x.shape[1] <= 16 and x.stride(1) == 1)


def dx_x6_wgrad(g, w, mask, x, dw, db, defer, tile=27):
    """The lower Linear+ReLU layer's (dw, db) from this layer's dX = g W without storing dX:
    gp = mask > 0 ? g W : 0, db = gp.sum(0), dw = gp^T x (ocppo_gemm_x6_wgrad; g [M, N], W [N, K],
    mask [M, K] the lower layer's ReLU output, x [M, K1] its input rows). The per-row-tile records
    are finished by the filled DeferredFinish `defer` (sum_splits_db(..., finish=) or run())."""
    M, N = g.shape
    K = w.shape[1]
    K1 = x.shape[1]
    dev = g.device
    bm = 64 if tile == 27 else 128
    kp = 4 if K1 <= 4 else 8 if K1 <= 8 else 12 if K1 <= 12 else 16
    nrec = (M // bm) * ((K + 255) // 256) * 256 * (kp + 1)
    key = (dev, M, K, kp, tile)
    rec = _WG_REC.get(key)
    if rec is None:
        rec = _WG_REC[key] = torch.empty(nrec, dtype=torch.float32, device=dev)
    f = torch.float32
    args = (g.data_ptr(), g.stride(0), 1, w.data_ptr(), 1, w.stride(0), M, K, N,
            mask.data_ptr(), mask.stride(0), x.data_ptr(), x.stride(0), K1,
            _check(dw, "dw", f, dev, K * K1), _check(db, "db", f, dev, K), rec.data_ptr(),
            rec.numel(), int(tile), defer.ptr())
    keep = (g, w, mask, x, dw, db, rec)
    timed(f"gemm_x6_{M}x{K}x{N}s1w", lambda: call("ocppo_gemm_x6_wgrad", _stream(dev), *args)
          or keep)
    defer.pending = defer.filled = True


def dx_x6_relu(g, w, mask, mbits=None, planes=None):
    """gp = threshold_backward(g W, mask, 0) for the Linear+ReLU layer below whose output is
    `mask` [M, K], with that layer's bias-gradient partials: returns (gp, dbp [M / tile rows, K])
    (dbp summed in row-tile order by sum_splits_db). mbits = (bitmask, tile) from that layer's
    linear_x6(..., mbits=True): read instead of the f32 mask when this product has the same tile."""
    M, N = g.shape
    K = w.shape[1]
    t = x6_tile(M, K)
    gp = torch.empty((M, K), dtype=torch.float32, device=g.device)
    dbp = torch.empty((M // X6_TILES[t][0], K), dtype=torch.float32, device=g.device)
    if mbits is not None and mbits[1] == t:
        gemm_x6(g, g.stride(0), 1, w, 1, w.stride(0), gp, K, M, K, N, dbp=dbp, tile=t,
                mbits_in=mbits[0], b_planes=planes)
    else:
        gemm_x6(g, g.stride(0), 1, w, 1, w.stride(0), gp, K, M, K, N, mask=mask, dbp=dbp, tile=t,
                b_planes=planes)
    return gp, dbp


class WeightPlanes:
    """Pre-split bf16 planes of Linear weights for the update GEMMs' B operand (ocppo_gemm_x6 with
    b_planes): [3, N, K] of W for the forward, [3, K, N] of W^T for dX, written by ONE
    ocppo_split_planes launch per refresh (after every optimizer step: the trainer refreshes at
    the start of each minibatch). The parameters are views of a flat buffer at fixed addresses,
    so the job table is built once. Attaches w._ocppo_planes = {"fwd": ..., "dx": ...}."""

    def __init__(self, fwd=(), dx=()):
        jobs = []
        for ws, trans in ((fwd, 0), (dx, 1)):
            for w in ws:
                if w.dtype != torch.float32 or w.dim() != 2 or w.stride(1) != 1:
                    raise ValueError("WeightPlanes: row-major f32 weights")
                R, C = w.shape
                shape = (3, C, R) if trans else (3, R, C)
                if shape[2] % 8:
                    raise ValueError(f"WeightPlanes: plane rows of {shape[2]} elements")
                dst = torch.empty(shape, dtype=torch.bfloat16, device=w.device)
                d = getattr(w, "_ocppo_planes", None) or {}
                d["dx" if trans else "fwd"] = dst
                w._ocppo_planes = d
                jobs.append((w, trans, dst))
        self.jobs = jobs
        self.dev = jobs[0][0].device if jobs else None
        c = ctypes
        self.calls = []
        for i in range(0, len(jobs), 8):
            part = jobs[i:i + 8]
            n = len(part)
            arrs = ((c.c_void_p * n)(*[w.data_ptr() for w, _, _ in part]),
                    (c.c_int64 * n)(*[w.stride(0) for w, _, _ in part]),
                    (c.c_int64 * n)(*[w.shape[0] for w, _, _ in part]),
                    (c.c_int64 * n)(*[w.shape[1] for w, _, _ in part]),
                    (c.c_int * n)(*[t for _, t, _ in part]),
                    (c.c_void_p * n)(*[d.data_ptr() for _, _, d in part]))
            self.calls.append((n, arrs))

    def refresh(self):
        for n, arrs in self.calls:
            call("ocppo_split_planes", _stream(self.dev), n, *arrs)


def split_planes_ref(x):
    """The exact three-piece bf16 split of an f32 tensor in torch (round to nearest even at each
    step): the reference ocppo_split_planes / gemm_x6 are checked against (tests)."""
    x0 = x.to(torch.bfloat16)
    r1 = x - x0.float()
    x1 = r1.to(torch.bfloat16)
    x2 = (r1 - x1.float()).to(torch.bfloat16)
    return torch.stack([x0, x1, x2])


def dw_x6_ok(g, x, splits: int) -> bool:
    """dW = g^T x on gemm_x6 as `splits` partial products over the rows (in steps of 32)."""
    rows = g.shape[0]
    return (_x6_operand_ok(g) and _x6_operand_ok(x) and x.shape[0] == rows and splits >= 1
            and rows % 32 == 0 and rows // 32 >= splits
            and x6_tile(g.shape[1], x.shape[1], splits) is not None)


def dw_x6_parts(g, x, splits: int, part=None, tile=None):
    """part[s] = g[rows of split s]^T x[rows of split s] -> [splits, N, K], the rows split evenly
    in steps of 32 (combined by sum_splits / sum_splits_db in split order)."""
    rows, N = g.shape
    K = x.shape[1]
    part = (torch.empty((splits, N, K), dtype=torch.float32, device=g.device)
            if part is None else part)
    return gemm_x6(g, 1, g.stride(0), x, 1, x.stride(0), part, K, N, K, rows, splits=splits,
                   split_c=N * K, tile=tile)


def dw_x6_parts_gather(g, src, idx, splits: int, part=None):
    """dw_x6_parts with x never materialised: x[r] = concat(src[idx[r, 0..W)]) (src [C, E],
    idx [rows, W] int32; the 128 x 128 tile, rows / splits <= 1024) -> [splits, N, W * E]."""
    rows, N = g.shape
    W = idx.shape[1]
    E = src.shape[1]
    K = W * E
    part = (torch.empty((splits, N, K), dtype=torch.float32, device=g.device)
            if part is None else part)
    return gemm_x6_gather(g, 1, g.stride(0), src, 1, src.stride(0), part, K, N, K, rows, idx, W,
                          E, 2, splits=splits, split_c=N * K)


# ---------------------------------------------------------------------------------------------
# Frame-deduplicated PPObj minibatch encoder (ppo_atari_oc.py:566 through architectures/ppo.py:60-84)
# ---------------------------------------------------------------------------------------------
def _obs_TNWF(obs):
    if obs.dim() != 4:
        raise ValueError(f"obs must be [T+1, N, W, F], got {tuple(obs.shape)}")
    T1, N, W, F = obs.shape
    return T1 - 1, N, W, F


def frames_gather(obs, uniq, out=None):
    """x[c, :] = f32(frame with timeline id uniq[c]) of the rollout obs [T+1, N, W, F]
    (padding ids < 0 give zero rows). uniq [C] int32 -> x [C, F] f32."""
    T, N, W, F = _obs_TNWF(obs)
    dev = obs.device
    C = uniq.numel()
    if out is None:
        out = torch.empty((C, F), dtype=torch.float32, device=dev)
    call("ocppo_frames_gather", _stream(dev), _check(obs, "obs", None, dev),
         _DTYPE_CODE[obs.dtype], T, N, W, F, _check(uniq, "uniq", torch.int32, dev), C,
         _check(out, "out", torch.float32, dev, C * F))
    return out


def frames_gather_linear(obs, uniq, weight, bias=None, relu: bool = True, x_out=None,
                         h_out=None, index=None):
    """(x, h): frames_gather(obs, uniq) and act(x @ weight.T + bias) in one launch
    (ocppo_frames_gather_linear: the update's first encoder layer over the distinct frames).
    index = (pos_of, perm, dones[, out]): also frames_expand_index's row table in the same launch;
    returns (x, h, idx) then."""
    T, N, W, F = _obs_TNWF(obs)
    dev = obs.device
    C = uniq.numel()
    N1 = weight.shape[0]
    f = torch.float32
    if x_out is None:
        x_out = torch.empty((C, F), dtype=f, device=dev)
    if h_out is None:
        h_out = torch.empty((C, N1), dtype=f, device=dev)
    ix, idx = (None, None, 0, None, None), None
    if index is not None:
        pos_of, perm, dones = index[:3]
        M = perm.numel()
        idx = index[3] if len(index) > 3 else torch.empty((M, W), dtype=torch.int32, device=dev)
        ix = (_check(pos_of, "pos_of", torch.int32, dev, (T + W - 1) * N),
              _check(perm, "perm", torch.int64, dev), M,
              _check(dones, "dones", f, dev, (T + 1) * N), _check(idx, "idx", torch.int32, dev, M * W))
    call("ocppo_frames_gather_linear", _stream(dev), _check(obs, "obs", None, dev),
         _DTYPE_CODE[obs.dtype], T, N, W, F, _check(uniq, "uniq", torch.int32, dev), C,
         _check(weight, "weight", f, dev, N1 * F), _opt(bias, "bias", f, dev, N1), N1,
         int(bool(relu)), _check(x_out, "x_out", f, dev, C * F),
         _check(h_out, "h_out", f, dev, C * N1), *ix)
    return (x_out, h_out) if index is None else (x_out, h_out, idx)


def frames_expand(enc, pos_of, perm, dones, T: int, N: int, W: int, out=None):
    """h[i, k, :] = enc[pos_of[timeline id of slot k of sample perm[i]]] -> [M, W, E] f32.
    enc [C, E] f32, pos_of [(T+W-1)*N] int32, perm [M] int64, dones [T+1, N] f32."""
    C, E = enc.shape
    M = perm.numel()
    dev = enc.device
    if out is None:
        out = torch.empty((M, W, E), dtype=torch.float32, device=dev)
    call("ocppo_frames_expand", _stream(dev), _check(enc, "enc", torch.float32, dev), C, E,
         _check(pos_of, "pos_of", torch.int32, dev, (T + W - 1) * N),
         _check(perm, "perm", torch.int64, dev), M,
         _check(dones, "dones", torch.float32, dev, (T + 1) * N), T, N, W,
         _check(out, "out", torch.float32, dev, M * W * E))
    return out


def frames_expand_index(pos_of, perm, dones, T: int, N: int, W: int, out=None):
    """idx[i, k] = pos_of[timeline id of slot k of sample perm[i]] -> [M, W] int32: the source
    rows frames_expand copies, for the gathered decoder GEMMs (gemm_x6_gather)."""
    M = perm.numel()
    dev = perm.device
    if out is None:
        out = torch.empty((M, W), dtype=torch.int32, device=dev)
    call("ocppo_frames_expand_index", _stream(dev),
         _check(pos_of, "pos_of", torch.int32, dev, (T + W - 1) * N),
         _check(perm, "perm", torch.int64, dev), M,
         _check(dones, "dones", torch.float32, dev, (T + 1) * N), T, N, W,
         _check(out, "idx", torch.int32, dev, M * W))
    return out


def frames_scatter(dh, uniq, inv, mb: int, dones, T: int, N: int, W: int, out=None):
    """Backward of frames_expand: denc[c, :] = sum of dh[i, k, :] over the uses of frame uniq[c]
    by minibatch `mb` (inv [T*N] int32: position of each sample in the epoch permutation).
    dh [M, W, E] f32 -> denc [C, E] f32, deterministic."""
    M = dh.shape[0]
    E = dh.shape[-1]
    if dh.numel() != M * W * E:
        raise ValueError(f"dh must be [M, W, E] with W={W}, got {tuple(dh.shape)}")
    C = uniq.numel()
    dev = dh.device
    if out is None:
        out = torch.empty((C, E), dtype=torch.float32, device=dev)
    call("ocppo_frames_scatter", _stream(dev), _check(dh, "dh", torch.float32, dev), M, E,
         _check(uniq, "uniq", torch.int32, dev), C, _check(inv, "inv", torch.int32, dev, T * N),
         int(mb), _check(dones, "dones", torch.float32, dev, (T + 1) * N), T, N, W,
         _check(out, "out", torch.float32, dev, C * E))
    return out


_SCATTER_DBP: dict = {}


def frames_scatter_relu(dh, uniq, inv, mb: int, dones, T: int, N: int, W: int, out=None,
                        gp=None, with_db: bool = True, mbits=None):
    """frames_scatter with the ReLU backward of the layer whose output `out` [C, E] encoded the
    frames: gp = out <= 0 ? 0 : denc (ocppo_frames_scatter_relu). mbits: that output's row-major
    ReLU bitmask (linear_x6(..., mbits="rows")), read instead of `out`. Returns (gp, (partials,
    chunks)): the bias-gradient chunk sums (16 frames per chunk; a per-shape persistent buffer,
    graph-safe) for sum_splits_db, or (gp, None) without with_db."""
    M = dh.shape[0]
    E = dh.shape[-1]
    if dh.numel() != M * W * E:
        raise ValueError(f"dh must be [M, W, E] with W={W}, got {tuple(dh.shape)}")
    C = uniq.numel()
    dev = dh.device
    f = torch.float32
    if gp is None:
        gp = torch.empty((C, E), dtype=f, device=dev)
    part = None
    if with_db:
        key = (dev, C, E)
        part = _SCATTER_DBP.get(key)
        if part is None:
            chunks = int(_lib.LIB.ocppo_frames_scatter_chunks(C))
            part = _SCATTER_DBP[key] = (torch.zeros((chunks, E), dtype=f, device=dev), chunks)
    call("ocppo_frames_scatter_relu", _stream(dev), _check(dh, "dh", f, dev), M, E,
         _check(uniq, "uniq", torch.int32, dev), C, _check(inv, "inv", torch.int32, dev, T * N),
         int(mb), _check(dones, "dones", f, dev, (T + 1) * N), T, N, W,
         _opt(out, "out", f, dev, C * E) if mbits is None else None,
         _opt(mbits, "mbits", torch.int32, dev, C * E // 32), _check(gp, "gp", f, dev, C * E),
         part[0].data_ptr() if part is not None else None)
    return gp, part


def frame_cache_shift(enc, fresh, done=None):
    """In-place shift of the rollout's frame-encoding cache (PPObj): enc [N, W, E] f32,
    fresh [N, E] f32 (row stride may exceed E), done [N] f32 or None:
    enc[n, w] = fresh[n] if done[n] or w == W-1 else enc[n, w+1]  (the frame stack's own rule,
    ppo_atari_oc.py:506 re-encoding all W frames every step is what this saves)."""
    dev = enc.device
    if enc.dim() != 3 or fresh.dim() != 2:
        raise ValueError(f"enc must be [N, W, E] and fresh [N, E], got {tuple(enc.shape)}, "
                         f"{tuple(fresh.shape)}")
    N, W, E = enc.shape
    if tuple(fresh.shape) != (N, E) or fresh.stride(1) != 1 or fresh.dtype != torch.float32 \
            or fresh.device != dev:
        raise ValueError("fresh must be an f32 [N, E] row-major view on enc's device")
    _stream(fresh.device)
    call("ocppo_frame_cache_shift", _stream(dev), _check(enc, "enc", torch.float32, dev),
         fresh.data_ptr(), fresh.stride(0) if N > 1 else E,
         _opt(done, "done", torch.float32, dev, N), N, W, E)
    return enc


def gather_rows(src, idx, out=None, scale255: bool = False):
    """out[i] = float32(src[idx[i]]) for src [B, ...] f32|bf16|u8 → out [M, ...] f32. A
    channels_last `out` [M, C, H, X] gets the rows in NHWC order (ocppo_gather_rows_cl), divided
    by 255 as NormalizeImg does when scale255."""
    dev = src.device
    M = idx.numel()
    R = src[0].numel() if src.shape[0] else 0
    if out is None:
        out = torch.empty((M,) + tuple(src.shape[1:]), dtype=torch.float32, device=dev)
    if src.dtype not in _DTYPE_CODE:
        raise ValueError(f"unsupported src dtype {src.dtype}")
    if not out.is_contiguous():
        if not (out.dim() == 4 and out.is_contiguous(memory_format=torch.channels_last) and
                tuple(out.shape[1:]) == tuple(src.shape[1:]) and out.shape[0] == M and
                out.dtype == torch.float32 and out.device == dev):
            raise ValueError("out must be contiguous or a channels_last [M, C, H, X] f32 tensor")
        C = src.shape[1]
        call("ocppo_gather_rows_cl", _stream(dev), _check(src, "src", None, dev),
             _DTYPE_CODE[src.dtype], _check(idx, "idx", torch.int64, dev, M), M, C, R // C,
             out.data_ptr(), 2 if scale255 else 0)
        return out
    if scale255:
        raise ValueError("scale255 needs a channels_last out (ocppo_gather_rows_cl)")
    call("ocppo_gather_rows", _stream(dev), _check(src, "src", None, dev), _DTYPE_CODE[src.dtype],
         _check(idx, "idx", torch.int64, dev, M), M, R,
         _check(out, "out", torch.float32, dev, M * R))
    return out


# ---------------------------------------------------------------------------------------------
# VecNormalize reward normalisation (ppo_atari_oc.py:414, SB3 2.0.0 semantics)
# ---------------------------------------------------------------------------------------------
def vecnorm_reward(reward, done, ret_state, rms_state, reward_out, gamma=0.99, epsilon=1e-8,
                   clip_reward=10.0):
    N = reward.numel()
    dev = reward.device
    f = torch.float32
    call("ocppo_vecnorm_reward", _stream(dev), _check(reward, "reward", f, dev),
         _check(done, "done", f, dev, N), N, float(gamma), float(epsilon), float(clip_reward),
         _check(ret_state, "ret_state", torch.float64, dev, N),
         _check(rms_state, "rms_state", torch.float64, dev, 3),
         _check(reward_out, "reward_out", f, dev, N))
    return reward_out


# ---------------------------------------------------------------------------------------------
# synthetic env (harness)
# ---------------------------------------------------------------------------------------------
def synth_env_step(seed: int, step_base, step_offset: int, actions, frame_out, reward_out,
                   done_out, ep_state=None):
    N = reward_out.numel()
    D = frame_out[0].numel()
    dev = frame_out.device
    pixel = frame_out.dtype == torch.uint8
    if not pixel and frame_out.dtype != torch.float32:
        raise ValueError("frame_out must be f32 (objects) or u8 (pixels)")
    call("ocppo_synth_env_step", _stream(dev), seed & 0xFFFFFFFFFFFFFFFF,
         _check(step_base, "step_base", torch.int64, dev, 1), int(step_offset),
         _opt(actions, "actions", torch.int64, dev, N), N, D, int(pixel),
         _check(frame_out, "frame_out", None, dev, N * D),
         _check(reward_out, "reward_out", torch.float32, dev, N),
         _check(done_out, "done_out", torch.float32, dev, N),
         _opt(ep_state, "ep_state", torch.float32, dev, N * 5))


def cartpole_step(seed: int, actions, state, counters, obs_out, reward_out=None, done_out=None,
                  ep_state=None):
    """One step (actions [N] i64) or, with actions None, a reset of N device CartPole-v1 envs
    (gymnasium 0.28.1 dynamics, TimeLimit 500, same-step auto-reset): state [N, 4] f64 and
    counters [N, 2] i64 in/out, obs_out [N, 4] f32, reward_out / done_out [N] f32."""
    N = obs_out.shape[0]
    dev = obs_out.device
    f = torch.float32
    call("ocppo_cartpole_step", _stream(dev), int(seed) & 0xFFFFFFFFFFFFFFFF,
         _opt(actions, "actions", torch.int64, dev, N), N,
         _check(state, "state", torch.float64, dev, 4 * N),
         _check(counters, "counters", torch.int64, dev, 2 * N),
         _check(obs_out, "obs_out", f, dev, 4 * N), _opt(reward_out, "reward_out", f, dev, N),
         _opt(done_out, "done_out", f, dev, N), _opt(ep_state, "ep_state", f, dev, 5 * N))


# ---------------------------------------------------------------------------------------------
# clip_grad_norm_ + Adam over flat buffers (ppo_atari_oc.py:608-610)
# ---------------------------------------------------------------------------------------------
OPT_STEP, OPT_TOTAL_NORM, OPT_CLIP_COEF = 0, 1, 2


FLAT_ALIGN = 64  # floats: every parameter / grad view in a flat buffer starts 256-B aligned


def flat_offsets(params):
    """Offsets of `params` in one flat f32 buffer, each rounded up to FLAT_ALIGN elements so the
    views keep the 16-B alignment the vectorised kernels (policy head, Adam) need; returns
    (offsets, total length)."""
    offs, off = [], 0
    for p in params:
        offs.append(off)
        off += -(-p.numel() // FLAT_ALIGN) * FLAT_ALIGN
    return offs, off


class FlatAdam:
    """Adam (torch.optim.Adam semantics, eps as given) + global-norm gradient clipping over ONE
    flat f32 parameter buffer. Construct it over the module's parameters: every parameter becomes
    a view of `self.params` and its `.grad` a view of `self.grads` (so the DP all-reduce is one
    call). `step()` is two HIP launches and is graph-capturable (step count, lr on device)."""

    def __init__(self, params, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_grad_norm: float = 0.0):
        params = [p for p in params if p.requires_grad]
        dev = params[0].device
        offs, n = flat_offsets(params)
        self.numel = n
        # zero padding between parameters is a fixed point of clip + Adam (g = m = v = p = 0)
        self.params = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(n, dtype=torch.float32, device=dev)
        for p, off in zip(params, offs):
            k = p.numel()
            if p.dtype != torch.float32:
                raise ValueError("FlatAdam needs f32 parameters")
            # same strides as the parameter (e.g. channels_last conv weights keep their layout)
            view = self.params[off:off + k].as_strided(p.shape, p.stride())
            view.copy_(p.detach())
            p.data = view
            p.grad = self.grads[off:off + k].as_strided(p.shape, p.stride())
            p._ocppo_direct_grad = True  # agents.py's autograd Functions write grads in place
        self.param_list = params
        self.exp_avg = torch.zeros_like(self.params)
        self.exp_avg_sq = torch.zeros_like(self.params)
        self.lr = torch.tensor(float(lr), dtype=torch.float32, device=dev)
        self.scalars = torch.zeros(8, dtype=torch.float32, device=dev)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.max_grad_norm = float(max_grad_norm)
        nb = _lib.LIB.ocppo_clip_adam_workspace_bytes(n)
        self.ws = torch.zeros(int(nb), dtype=torch.uint8, device=dev)
        self._planes = (0, None, None, None, None, None)

    def write_planes(self, jobs):
        """jobs [(weight, trans, planes)] (WeightPlanes.jobs): every step also writes each
        weight's new values as its three exact bf16 pieces ([3, N, K], or of W^T [3, K, N] with
        trans) into planes, so the next GEMMs need no split launch (ocppo_clip_adam_step's plane
        jobs, <= 8)."""
        jobs = list(jobs)
        if len(jobs) > 8:
            raise ValueError("FlatAdam.write_planes: at most 8 weights")
        base = self.params.data_ptr()
        offs, rows, cols, trs, dsts = [], [], [], [], []
        for w, trans, d in jobs:
            off = (w.data_ptr() - base) // 4
            if (w.dtype != torch.float32 or w.dim() != 2 or not w.is_contiguous()
                    or not 0 <= off < self.numel or d.dtype != torch.bfloat16
                    or d.numel() != 3 * w.numel() or not d.is_contiguous()):
                raise ValueError("FlatAdam.write_planes: a contiguous 2-D weight of this buffer "
                                 "and its bf16 [3, ...] planes")
            offs.append(off)
            rows.append(w.shape[0])
            cols.append(w.shape[1])
            trs.append(int(trans))
            dsts.append(d.data_ptr())
        c = ctypes
        n = len(jobs)
        self._planes = ((n, (c.c_int64 * n)(*offs), (c.c_int64 * n)(*rows),
                         (c.c_int64 * n)(*cols), (c.c_int * n)(*trs), (c.c_void_p * n)(*dsts))
                        if n else (0, None, None, None, None, None))
        self._plane_keep = [d for _, _, d in jobs]

    def zero_grad(self):
        self.grads.zero_()

    def step(self, grad_scale: float = 1.0):
        dev = self.params.device
        call("ocppo_clip_adam_step", _stream(dev), self.params.data_ptr(), self.grads.data_ptr(),
             self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), self.numel,
             self.lr.data_ptr(), self.betas[0], self.betas[1], self.eps, float(grad_scale),
             self.max_grad_norm, self.scalars.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
             *self._planes)


# ---------------------------------------------------------------------------------------------
# DQN (config 5): HBM replay buffer, epsilon-greedy, fused TD target + MSE (dqn_atari_oc.py)
# ---------------------------------------------------------------------------------------------
class ReplayBuffer:
    """SB3 ReplayBuffer(optimize_memory_usage=True, handle_timeout_termination=False) in HBM
    (dqn_atari_oc.py:317-325): obs [size, E, D] in an exact compact dtype, next obs of slot i at
    slot i+1; device {pos, full} state so add/sample are graph-replayable."""

    def __init__(self, size: int, n_envs: int, obs_shape, device, obs_dtype=torch.uint8,
                 seed: int = 0):
        self.size, self.E = int(size), int(n_envs)
        self.obs_shape = tuple(obs_shape)
        self.D = 1
        for d in self.obs_shape:
            self.D *= d
        dev = torch.device(device)
        self.device = dev
        self.obs = torch.zeros((self.size, self.E) + self.obs_shape, dtype=obs_dtype, device=dev)
        self.actions = torch.zeros((self.size, self.E), dtype=torch.int64, device=dev)
        self.rewards = torch.zeros((self.size, self.E), dtype=torch.float32, device=dev)
        self.dones = torch.zeros((self.size, self.E), dtype=torch.float32, device=dev)
        self.state = torch.zeros(2, dtype=torch.int64, device=dev)  # pos, full
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        self.ws = torch.zeros(int(_lib.LIB.ocppo_replay_workspace_bytes()), dtype=torch.uint8,
                              device=dev)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF

    def add(self, obs, next_obs, actions, rewards, dones):
        dev = self.device
        f = torch.float32
        if obs.dtype not in _DTYPE_CODE or next_obs.dtype != obs.dtype:
            raise ValueError("obs/next_obs must both be f32, bf16 or u8")
        n = self.E * self.D
        call("ocppo_replay_add", _stream(dev), _check(obs, "obs", None, dev, n),
             _check(next_obs, "next_obs", None, dev, n), _DTYPE_CODE[obs.dtype],
             _check(actions, "actions", torch.int64, dev, self.E),
             _check(rewards, "rewards", f, dev, self.E), _check(dones, "dones", f, dev, self.E),
             self.E, self.D, self.state.data_ptr(), self.size, self.obs.data_ptr(),
             _DTYPE_CODE[self.obs.dtype], self.actions.data_ptr(), self.rewards.data_ptr(),
             self.dones.data_ptr(), self.ws.data_ptr())

    def sample(self, batch_size: int, out: dict | None = None, with_indices: bool = False):
        dev = self.device
        B = int(batch_size)
        if out is None:
            out = {"observations": torch.empty((B,) + self.obs_shape, device=dev),
                   "next_observations": torch.empty((B,) + self.obs_shape, device=dev),
                   "actions": torch.empty((B, 1), dtype=torch.int64, device=dev),
                   "rewards": torch.empty((B, 1), device=dev),
                   "dones": torch.empty((B, 1), device=dev)}
            if with_indices:
                out["indices"] = torch.empty((B, 2), dtype=torch.int64, device=dev)
        call("ocppo_replay_sample", _stream(dev), self.seed, self.counter.data_ptr(),
             self.state.data_ptr(), self.size, self.E, self.D, self.obs.data_ptr(),
             _DTYPE_CODE[self.obs.dtype], self.actions.data_ptr(), self.rewards.data_ptr(),
             self.dones.data_ptr(), B, out["observations"].data_ptr(),
             out["next_observations"].data_ptr(), out["actions"].data_ptr(),
             out["rewards"].data_ptr(), out["dones"].data_ptr(),
             out["indices"].data_ptr() if "indices" in out else None)
        return out


def epsilon_greedy(q, seed: int, step, start_e: float, end_e: float, duration: float,
                   actions_out=None, epsilon_out=None, step_offset: int = 0):
    E, A = q.shape
    dev = q.device
    if actions_out is None:
        actions_out = torch.empty(E, dtype=torch.int64, device=dev)
    call("ocppo_epsilon_greedy", _stream(dev), _check(q, "q", torch.float32, dev), E, A,
         int(seed) & 0xFFFFFFFFFFFFFFFF, _check(step, "step", torch.int64, dev, 1),
         int(step_offset), float(start_e),
         float(end_e), float(duration), _check(actions_out, "actions", torch.int64, dev, E),
         _opt(epsilon_out, "epsilon_out", torch.float32, dev, 1))
    return actions_out


def q_head_epsilon_greedy(hidden, wq, bq, seed: int, step, start_e: float, end_e: float,
                          duration: float, actions_out=None, epsilon_out=None,
                          step_offset: int = 0, q_out=None):
    """epsilon_greedy(hidden @ wq.T + bq, ...) in one launch (ocppo_q_head_epsilon_greedy)."""
    E, H = hidden.shape
    A = wq.shape[0]
    dev = hidden.device
    f = torch.float32
    if actions_out is None:
        actions_out = torch.empty(E, dtype=torch.int64, device=dev)
    call("ocppo_q_head_epsilon_greedy", _stream(dev), _check(hidden, "hidden", f, dev), E, H,
         _check(wq, "wq", f, dev, A * H), _check(bq, "bq", f, dev, A), A,
         int(seed) & 0xFFFFFFFFFFFFFFFF, _check(step, "step", torch.int64, dev, 1),
         int(step_offset), float(start_e), float(end_e), float(duration),
         _check(actions_out, "actions", torch.int64, dev, E),
         _opt(epsilon_out, "epsilon_out", f, dev, 1), _opt(q_out, "q_out", f, dev, E * A))
    return actions_out


def dqn_act_step_ok(hidden, wq, env, prev_obs, rb) -> bool:
    """dqn_act_step applies: <= 64 envs, the q_head_epsilon_greedy head shapes, an object-frame
    synthetic env and a replay in the stacks' dtype."""
    E, H = hidden.shape
    fr = getattr(env, "frame", None)
    return (getattr(env, "synthetic", False) and fr is not None and fr.dtype == torch.float32
            and fr.is_contiguous() and fr.shape[0] == E and 1 <= E <= 64
            and H % 256 == 0 and 256 <= H <= 1024 and 1 <= wq.shape[0] <= 8
            and hidden.is_contiguous() and wq.is_contiguous()
            and (hidden.data_ptr() | wq.data_ptr()) % 16 == 0
            and rb.obs.dtype == prev_obs.dtype and rb.E == E and prev_obs.is_contiguous()
            and rb.D == prev_obs[0].numel())


def dqn_act_step(hidden, wq, bq, seed: int, step, start_e: float, end_e: float, duration: float,
                 actions_out, epsilon_out, step_offset: int, env, env_step_offset: int, prev_obs,
                 obs_out, net_obs, done_out, reward_out, rb, vecnorm_state=None, gamma=0.99,
                 epsilon=1e-8, clip_reward=10.0, advance: int = 0):
    """q_head_epsilon_greedy + env.step + rollout_store(_vecnorm) + rb.add(prev_obs, obs_out,
    actions, reward_out, done_out) in one launch (ocppo_dqn_act_step; see dqn_act_step_ok);
    advance: then step += advance and env.advance(advance) in the same launch."""
    E, H = hidden.shape
    A = wq.shape[0]
    dev = hidden.device
    f = torch.float32
    W = obs_out.shape[1]
    D = env.frame.shape[1]
    if prev_obs.shape != obs_out.shape or prev_obs.dtype != obs_out.dtype or \
            obs_out[0, 0].numel() != D:
        raise ValueError("prev_obs / obs_out must be [E, W, D] stacks of one dtype")
    ret, rms = vecnorm_state if vecnorm_state is not None else (None, None)
    call("ocppo_dqn_act_step", _stream(dev), _check(hidden, "hidden", f, dev), E, H,
         _check(wq, "wq", f, dev, A * H), _check(bq, "bq", f, dev, A), A,
         int(seed) & 0xFFFFFFFFFFFFFFFF, _check(step, "step", torch.int64, dev, 1),
         int(step_offset), float(start_e), float(end_e), float(duration),
         _check(actions_out, "actions", torch.int64, dev, E),
         _opt(epsilon_out, "epsilon_out", f, dev, 1), env.seed & 0xFFFFFFFFFFFFFFFF,
         _check(env.step_base, "step_base", torch.int64, dev, 1), int(env_step_offset), D,
         _check(env.frame, "frame", f, dev, E * D), _check(env.reward, "reward", f, dev, E),
         _check(env.done, "done", f, dev, E), _opt(env.ep_state, "ep_state", f, dev, E * 5), W,
         _check(prev_obs, "prev_obs", None, dev, E * W * D),
         _check(obs_out, "obs_out", None, dev, E * W * D), _DTYPE_CODE[obs_out.dtype],
         _opt(net_obs, "net_obs", f, dev, E * W * D), _check(done_out, "done_out", f, dev, E),
         _check(reward_out, "reward_out", f, dev, E), int(vecnorm_state is not None),
         float(gamma), float(epsilon), float(clip_reward),
         _opt(ret, "ret_state", torch.float64, dev, E), _opt(rms, "rms_state", torch.float64, dev, 3),
         rb.state.data_ptr(), rb.size, rb.obs.data_ptr(), rb.actions.data_ptr(),
         rb.rewards.data_ptr(), rb.dones.data_ptr(), int(advance))
    return actions_out


def td_loss_fwd_bwd(q, q_next, actions, rewards, dones, gamma: float, dq=None, stats=None):
    """(stats [2] = {td_loss, mean q(s,a)}, dq [B, A] = d loss / d q)."""
    B, A = q.shape
    dev = q.device
    f = torch.float32
    if dq is None:
        dq = torch.empty_like(q)
    if stats is None:
        stats = torch.empty(2, dtype=f, device=dev)
    call("ocppo_td_loss_fwd_bwd", _stream(dev), _check(q, "q", f, dev),
         _check(q_next, "q_next", f, dev, B * A), _check(actions, "actions", torch.int64, dev, B),
         _check(rewards, "rewards", f, dev, B), _check(dones, "dones", f, dev, B), B, A,
         float(gamma), _check(dq, "dq", f, dev, B * A), _check(stats, "stats", f, dev, 2))
    return stats, dq
