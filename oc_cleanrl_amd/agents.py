"""Agents with the reference's duck-typed interface and module layout.

`PPObj` and `PPODefault` mirror cleanrl/architectures/ppo.py:15-95 module for module (same
nn.Sequential indices, so `state_dict()` keys such as `network.0.weight`, `actor.weight`,
`critic.bias` interchange with the reference's `.cleanrl_model` checkpoints), and construct and
initialise their layers in the same order (orthogonal init, architectures/ppo.py:9-13), so a
seeded construction reproduces the reference's weights bit for bit.

The network forward/backward stays in PyTorch (hipBLASLt / MIOpen); what changes is the action
head: `get_action_and_value` samples, scores and takes the entropy with the HIP Categorical
kernels (one launch instead of logsumexp/softmax/multinomial/gather/entropy chains, and no
host sync — torch's multinomial syncs on `probs.max() < inf`). The sampler consumes the default
device generator exactly like torch's Categorical.sample (an Exp(1) draw of shape [B, A]), so
actions are bit-identical to the reference's under the same seed.
"""
from __future__ import annotations

import threading

import numpy as np
import torch
import torch.nn as nn

from . import ops


def layer_init(layer, std=np.sqrt(2), bias_const=0.0):
    """Orthogonal weight, constant bias (architectures/ppo.py:9-13, common.py:7-10)."""
    nn.init.orthogonal_(layer.weight, std)
    if layer.bias is not None:
        nn.init.constant_(layer.bias, bias_const)
    return layer


class NormalizeImg(nn.Module):
    """x / 255 (architectures/common.py:19-22)."""

    @staticmethod
    def forward(x):
        return x / 255.0


class Predictor(nn.Module):
    """Greedy `predict` used by the eval harness (architectures/common.py:13-16)."""

    def predict(self, x, states=None, **_):
        with torch.no_grad():
            dev = next(self.parameters()).device
            logits = self.actor(self.network(torch.as_tensor(np.asarray(x), dtype=torch.float32,
                                                             device=dev)))
            return np.argmax(logits.cpu().numpy(), axis=1), states


def _splitk(rows: int, k: int, n: int) -> int:
    """K-split for the weight-gradient GEMM dW = g^T x (rows = reduction length): hipBLASLt's
    default kernels leave the tall-skinny update shapes at 2-42 TFLOP/s; a batched GEMM over
    row chunks + a sum restores 100+ TFLOP/s (tools/exp_gemm_shapes.py, gfx950)."""
    if rows < 8192:
        return 8 if k * n <= 16384 and rows % 8 == 0 else 1
    if k * n <= 4096:
        s = 8  # [12288 x 12] x [12288 x 256]: 13.3 us at 8 vs 22.8 at 16 (exp_update_gemms.py)
    elif k * n <= 16384:
        s = 16
    elif k * n <= 131072:
        s = 4
    else:
        s = 8
    while rows % s:
        s //= 2
    return max(s, 1)


# The update's f32 GEMMs on the bf16 matrix cores (ops.gemm_x6: each f32 operand split exactly
# into three bf16 pieces, six piece products accumulated in f32 -- f32 accuracy at 6/16 of the f32
# MFMA's time, tests/test_gemm_gpu.py); shapes it does not tile stay on hipBLASLt. The route is
# per parameter: a Linear whose weight carries `_ocppo_x6` (set_update_gemm, done by each
# PPOTrainer for its own agent from Args.x6_gemm) uses that; any other weight uses this default.
X6_GEMM_DEFAULT = True
# Where it wins (tools/exp_gemm_x6.py at the config-2 update shapes): products whose output holds
# >= 256 tiles of 128 x 128 (forward / dX), and weight gradients with >= 32 such tiles (the rows
# split over up to 16 workgroups per tile); smaller outputs leave the chip half idle and stay on
# hipBLASLt (e.g. the decoder forward [4096 x 512] from K = 2048: 84 vs 63 us).
X6_MIN_TILES, X6_MIN_TILES_DW = 256, 32
# Forward products with 32-255 such tiles as K-split gemm_x6 + a combine with the bias / ReLU
# epilogue (ops.x6_fwd_splits: the decoder forward [4096 x 512] from K = 2048)
X6_FWD_SPLITK = True


def x6_route(w) -> bool:
    """The update-GEMM route of the Linear owning weight `w` (gemm_x6 or hipBLASLt)."""
    return bool(getattr(w, "_ocppo_x6", X6_GEMM_DEFAULT))


def set_update_gemm(module: nn.Module, x6: bool) -> None:
    """Route every Linear of `module` (forward, dX, dW and the fused ReLU-backward dX epilogue)
    through gemm_x6 (x6) or hipBLASLt: per-agent state, so two trainers in one process with
    different Args.x6_gemm do not interfere."""
    for m in module.modules():
        if isinstance(m, nn.Linear):
            m.weight._ocppo_x6 = bool(x6)


# Pre-split weights (ops.WeightPlanes): the forward's and dX's B operand read as three bf16 planes
# split once per minibatch instead of in every row tile's K loop (bitwise the same products).
# Only inside a weight_planes() scope, opened by the owner that refreshed the planes after the
# last optimizer step (the trainer, per minibatch): outside it a weight's planes may be stale.
_PLANES = threading.local()


class weight_planes:
    """Scope in which _LinearAct reads its weight's pre-split planes (w._ocppo_planes)."""

    def __enter__(self):
        _PLANES.live = getattr(_PLANES, "live", 0) + 1
        return self

    def __exit__(self, *exc):
        _PLANES.live -= 1


def _planes(w, kind: str):
    if not getattr(_PLANES, "live", 0):
        return None
    d = getattr(w, "_ocppo_planes", None)
    return None if d is None else d.get(kind)


def _x6(M: int, N: int, K: int, on: bool = True) -> bool:
    """Forward / dX product [M, N] = [M, K] x [K, N] on gemm_x6."""
    return on and M * N >= X6_MIN_TILES * 16384 and K >= 64


def _x6_dw(n: int, k: int, rows: int, on: bool = True) -> bool:
    """Weight gradient [n, k] = g^T x over `rows` on gemm_x6."""
    return on and n * k >= X6_MIN_TILES_DW * 16384 and rows >= 1024


# The pipelined gemm_x6 tile (ops.X6_PIPE: 128 x 256, two LDS stages, one workgroup per CU) for
# the products that fill exactly one wave of 256 workgroups with it: the encoder weight
# gradients [1024 x 512] / [512 x 1024] as 16 row splits (63.6 / 63.3 vs 71.2 / 69.9 us with the
# combine) and the decoder's dX [4096 x 2048] (44.7 vs 49.8 us), profiles/r05/exp_x6_pipe.txt
X6_PIPE = True


def x6_pipe_tile(M: int, N: int, splits: int = 1):
    """58 when [M x N] x splits is exactly 256 tiles of 128 x 256, else None."""
    if not X6_PIPE or M % 128 or N % 256:
        return None
    return 58 if splits * (M // 128) * (N // 256) == 256 else None


def _x6_pipe_splits(rows: int, n: int, k: int):
    """(splits, 58) for dW = g^T x [n, k] when some split count in 1..16 gives exactly 256
    pipelined tiles with >= 8 K steps per split (the rows' 32-row steps dealt to the splits as
    evenly as they go, as gemm_x6 does: 11520 rows = 360 steps, 22-23 per split of 16); else
    None."""
    if rows % 32:
        return None
    for s in (1, 2, 4, 8, 16):
        if x6_pipe_tile(n, k, s) and rows // 32 >= 8 * s:
            return s, 58
    return None


def _x6_splits(rows: int, n: int, k: int):
    """(splits, variant) of dW = g^T x on gemm_x6 (rows in steps of 32, split evenly): the
    largest tile that reaches >= 512 workgroups (two per CU) over the [n, k] output with at most
    16 splits, at the fewest splits; else the most workgroups. The combine is sum_splits[_db]."""
    if rows % 32:
        return None
    best, best_units = None, -1
    for t in range(ops.X6_AUTO, ops.X6_AUTO + 4):
        bm, bn = ops.X6_TILES[t]
        if n % bm or k % bn:
            continue
        for s in (1, 2, 4, 8, 16):
            if s > rows // 32:
                break
            units = s * (n // bm) * (k // bn)
            if units >= 512:
                return s, t
            if units > best_units:
                best, best_units = (s, t), units
    return best


# The ReLU backward + bias-gradient partials of a Linear+ReLU layer fused into the next layer's
# dX GEMM (ops.dx_x6_relu) on the gemm_x6 route: replaces that layer's relu_bias_grad pass.


def _x6_dx_shape_ok(M: int, N: int, K: int, on: bool = True) -> bool:
    """dX [M, K] = g [M, N] W [N, K] runs on gemm_x6 (agents._dx's rule, decided from shapes)."""
    return _x6(M, K, N, on) and N % 32 == 0 and ops.x6_tile(M, K) is not None


def _weight_grad(g, x, out=None, db=None, x6: bool = True, finish=None):
    """dW = g^T x (g [rows, n], x [rows, k]) with the split-K rule; written into `out` if given.
    db = (partials of ops.relu_bias_grad_partial, bias grad): the bias gradient is finished in
    the same launch as the split-K combine (only when _defer_db_ok said so). finish = a pending
    ops.DeferredFinish (the heads-loss finish): folded into the split-K combine when there is
    one, else run right after."""
    if finish is not None and finish.pending:
        dw = _weight_grad_core(g, x, out, db, x6, finish)
        finish.run()  # no-op when the combine took it
        return dw
    return _weight_grad_core(g, x, out, db, x6, None)


def _weight_grad_core(g, x, out, db, x6, finish):
    rows, n = g.shape
    k = x.shape[1]
    s = _splitk(rows, k, n)
    st = ((_x6_pipe_splits(rows, n, k) or _x6_splits(rows, n, k)) if _x6_dw(n, k, rows, x6)
          else None)
    if st is not None and ops.dw_x6_ok(g, x, st[0]):
        s6, t6 = st
        if s6 == 1 and out is not None and db is None and out.is_contiguous():
            return ops.gemm_x6(g, 1, g.stride(0), x, 1, x.stride(0), out, k, n, k, rows, tile=t6)
        s = s6
        part = ops.dw_x6_parts(g, x, s, tile=t6)
    elif s == 1:
        return torch.mm(g.t(), x, out=out) if out is not None else g.t().mm(x)
    else:
        part = torch.bmm(g.view(s, rows // s, n).transpose(1, 2), x.view(s, rows // s, k))
    if db is not None:
        if finish is not None:
            return ops.timed(f"sum_splits_db_fin_{s}x{n}x{k}",
                             lambda: ops.sum_splits_db(part, out, *db, finish=finish))
        return ops.timed(f"sum_splits_db_{s}x{n}x{k}", lambda: ops.sum_splits_db(part, out, *db))
    if out is not None and HIP_SUM_SPLITS and ops.sum_splits_ok(part, out):
        if finish is not None:
            return ops.timed(f"sum_splits_fin_{s}x{n}x{k}",
                             lambda: ops.sum_splits(part, out, finish=finish))
        return ops.timed(f"sum_splits_{s}x{n}x{k}", lambda: ops.sum_splits(part, out))
    return torch.sum(part, 0, out=out) if out is not None else part.sum(0)


# dX = g W for a few hundred rows and <= 256 output columns: hipBLASLt's kernel for
# [128 x 512] x [512 x 256] (the DQN train step's second encoder layer) takes ~60 us; the HIP
# rollout Linear kernel on W^T takes 4.0 us + 2.9 us for the transpose (tools/exp_dqn_gemms.py).
HIP_SMALL_DX = True


def _dx(g, w, x6: bool = True, planes=None):
    M, N = g.shape
    K = w.shape[1]
    if _x6(M, K, N, x6) and ops.dx_x6_ok(g, w):
        return ops.dx_x6(g, w, planes=planes, tile=x6_pipe_tile(M, K))
    if (HIP_SMALL_DX and g.is_cuda and M <= 256 and K <= 256 and N >= 256 and N % 16 == 0 and
            g.dtype == torch.float32 and g.is_contiguous()):
        return ops.linear_act(g, w.t().contiguous())
    return g.mm(w)


def _defer_db_ok(g, x, wgrad, b) -> bool:
    """The bias gradient can ride in the split-K combine of the weight gradient (HIP sum_splits
    path, FlatAdam-owned aligned grads; wgrad = where the weight gradient is written)."""
    rows, n = g.shape
    k = x.shape[1]
    return (DEFER_BIAS_GRAD and HIP_SUM_SPLITS and _splitk(rows, k, n) > 1 and (n * k) % 4 == 0
            and n % 4 == 0 and wgrad.data_ptr() % 16 == 0 and b.grad.data_ptr() % 16 == 0
            and wgrad.is_contiguous())


def _cols_to_nhwc(w, chw):
    """Linear weight [O, C*H*W] (columns in nn.Flatten's NCHW order) -> [O, H*W*C] (a copy)."""
    C, H, W = chw
    return w.view(w.shape[0], C, H, W).permute(0, 2, 3, 1).reshape(w.shape[0], H * W * C)


def _cols_from_nhwc(w_nhwc, chw, out=None):
    """Inverse of _cols_to_nhwc, written into `out` when given."""
    C, H, W = chw
    v = w_nhwc.view(w_nhwc.shape[0], H, W, C).permute(0, 3, 1, 2)
    if out is not None:
        out.view(out.shape[0], C, H, W).copy_(v)
        return out
    return v.reshape(w_nhwc.shape[0], C * H * W)


# relu_bias_grad without its last-arriver tail: bias-gradient chunk sums finished by the weight
# gradient's split-K combine (ops.relu_bias_grad_partial + ops.sum_splits_db).
DEFER_BIAS_GRAD = True

# The second encoder layer's weight gradient computed after the first layer's rows launch, so
# that launch's finish rides in its split-K combine (ops.sum_splits_db(..., finish=)).
DEFER_WGRAD_AFTER_FIRST_LAYER = True

# The second encoder layer's dX on gemm_x6 with the first layer's whole backward in its epilogue
# (ops.dx_x6_wgrad): the dX is never stored and relu_bias_wgrad's rows launch is gone.
FUSED_L1_IN_DX = True


# Split-K partials of FlatAdam-owned weight gradients summed by one HIP pass (ops.sum_splits).
HIP_SUM_SPLITS = True


def _direct(p) -> bool:
    """Parameters owned by ops.FlatAdam get their grads written in place (no AccumulateGrad)."""
    return getattr(p, "_ocppo_direct_grad", False) and p.grad is not None


# Autograd forwards of <= SMALL_FWD_ROWS rows on the HIP rollout Linear kernel (ops.linear_act,
# f32 MFMA, LDS-staged; bias + ReLU epilogue) instead of hipBLASLt: at these sizes both are launch-
# and latency-bound and the library's kernels take 8-10 us against 4-6 (the DQN train step's
# forwards at 128 / 32 rows, profiles/r05/dqn/fused_step_kernel_stats.csv)
SMALL_FWD = True
SMALL_FWD_ROWS = 128


def _small_fwd_ok(x, w) -> bool:
    if not (SMALL_FWD and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and
            w.dtype == torch.float32 and w.is_contiguous()):
        return False
    M, K = x.shape
    return (1 <= M <= SMALL_FWD_ROWS and (M == 1 or x.stride(1) == 1) and
            (K <= 64 or (K <= 2048 and K % 16 == 0)))


class _LinearAct(torch.autograd.Function):
    """y = act(x @ W^T + b), act = ReLU (one hipBLASLt GEMM with a bias+ReLU epilogue,
    torch._addmm_activation) or identity (addmm). Backward = autograd's linear(+ReLU) formulas
    (threshold_backward, dX = g'W, dW = g'^T x, db = sum g') with a split-K weight gradient, and
    for FlatAdam-owned parameters dW/db are written straight into the flat grad buffer."""

    @staticmethod
    def forward(ctx, x, w, b, relu: bool, box=None, chw=None, below=None, wslot=None):
        # chw = (C, H, W): x is a channels_last activation flattened in its memory (H, W, C)
        # order, so the weight's columns are permuted to match instead (linear_act_nhwc)
        wm = _cols_to_nhwc(w, chw) if chw is not None else w
        x6 = ctx.x6 = x6_route(w)
        pf, ctx.pdx = (_planes(w, "fwd"), _planes(w, "dx")) if chw is None else (None, None)
        # below = the box of the Linear+ReLU that produced x: its ReLU backward and bias-gradient
        # partials ride in this layer's dX GEMM (ops.dx_x6_relu, mask = x)
        ctx.below = None
        if (x6 and below is not None and not below["premasked"]
                and (chw is None or below.get("conv"))
                and x.requires_grad and _x6_dx_shape_ok(x.shape[0], wm.shape[0], x.shape[1])):
            below["premasked"] = True
            ctx.below = below
        fs = (ops.x6_fwd_splits(x.shape[0], wm.shape[0], x.shape[1])
              if x6 and X6_FWD_SPLITK else None)
        if _x6(x.shape[0], wm.shape[0], x.shape[1], x6) and ops.linear_x6_ok(x, wm):
            if relu and box is not None:
                # the ReLU bitmask for the box's consumer: the next layer's fused dX epilogue
                # (fragment order), or the frame scatter (row-major)
                out, box["mbits"] = ops.linear_x6(x, wm, b, relu,
                                                  mbits="rows" if box.get("rows") else True,
                                                  planes=pf)
            else:
                out = ops.linear_x6(x, wm, b, relu, planes=pf)
        elif chw is None and _small_fwd_ok(x, wm):
            # a few rows under autograd (the DQN train step's batch of 32, CartPole's minibatch):
            # the rollout's LDS-staged f32-MFMA kernel instead of a library launch
            out = ops.linear_act(x, wm, b, relu)
        elif fs is not None and ops._x6_operand_ok(x) and ops._x6_operand_ok(wm) and \
                (b is None or b.data_ptr() % 16 == 0):
            # K-split partials + the combine with bias / ReLU (no bitmask: a consumer's fused dX
            # reads the f32 output as its mask)
            out = ops.linear_x6_split(x, wm, b, relu, fs, planes=pf)
        else:
            out = torch._addmm_activation(b, x, wm.t(), use_gelu=False) if relu else \
                torch.addmm(b, x, wm.t())
        ctx.relu = relu
        ctx.save_for_backward(x, w, out if relu else None)
        ctx.w, ctx.b = w, b
        ctx.chw, ctx.wm = chw, (wm if chw is not None else None)
        ctx.box = box  # _Heads sets box["premasked"]: g arrives masked, bias grad already written
        # wslot: x is the first encoder layer's output (frames._GatherLinear1), whose backward
        # runs after this one; this layer's weight gradient may wait for it (see _backward)
        ctx.wslot = wslot
        return out

    @staticmethod
    def backward(ctx, g):
        chw = ctx.chw
        if chw is None:
            return _LinearAct._backward(ctx, g, ctx.w.grad) + (None, None)
        # permuted columns: weight gradient formed in the NHWC column order, then put back
        direct = _direct(ctx.w)
        wgrad = torch.empty_like(ctx.wm) if direct else None
        dx, dw, db, _, _, _ = _LinearAct._backward(ctx, g, wgrad)
        if direct and ctx.needs_input_grad[1]:
            _cols_from_nhwc(wgrad, chw, out=ctx.w.grad)
        if dw is not None:
            dw = _cols_from_nhwc(dw, chw)
        return dx, dw, db, None, None, None, None, None

    @staticmethod
    def _dx_of(ctx, g, w):
        """dX of this layer; when the forward claimed the layer below's ReLU backward (ctx.below:
        x is that layer's ReLU output, consumed by this layer alone — fused_trunk's chains), the
        mask and the below layer's bias-gradient partials come with it. Operands the fused C
        entry refuses (layout, alignment) take the plain dX plus the same two results, so the
        claim always holds."""
        if ctx.below is None:
            return _dx(g, w, ctx.x6, ctx.pdx)
        x = ctx.saved_tensors[0]
        if ctx.below.get("conv"):
            # a convolution's ReLU output flattened in its (H, W, C) memory order: the bias
            # gradient sums the masked gradient over rows and positions per channel C
            C = ctx.chw[0]
            b = ctx.below["bias"]
            db = b.grad if _direct(b) else torch.empty_like(b)
            if ops.dx_x6_ok(g, w):
                gp, dbp = ops.dx_x6_relu(g, w, x, planes=ctx.pdx)
                db.copy_(dbp.view(-1, C).double().sum(0))  # row tiles and positions, f64
            else:
                dx = _dx(g, w, ctx.x6, ctx.pdx).contiguous()
                gp, _ = ops.relu_bias_grad(dx.view(-1, C), x.contiguous().view(-1, C), db=db)
                gp = gp.view(dx.shape)
            ctx.below["db"] = db
            return gp
        if ops.dx_x6_ok(g, w):
            gp, dbp = ops.dx_x6_relu(g, w, x, mbits=ctx.below.get("mbits"), planes=ctx.pdx)
            ctx.below["dbp"] = (dbp, dbp.shape[0])  # relu_bias_grad_partial's (partials, chunks)
            return gp
        dx = _dx(g, w, ctx.x6, ctx.pdx).contiguous()
        if ops.relu_bias_grad_ok(dx):
            gp, ctx.below["dbp"] = ops.relu_bias_grad_partial(dx, x.contiguous())
        else:
            gp = torch.ops.aten.threshold_backward(dx, x, 0)
            ctx.below["dbp"] = (gp.sum(0, keepdim=True), 1)
        return gp

    @staticmethod
    def _backward(ctx, g, wgrad):
        x, w, out = ctx.saved_tensors
        if ctx.wm is not None:
            w = ctx.wm
        db = None
        bias_done = False
        g = g.contiguous()
        if ctx.box is not None and ctx.box["premasked"]:
            # the consumer already applied this layer's ReLU mask: the fused heads backward
            # (_Heads) also wrote its bias gradient; the frame scatter (frames._FramesExpand)
            # left the bias-gradient partials in the box ("dbp"). Only dX and dW remain.
            dbp = ctx.box.get("dbp")
            l1 = ctx.wslot.get("l1") if ctx.wslot is not None else None
            if (l1 is not None and dbp is not None and FUSED_L1_IN_DX and ctx.x6 and
                    ctx.needs_input_grad[0] and _defer_db_ok(g, x, wgrad, ctx.b) and
                    ops.dx_x6_wgrad_ok(g, w, x, l1[0])):
                # this layer's dX is never stored: its epilogue runs the first layer's backward
                # (mask = x, that layer's ReLU output; ops.dx_x6_wgrad), finished in this layer's
                # weight-gradient combine; no gradient flows down (the slot says "done")
                xf, w1, b1 = l1
                fin = ops.DeferredFinish(g.device)
                ops.dx_x6_wgrad(g, w, x, xf, w1.grad, b1.grad, fin)
                ctx.wslot["done"] = True
                _weight_grad(g, x, out=wgrad, db=(dbp, ctx.b.grad), x6=ctx.x6, finish=fin)
                return None, None, None, None, None, None
            dx = _LinearAct._dx_of(ctx, g, w) if ctx.needs_input_grad[0] else None
            if dbp is None:
                _weight_grad(g, x, out=wgrad, x6=ctx.x6, finish=ctx.box.get("finish"))
            elif _defer_db_ok(g, x, wgrad, ctx.b):
                if ctx.wslot is not None and DEFER_WGRAD_AFTER_FIRST_LAYER:
                    # after the first layer's rows launch, with its finish in this combine
                    # (frames._GatherLinear1.backward runs it: the finish-carrying
                    # sum_splits_db saves the finish's own launch)
                    bg, x6 = ctx.b.grad, ctx.x6
                    ctx.wslot["run"] = lambda fin, g=g, x=x, wg=wgrad: _weight_grad(
                        g, x, out=wg, db=(dbp, bg), x6=x6, finish=fin)
                else:
                    _weight_grad(g, x, out=wgrad, db=(dbp, ctx.b.grad), x6=ctx.x6)
            else:
                _weight_grad(g, x, out=wgrad, x6=ctx.x6)
                torch.sum(dbp[0], 0, out=ctx.b.grad)
            return dx, None, None, None, None, None
        if FUSED_FIRST_LAYER_BWD and not ctx.needs_input_grad[0] and ctx.needs_input_grad[1] \
                and ctx.needs_input_grad[2] and _direct(ctx.w) and _direct(ctx.b) and \
                ops.relu_bias_wgrad_ok(g, x):
            # input layer (no dX): ReLU-backward + bias grad + weight grad in one HIP pass
            o = out if ctx.relu else None
            ops.timed(f"relu_bias_wgrad_{g.shape[0]}x{g.shape[1]}x{x.shape[1]}",
                      lambda: ops.relu_bias_wgrad(g, o, x, dw=wgrad, db=ctx.b.grad))
            return None, None, None, None, None, None
        if FUSED_RELU_BIAS_GRAD and ctx.needs_input_grad[2] and _direct(ctx.b) and \
                ops.relu_bias_grad_ok(g) and ctx.needs_input_grad[1] and _direct(ctx.w) and \
                _defer_db_ok(g, x, wgrad, ctx.b):
            # ReLU-backward in one pass, bias grad finished with the split-K weight-grad combine
            o = out if ctx.relu else None
            gp, dbp = ops.timed(f"relu_bias_grad_{g.shape[0]}x{g.shape[1]}" +
                                ("" if ctx.relu else "_norelu"),
                                lambda: ops.relu_bias_grad_partial(g, o))
            dx = _LinearAct._dx_of(ctx, gp, w) if ctx.needs_input_grad[0] else None
            _weight_grad(gp, x, out=wgrad, db=(dbp, ctx.b.grad), x6=ctx.x6)
            return dx, None, None, None, None, None
        if FUSED_RELU_BIAS_GRAD and ctx.needs_input_grad[2] and _direct(ctx.b) and \
                ops.relu_bias_grad_ok(g):
            # threshold_backward + bias sum in one HIP pass, bias grad written in place
            o, db_out = out if ctx.relu else None, ctx.b.grad
            gp, _ = ops.timed(f"relu_bias_grad_{g.shape[0]}x{g.shape[1]}" +
                              ("" if ctx.relu else "_norelu"),
                              lambda: ops.relu_bias_grad(g, o, db=db_out))
            bias_done = True
        else:
            gp = torch.ops.aten.threshold_backward(g, out, 0) if ctx.relu else g
        dx = _LinearAct._dx_of(ctx, gp, w) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            if _direct(ctx.w):
                _weight_grad(gp, x, out=wgrad, x6=ctx.x6)
            else:
                dw = _weight_grad(gp, x, x6=ctx.x6)
        if ctx.needs_input_grad[2] and not bias_done:
            if _direct(ctx.b):
                torch.sum(gp, 0, out=ctx.b.grad)
            else:
                db = gp.sum(0)
        return dx, dw, db, None, None, None


class _Heads(torch.autograd.Function):
    """logits = h Wa^T + ba, value = h Wc^T + bc (architectures/ppo.py:81-84, the two head
    Linears on the decoder output h). Backward = ONE HIP pass (ops.heads_bwd): dh from both heads,
    the dW / db of both heads and, when h is the ReLU output of a Linear whose grads are written in
    place (box), that layer's ReLU mask and bias gradient too (its _LinearAct backward then only
    runs dX / dW). Same formulas as autograd's, fixed summation orders."""

    @staticmethod
    def forward(ctx, h, wa, ba, wc, bc, box):
        logits = torch.addmm(ba, h, wa.t())
        value = torch.addmm(bc, h, wc.t())
        ctx.save_for_backward(h, wa, wc)
        ctx.params = (wa, ba, wc, bc)
        ctx.box = box
        if box is not None:
            box["premasked"] = True
        return logits, value

    @staticmethod
    def backward(ctx, g_logits, g_value):
        h, wa, wc = ctx.saved_tensors
        pa, pba, pc, pbc = ctx.params
        M, A = h.shape[0], wa.shape[0]
        if g_logits is None:
            g_logits = torch.zeros(M, A, dtype=h.dtype, device=h.device)
        if g_value is None:
            g_value = torch.zeros(M, 1, dtype=h.dtype, device=h.device)
        box = ctx.box
        db_h = box["bias"].grad if box is not None else None
        outs = [p.grad if _direct(p) else None for p in (pa, pc, pba, pbc)]
        gp, _, dwa, dwc, dba, dbc = ops.timed(
            "heads_bwd", lambda: ops.heads_bwd(
                h, g_logits.contiguous(), g_value.reshape(-1).contiguous(), wa, wc.reshape(-1),
                relu=box is not None, db_h=db_h, dwa=outs[0], dwc=outs[1], dba=outs[2],
                dbc=outs[3]))
        ret = [None if outs[i] is not None else t for i, t in enumerate((dwa, dwc, dba, dbc))]
        return gp, ret[0], ret[2], ret[1], ret[3], None


class _QHead(torch.autograd.Function):
    """q = h Wq^T + bq, a single head (the DQN Q head, architectures/dqn.py:14-25 and the obj
    Q-network's last Linear): backward = ops.heads_bwd without a critic row, with the producing
    layer's ReLU mask + bias grad when `box` says so (as _Heads)."""

    @staticmethod
    def forward(ctx, h, wq, bq, box):
        ctx.save_for_backward(h, wq)
        ctx.params = (wq, bq)
        ctx.box = box
        if box is not None:
            box["premasked"] = True
        if _small_fwd_ok(h, wq) and bq is not None:
            return ops.linear_act(h, wq, bq, False)
        return torch.addmm(bq, h, wq.t())

    @staticmethod
    def backward(ctx, g):
        h, wq = ctx.saved_tensors
        pw, pb = ctx.params
        box = ctx.box
        db_h = box["bias"].grad if box is not None else None
        ow, ob = (pw.grad if _direct(pw) else None), (pb.grad if _direct(pb) else None)
        gp, _, dw, _, db, _ = ops.timed("heads_bwd", lambda: ops.heads_bwd(
            h, g.contiguous(), None, wq, None, relu=box is not None, db_h=db_h, dwa=ow, dba=ob))
        return gp, (None if ow is not None else dw), (None if ob is not None else db), None


def q_head(hidden, lin: nn.Linear):
    """lin(hidden) for the last Linear of a Q-network; the fused single-head backward under
    autograd on the GPU (same single-consumer contract as _ActorCritic.heads)."""
    if (FUSED_HEADS_BWD and torch.is_grad_enabled() and hidden.requires_grad and hidden.is_cuda
            and hidden.dtype == torch.float32 and hidden.dim() == 2 and lin.bias is not None
            and ops.heads_bwd_ok(hidden, lin.out_features)):
        return _QHead.apply(hidden, lin.weight, lin.bias, getattr(hidden, "_ocppo_box", None))
    return linear_act(hidden, lin, False) if hidden.is_cuda else lin(hidden)


# Actor + critic backward (and the decoder's ReLU mask + bias grad) as one HIP pass (_Heads).
FUSED_HEADS_BWD = True


def heads_ok(h, actor, critic) -> bool:
    return (FUSED_HEADS_BWD and torch.is_grad_enabled() and h.requires_grad and h.is_cuda and
            h.dtype == torch.float32 and h.dim() == 2 and isinstance(actor, nn.Linear) and
            isinstance(critic, nn.Linear) and actor.bias is not None and critic.bias is not None
            and critic.out_features == 1 and ops.heads_bwd_ok(h, actor.out_features))


# One-pass HIP ReLU-backward + bias gradient (ops.relu_bias_grad) for FlatAdam-owned biases.
FUSED_RELU_BIAS_GRAD = True
# Input layers with K <= 16 features (PPObj's first encoder layer): ReLU-backward, bias and
# weight gradient in one HIP pass (ops.relu_bias_wgrad), gp never materialised.
FUSED_FIRST_LAYER_BWD = True


class _ConvAct(torch.autograd.Function):
    """y = act(conv2d(x, w) + b) for a channels_last (NHWC) input: MIOpen's bias-less NHWC
    convolution, then ONE HIP pass for bias + ReLU (ATen runs them as two); backward: ONE HIP pass
    for ReLU-backward + bias gradient over the NHWC gradient viewed [B*H*W, C]
    (ops.relu_bias_grad), then aten.convolution_backward for dX / dW. Same arithmetic as
    nn.Conv2d + nn.ReLU up to the bias-gradient summation order (architectures/ppo.py:20-31)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, relu: bool):
        y = torch.ops.aten.convolution(x, w, None, stride, padding, (1, 1), False, (0, 0), 1)
        y = y.contiguous(memory_format=torch.channels_last)
        C = y.shape[1]
        ops.timed("bias_act", lambda: ops.bias_act(y.permute(0, 2, 3, 1).reshape(-1, C), b, relu))
        ctx.conv = (stride, padding, relu)
        ctx.b = b
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, y = ctx.saved_tensors
        stride, padding, relu = ctx.conv
        g = g.contiguous(memory_format=torch.channels_last)
        C = g.shape[1]
        g2 = g.permute(0, 2, 3, 1).reshape(-1, C)
        b = ctx.b
        direct_b = _direct(b)
        db_out = b.grad if direct_b else torch.empty_like(b)
        o2 = y.permute(0, 2, 3, 1).reshape(-1, C) if relu else None
        gp2, _ = ops.timed(f"relu_bias_grad_{g2.shape[0]}x{C}" + ("" if relu else "_norelu"),
                           lambda: ops.relu_bias_grad(g2, o2, db=db_out))
        gp = gp2.view(g.shape[0], g.shape[2], g.shape[3], C).permute(0, 3, 1, 2)
        dx, dw, _ = torch.ops.aten.convolution_backward(
            gp, x, w, None, stride, padding, (1, 1), False, (0, 0), 1,
            (ctx.needs_input_grad[0], ctx.needs_input_grad[1], False))
        if dw is not None and _direct(w):
            w.grad.copy_(dw)
            dw = None
        return dx, dw, (None if direct_b else db_out), None, None, None


class _ConvX6(torch.autograd.Function):
    """y = act(conv2d(x, w) + b) on this package's implicit GEMMs (ops.conv_x6: bias + ReLU in
    the product's epilogue); backward: ONE HIP pass for ReLU-backward + bias gradient
    (ops.relu_bias_grad, as _ConvAct), then the weight gradient and, when x needs one, the data
    gradient on ops.conv_x6_wgrad / conv_x6_dgrad. No MIOpen and no atomics: deterministic, the
    reference's torch.use_deterministic_algorithms(True) default (ppo_atari_oc.py:200-211) at full
    speed. nn.Conv2d + nn.ReLU's arithmetic at f32 accuracy (architectures/ppo.py:20-31)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, relu: bool, box=None, below=None):
        B, Cin, H, W = x.shape
        Cout = w.shape[0]
        wp = _planes(w, "fwd") if CONV_X6_PLANES else None  # refreshed by the trainer
        OH = (H - w.shape[2]) // stride + 1
        mb = (torch.empty(B * OH * OH * Cout // 32, dtype=torch.int32, device=x.device)
              if CONV_RELU_BITS and relu and Cout % 32 == 0 and H == W and
              not ops._conv_rows_form(B * OH * OH, Cout) else None)
        y = ops.timed(f"conv_x6_{B}x{Cin}x{H}_{Cout}",
                      lambda: ops.conv_x6(x, w, b, stride, relu, w_planes=wp, mbits=mb))
        ctx.conv = (stride, relu)
        ctx.b = b
        ctx.mb = mb
        ctx.box, ctx.below = box, below
        ctx.save_for_backward(x, w, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, y = ctx.saved_tensors
        stride, relu = ctx.conv
        cl = torch.channels_last
        g = g.contiguous(memory_format=cl)
        B, C, OH, OW = g.shape
        g2 = g.permute(0, 2, 3, 1).reshape(-1, C)
        b = ctx.b
        mb, ctx.mb = ctx.mb, None
        gp2, db_out, direct_b = _conv_relu_backward(ctx.box, g2, y, b, relu, bits=mb)
        KH, KW = w.shape[2], w.shape[3]
        dw = None
        if ctx.needs_input_grad[1]:
            if _direct(w) and w.grad.is_contiguous(memory_format=cl):
                ops.timed(f"conv_x6_wgrad_{C}x{KH * KW * x.shape[1]}",
                          lambda: ops.conv_x6_wgrad(gp2, x, (KH, KW), stride, out=w.grad))
            else:
                dw = ops.conv_x6_wgrad(gp2, x, (KH, KW), stride)
                dw = dw.view(C, KH, KW, x.shape[1]).permute(0, 3, 1, 2)
                if _direct(w):
                    w.grad.copy_(dw)
                    dw = None
        dx = None
        if ctx.needs_input_grad[0]:
            gp = gp2.view(B, OH, OW, C).permute(0, 3, 1, 2)
            hw = (x.shape[2], x.shape[3])
            below = ctx.below
            if below is not None and CONV_DGRAD_RELU and ops.conv_x6_dgrad_fuses_relu(
                    B * (hw[0] // stride) * (hw[1] // stride), x.shape[1], stride):
                # the layer below's ReLU backward + bias gradient in this dX's epilogue
                bb = below["bias"]
                db_below = bb.grad if _direct(bb) else torch.empty_like(bb)
                dx = ops.timed(f"conv_x6_dgrad_relu_{C}x{x.shape[1]}",
                               lambda: ops.conv_x6_dgrad(gp, w, stride, hw, relu_out=x,
                                                         db=db_below))
                below.update(premasked=True, db=db_below)
            else:
                dx = ops.timed(f"conv_x6_dgrad_{C}x{x.shape[1]}",
                               lambda: ops.conv_x6_dgrad(gp, w, stride, hw))
        return dx, dw, (None if direct_b else db_out), None, None, None, None


def _conv_relu_backward(box, g2, y, b, relu: bool, bits=None):
    """(gp rows, bias gradient, whether it went to b.grad in place) of a convolution + ReLU whose
    output gradient rows are g2: one relu_bias_grad pass, or nothing when the layer above's data
    gradient already applied this ReLU's backward and wrote the bias gradient (box premasked)."""
    direct_b = _direct(b)
    if box is not None and box.get("premasked"):
        box["premasked"] = False
        return g2, box["db"], direct_b
    C = g2.shape[1]
    db_out = b.grad if direct_b else torch.empty_like(b)
    if relu and bits is not None:  # the forward epilogue's row-major ReLU bitmask
        gp2, _ = ops.timed(f"relu_bias_grad_bits_{g2.shape[0]}x{C}",
                           lambda: ops.relu_bias_grad(g2, db=db_out, bits=bits))
        return gp2, db_out, direct_b
    o2 = y.permute(0, 2, 3, 1).reshape(-1, C) if relu else None
    gp2, _ = ops.timed(f"relu_bias_grad_{g2.shape[0]}x{C}" + ("" if relu else "_norelu"),
                       lambda: ops.relu_bias_grad(g2, o2, db=db_out))
    return gp2, db_out, direct_b


class _ConvX6U8(torch.autograd.Function):
    """The first convolution (+ ReLU) of the update's minibatch forward read straight from the
    rollout's u8 frame stacks through the minibatch indices (ops.conv_x6_u8: NormalizeImg's / 255
    in the epilogue; no f32 minibatch copy of the observations, ppo_atari_oc.py:566); backward:
    relu_bias_grad, then the weight gradient from the same u8 rows (the input needs none).
    Under U8_WGRAD_RELU the forward also leaves the ReLU's bitmask and the backward hands the
    unmasked gradient to the weight-gradient kernel, which applies the ReLU backward and sums the
    bias gradient itself (ops.conv_x6_u8_wgrad mbits / db): no relu_bias_grad pass."""

    @staticmethod
    def forward(ctx, w, b, frames, idx, stride, relu: bool, divisor: float, box=None, wn=None):
        mb = None
        if (U8_WGRAD_RELU and relu and box is None and ctx.needs_input_grad[0] and
                ops._conv_u8_img_ok(frames, w, stride) and
                ops._conv_u8_img_wgrad_ok(frames, tuple(w.shape[2:]), stride, w.shape[0])):
            P = ((frames.shape[2] - w.shape[2]) // stride + 1) * \
                ((frames.shape[3] - w.shape[3]) // stride + 1)
            mb = torch.empty(idx.numel() * P, dtype=torch.int32, device=frames.device)
        y = ops.timed(f"conv_x6_u8_{idx.numel()}",
                      lambda: ops.conv_x6_u8(frames, idx, w, b, stride, relu, divisor, mbits=mb,
                                             wn=wn))
        ctx.conv = (stride, relu, divisor)
        ctx.b = b
        ctx.box = box
        ctx.mb = mb
        ctx.save_for_backward(w, frames, idx, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        w, frames, idx, y = ctx.saved_tensors
        stride, relu, divisor = ctx.conv
        g = g.contiguous(memory_format=torch.channels_last)
        C = g.shape[1]
        g2 = g.permute(0, 2, 3, 1).reshape(-1, C)
        b = ctx.b
        mb, ctx.mb = ctx.mb, None
        if mb is not None and ctx.needs_input_grad[0]:
            # ReLU backward + bias gradient inside the weight-gradient kernel
            direct_b = _direct(b)
            db_out = b.grad if direct_b else torch.empty_like(b)
            KH, KW = w.shape[2], w.shape[3]
            dw = ops.timed(f"conv_x6_u8_wgrad_relu_{C}x{w[0].numel()}",
                           lambda: ops.conv_x6_u8_wgrad(g2, frames, idx, (KH, KW), stride,
                                                        divisor, mbits=mb,
                                                        db=db_out)).view(w.shape)
            if _direct(w):
                w.grad.copy_(dw)
                dw = None
            return dw, (None if direct_b else db_out), None, None, None, None, None, None, None
        gp2, db_out, direct_b = _conv_relu_backward(ctx.box, g2, y, b, relu)
        dw = None
        if ctx.needs_input_grad[0]:
            KH, KW = w.shape[2], w.shape[3]
            dw = ops.timed(f"conv_x6_u8_wgrad_{C}x{w[0].numel()}",
                           lambda: ops.conv_x6_u8_wgrad(gp2, frames, idx, (KH, KW), stride,
                                                        divisor)).view(w.shape)
            if _direct(w):
                w.grad.copy_(dw)  # nn.Conv2d's tap order into the channels_last grad
                dw = None
        return dw, (None if direct_b else db_out), None, None, None, None, None, None, None


# The update's first convolution straight from the u8 frame stacks (_ConvX6U8) when the trunk
# starts [NormalizeImg,] Conv2d: no minibatch gather of f32 observations
CONV_X6_U8 = True

# ... its ReLU backward and bias gradient inside the image-staged weight-gradient kernel (the
# forward's ReLU bitmask, ops.conv_x6_u8 / conv_x6_u8_wgrad mbits): no relu_bias_grad pass over
# the first layer's [B OH OW, 32] gradient (read twice, written once)
U8_WGRAD_RELU = True


# The update's convolution forwards read their weight pre-split into bf16 planes (one
# ocppo_split_planes launch per minibatch for all of them, trainer._weight_planes) instead of
# splitting it in every workgroup
CONV_X6_PLANES = True

# NatureCNN convolutions on this package's implicit GEMMs (ops.conv_x6, x6 products: no MIOpen,
# deterministic by construction), in the rollout forward and the update; shapes it does not take
# (conv_x6_ok: row counts the tiles do not divide, e.g. a few envs) stay on _ConvAct / MIOpen.
CONV_X6 = True


def _conv_x6_ok(x, conv) -> bool:
    if not (CONV_X6 and isinstance(conv, nn.Conv2d) and conv.bias is not None and x.is_cuda
            and conv.groups == 1 and conv.dilation == (1, 1) and conv.padding_mode == "zeros"
            and tuple(conv.padding) == (0, 0) and conv.stride[0] == conv.stride[1]):
        return False
    grad = torch.is_grad_enabled()
    return ops.conv_x6_ok(x, conv.weight, conv.stride[0],
                          wgrad=grad and conv.weight.requires_grad,
                          dgrad=grad and x.requires_grad)


# The data gradient of a convolution whose input is another convolution's ReLU output can take
# that ReLU's backward and bias gradient in its epilogue (ops.conv_x6_dgrad relu_out / db; no
# relu_bias_grad pass over the input gradient). Measured slower at config 3 (805 / 515 us per
# update against 371 + 254 / 373 + 105 us unfused: the masked, column-summing epilogue over the
# stride classes' scattered rows costs more than the streaming pass it removes): off by default
CONV_DGRAD_RELU = False

# The last convolution's ReLU backward and bias gradient in the dX epilogue of the Linear that
# reads its flattened channels_last output (NatureCNN's 3136 -> 512; ops.dx_x6_relu with the
# activation as the mask, the bias gradient from the epilogue's column sums over rows and
# positions in f64): no relu_bias_grad pass over that layer's gradient. Measured slower at config
# 3 (519.4k vs 522.1k env steps/s: the masked, column-summing epilogue of the 128 x 64-tile dX
# costs more than the 59 us streaming pass it removes; profiles/r06/config3/flat_dx/), so off
CONV_RELU_IN_FLAT_DX = False

# The update's convolution forwards (+ ReLU) also write their ReLU mask as a row-major bitmask
# (ops.conv_x6 mbits, the tile loop's epilogue), which the backward's ReLU pass reads instead of
# the f32 output (ops.relu_bias_grad bits=): 4 B -> 1 bit of mask traffic per element
CONV_RELU_BITS = True


def _conv_x6(x, conv, relu: bool):
    s = conv.stride[0]
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad or
                                    conv.bias.requires_grad):
        # the box lets the consumer of this ReLU output take its backward: the next convolution's
        # data gradient (CONV_DGRAD_RELU) or the flattened Linear's dX (CONV_RELU_IN_FLAT_DX)
        box = ({"bias": conv.bias, "premasked": False, "conv": True}
               if relu and (CONV_DGRAD_RELU or CONV_RELU_IN_FLAT_DX) else None)
        y = _ConvX6.apply(x, conv.weight, conv.bias, s, relu, box,
                          getattr(x, "_ocppo_cbox", None))
        if box is not None:
            y._ocppo_cbox = box
        return y
    B, Cin, H, _ = x.shape
    wp = (_planes_infer(conv.weight) if CONV_ROWS_PLANES and _IN_ROLLOUT[0] and
          not torch.is_grad_enabled() else None)
    return ops.timed(f"conv_x6_{B}x{Cin}x{H}_{conv.out_channels}",
                     lambda: ops.conv_x6(x, conv.weight, conv.bias, s, relu, w_planes=wp))


# The rollout's convolutions (ops.conv_x6's few-rows form) reading their weights pre-split into
# the three bf16 pieces once per rollout (ocppo_split_planes) instead of splitting them in every
# workgroup: measured SLOWER in that kernel (conv2 / conv3 at 256 envs 24.8 / 19.3 us against
# 21.2 / 16.1 us: the planes' 6 B per element against 4, read straight from L2 without an LDS
# stage; tools/exp_conv_rows.py, profiles/r06/config3/rows/), so off
CONV_ROWS_PLANES = False
_PLANES_INFER: dict = {}


def _planes_infer(w):
    """bf16 [3, Cout, KH KW C] pieces of a channels_last conv weight's [Cout, KH KW C] matrix,
    refreshed once per rollout (rollout_inference); None when the weight is not channels_last."""
    ent = _PLANES_INFER.get(id(w))
    if ent is None or ent[0] is not w:
        wm = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
        if wm.data_ptr() != w.data_ptr() or not wm.is_contiguous() or wm.shape[1] % 8:
            return None
        wp = ops.WeightPlanes(fwd=(wm,))
        ent = [w, wp, wm._ocppo_planes["fwd"], -1]
        _PLANES_INFER[id(w)] = ent
    if ent[3] != _WEIGHTS_GEN[0]:
        ent[1].refresh()
        ent[3] = _WEIGHTS_GEN[0]
    return ent[2]


def _conv_act_ok(x, conv) -> bool:
    return (FUSED_CONV_ACT and isinstance(conv, nn.Conv2d) and conv.bias is not None and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 4 and conv.groups == 1
            and conv.dilation == (1, 1) and conv.padding_mode == "zeros"
            and isinstance(conv.padding, tuple) and conv.out_channels % 4 == 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and conv.weight.is_contiguous(memory_format=torch.channels_last))


# NHWC conv + one-pass HIP bias/ReLU forward and ReLU-backward/bias-grad backward (_ConvAct).
FUSED_CONV_ACT = True

# Rollout-sized inference batches (no autograd) of the input convolution (Cin <= 4, e.g. the
# NatureCNN's 8x8/4 on the 4-frame stack) on the HIP implicit-GEMM kernel (ops.conv2d_act, bias
# and ReLU fused): 44 vs 60 us at 256 envs for MIOpen's default solution + layout copy +
# bias/ReLU; the deeper layers stay on MIOpen, which is faster there. With MIOpen's Find
# (cudnn.benchmark, Args.conv_benchmark) its conv1 solution is faster (38.5 us), so the kernel
# only stands in for MIOpen's immediate-mode choice (tools/exp_conv_rollout.py).
HIP_ROLLOUT_CONV = True


def _hip_conv_ok(x, conv) -> bool:
    return (HIP_ROLLOUT_CONV and not torch.is_grad_enabled() and
            not torch.backends.cudnn.benchmark and _conv_act_ok(x, conv) and
            conv.in_channels <= 4 and conv.in_channels & (conv.in_channels - 1) == 0 and
            conv.padding == (0, 0) and conv.stride[0] == conv.stride[1] and x.shape[0] <= 1024
            and (conv.kernel_size[0] * conv.kernel_size[1] * conv.in_channels) % 16 == 0)


# Rollout-sized inference batches (no autograd) of the shapes where the HIP f32-MFMA kernel beats
# the BLAS library's (tools/exp_rollout_linear.py on MI355X: K <= 256 at up to 512 rows; at up to
# 128 rows every K <= 2048 with K % 16 == 0 -- the LDS-staged form: 4.7 vs 6.1 us at 512 -> 1024,
# 4.7 vs 5.6 at 1024 -> 512, 6.8 vs 7.0 at 2048 -> 512); everything else, and every autograd
# forward, stays on hipBLASLt.
HIP_ROLLOUT_LINEAR = True


def _hip_linear_ok(x2, lin: nn.Linear) -> bool:
    if not HIP_ROLLOUT_LINEAR or torch.is_grad_enabled() or not x2.is_cuda or \
            x2.dtype != torch.float32 or (x2.shape[0] > 1 and x2.stride(1) != 1):
        return False
    M, K = x2.shape
    # M <= 8 (single-env acting, e.g. the DQN learner's epsilon-greedy forward): the library
    # takes a copy-bias + GEMV + separate ReLU path there (3 launches)
    return ((K <= 256 and M <= 512 and K % 16 == 0) or (K <= 64 and M <= 512) or
            (M <= 128 and (K <= 256 or (K <= 2048 and K % 16 == 0))) or M <= 8)


def linear_act(x, lin: nn.Linear, relu: bool, chw=None, rows: bool = False, below=None):
    """rows: the output's consumer walks it by rows (the frame scatter, frames.SCATTER_MBITS):
    its ReLU bitmask, if the forward writes one, in the row-major layout."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    if chw is None and _hip_linear_ok(x2, lin):
        y = ops.linear_act(x2, lin.weight, lin.bias, relu)
        return y.view(*lead, y.shape[-1])
    box = None
    if relu and FUSED_HEADS_BWD and torch.is_grad_enabled() and _direct(lin.weight) and \
            _direct(lin.bias):
        box = {"premasked": False, "bias": lin.bias, "rows": rows}
    y = _LinearAct.apply(x2, lin.weight, lin.bias, relu, box, chw,
                         below if below is not None else getattr(x, "_ocppo_box", None),
                         getattr(x, "_ocppo_wslot", None))
    y = y.view(*lead, y.shape[-1])
    if box is not None:
        y._ocppo_box = box
    return y


# Inference (the rollout): the last convolution's bias + ReLU pass writes its output in NCHW order
# (ops.bias_act_nchw) when an nn.Flatten follows, instead of the in-place NHWC pass and the
# Flatten's layout copy (3.2 MB per step at 256 envs).
CONV_NCHW_OUT = True


def _conv_nchw_out_ok(x, conv, nxt) -> bool:
    if not (CONV_NCHW_OUT and not torch.is_grad_enabled() and len(nxt) == 2 and
            isinstance(nxt[0], nn.ReLU) and isinstance(nxt[1], nn.Flatten) and
            nxt[1].start_dim == 1 and _conv_act_ok(x, conv) and x.shape[0] > 0):
        return False
    kh, kw = conv.kernel_size
    (sh, sw), (ph, pw) = conv.stride, conv.padding
    oh = (x.shape[2] + 2 * ph - kh) // sh + 1
    ow = (x.shape[3] + 2 * pw - kw) // sw + 1
    return oh * ow * (conv.out_channels + 1) <= 12288


# nn.Flatten -> nn.Linear on a channels_last activation under autograd (the NatureCNN's
# 3136 -> 512 layer in the update): the Linear reads the activation in its memory order with the
# weight's columns permuted to match (a 6.4 MB copy) instead of nn.Flatten's NCHW-order copy of the
# activation and the channels_last copy of its gradient (2 x 103 MB per minibatch of 8192).
FLAT_NHWC_LINEAR = True


def _flat_nhwc_ok(x, flat, lin) -> bool:
    return (FLAT_NHWC_LINEAR and torch.is_grad_enabled() and isinstance(flat, nn.Flatten)
            and isinstance(lin, nn.Linear) and lin.bias is not None and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 4 and flat.start_dim == 1
            and flat.end_dim in (-1, 3) and x.is_contiguous(memory_format=torch.channels_last)
            and not x.is_contiguous() and lin.in_features == x[0].numel())


def linear_act_nhwc(x, lin: nn.Linear, relu: bool):
    """act(lin(flatten(x))) for a channels_last x [B, C, H, W], without materialising the
    NCHW-order flatten: same products and sums as the reference layer, columns visited in (H, W,
    C) order (the f32 GEMM's summation order over K differs accordingly)."""
    B, C, H, W = x.shape
    below = getattr(x, "_ocppo_cbox", None) if CONV_RELU_IN_FLAT_DX else None
    return linear_act(x.permute(0, 2, 3, 1).reshape(B, H * W * C), lin, relu, (C, H, W),
                      below=below)


# Inference (the rollout) through nn.Flatten -> nn.Linear on a channels_last activation (the
# NatureCNN's last convolution at 256 envs): the Linear reads the activation in its memory order
# with the weight's columns permuted to match, instead of nn.Flatten's NCHW-order copy of the
# activation every step (3.2 MB, one ~6 us launch per step). The permuted weight is made once per
# rollout, inside rollout_inference() only (the trainer's rollout: the parameters cannot change
# within it; entering it marks the cache stale, and the copy rides in the first step, captured
# with the rollout graph), and reused by the other steps.
FLAT_NHWC_INFER = True
_NHWC_INFER: dict = {}
_WEIGHTS_GEN = [0]
_IN_ROLLOUT = [False]


class rollout_inference:
    """Context of one rollout (trainer._rollout): the parameters are fixed inside it, so the
    inference caches (linear_act_nhwc_infer's permuted weight) are valid; refreshed on entry."""

    def __enter__(self):
        _WEIGHTS_GEN[0] += 1
        _IN_ROLLOUT[0] = True

    def __exit__(self, *exc):
        _IN_ROLLOUT[0] = False


def _flat_nhwc_infer_ok(x, flat, lin) -> bool:
    return (FLAT_NHWC_INFER and _IN_ROLLOUT[0] and not torch.is_grad_enabled()
            and isinstance(flat, nn.Flatten)
            and isinstance(lin, nn.Linear) and lin.bias is not None and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 4 and flat.start_dim == 1
            and flat.end_dim in (-1, 3) and x.is_contiguous(memory_format=torch.channels_last)
            and not x.is_contiguous() and lin.in_features == x[0].numel())


_CONTIG_INFER: dict = {}


def _contig_infer(w):
    """A contiguous copy of parameter w, refreshed once per rollout (rollout_inference)."""
    ent = _CONTIG_INFER.get(id(w))
    if ent is None or ent[0] is not w:
        ent = [w, torch.empty(w.shape, dtype=w.dtype, device=w.device), -1]
        _CONTIG_INFER[id(w)] = ent
    if ent[2] != _WEIGHTS_GEN[0]:
        ent[1].copy_(w)
        ent[2] = _WEIGHTS_GEN[0]
    return ent[1]


def linear_act_nhwc_infer(x, lin: nn.Linear, relu: bool):
    """act(lin(flatten(x))) without autograd for a channels_last x, reading x in its memory order
    against a cached column-permuted weight (same products, columns visited in (H, W, C) order)."""
    B, C, H, W = x.shape
    key = id(lin)
    ent = _NHWC_INFER.get(key)
    if ent is None or ent[0] is not lin.weight:
        ent = [lin.weight, torch.empty_like(lin.weight), -1]
        _NHWC_INFER[key] = ent
    if ent[2] != _WEIGHTS_GEN[0]:
        ent[1].copy_(_cols_to_nhwc(lin.weight, (C, H, W)))
        ent[2] = _WEIGHTS_GEN[0]
    x2 = x.permute(0, 2, 3, 1).reshape(B, H * W * C)
    if HIP_FLAT_INFER:
        return ops.timed(f"linear_act_{B}x{lin.out_features}x{H * W * C}",
                         lambda: ops.linear_act(x2, ent[1], lin.bias, relu))
    if relu:
        return torch._addmm_activation(lin.bias, x2, ent[1].t(), use_gelu=False)
    return torch.addmm(lin.bias, x2, ent[1].t())


# ... on the HIP f32-MFMA rows kernel (ops.linear_act: 16 x 16 output tiles, K split over 8 waves,
# bias + ReLU fused) instead of hipBLASLt's f32 GEMM + epilogue: measured slower at 256 x 3136 ->
# 512 (17.3 vs 15.0 us, config 3 474.3k vs 476.2k env steps/s, profiles/r06/config3/SUMMARY.txt)
HIP_FLAT_INFER = False


def linear_relu(x, lin: nn.Linear, rows: bool = False):
    return linear_act(x, lin, True, rows=rows)


# The first two Linear->ReLU layers of a rollout-sized inference batch as ONE HIP launch
# (ops.linear2_act): the first layer's K <= 64 makes recomputing its rows per output tile free.
HIP_ROLLOUT_LINEAR2 = True


def _pair_ok(x, l1: nn.Linear, l2: nn.Linear) -> bool:
    if not (HIP_ROLLOUT_LINEAR2 and HIP_ROLLOUT_LINEAR) or torch.is_grad_enabled() or \
            not x.is_cuda or x.dtype != torch.float32 or l1.bias is None or l2.bias is None:
        return False
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N1 = l1.out_features
    return (M <= 256 and K <= 64 and N1 % 16 == 0 and N1 <= 512 and
            (M == 1 or x2.stride(1) == 1) and l2.weight.data_ptr() % 16 == 0)


def linear2_relu(x, l1: nn.Linear, l2: nn.Linear):
    lead = x.shape[:-1]
    y = ops.linear2_act(x.reshape(-1, x.shape[-1]), l1.weight, l1.bias, l2.weight, l2.bias)
    return y.view(*lead, y.shape[-1])


def fused_trunk(seq: nn.Sequential, x, rows_last: bool = False):
    """Run `seq` with every Linear→ReLU pair as one fused GEMM (same math, fewer launches) and
    every other biased Linear through the same path (so FlatAdam-owned grads are written in place,
    never accumulated). Used on GPU tensors; module structure and state-dict keys are untouched.
    rows_last: the last Linear→ReLU's output goes to the frame scatter (its bitmask row-major)."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        fusable = (isinstance(m, nn.Linear) and m.bias is not None and x.is_cuda
                   and x.dtype == torch.float32)
        if (isinstance(m, nn.Linear) and i + 3 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                and isinstance(mods[i + 2], nn.Linear) and isinstance(mods[i + 3], nn.ReLU)
                and _pair_ok(x, m, mods[i + 2])):
            x = linear2_relu(x, m, mods[i + 2])
            i += 4
        elif _conv_x6_ok(x, m):
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            x = _conv_x6(x, m, relu)
            i += 2 if relu else 1
        elif _hip_conv_ok(x, m):
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            x = ops.conv2d_act(x, m.weight, m.bias, m.stride[0], relu)
            i += 2 if relu else 1
        elif _conv_nchw_out_ok(x, m, mods[i + 1:i + 3]):
            # inference: the bias/ReLU pass writes NCHW, so the nn.Flatten after it is a view
            y = torch.ops.aten.convolution(x, m.weight, None, m.stride, m.padding, (1, 1), False,
                                           (0, 0), 1).contiguous(memory_format=torch.channels_last)
            x = ops.timed("bias_act_nchw",
                          lambda y=y, b=m.bias: ops.bias_act_nchw(y, b, True))  # bound now
            i += 2
        elif _conv_act_ok(x, m):
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            x = _ConvAct.apply(x, m.weight, m.bias, m.stride, m.padding, relu)
            i += 2 if relu else 1
        elif i + 1 < len(mods) and _flat_nhwc_ok(x, m, mods[i + 1]):
            relu = i + 2 < len(mods) and isinstance(mods[i + 2], nn.ReLU)
            x = linear_act_nhwc(x, mods[i + 1], relu)
            i += 3 if relu else 2
        elif i + 1 < len(mods) and _flat_nhwc_infer_ok(x, m, mods[i + 1]):
            relu = i + 2 < len(mods) and isinstance(mods[i + 2], nn.ReLU)
            x = linear_act_nhwc_infer(x, mods[i + 1], relu)
            i += 3 if relu else 2
        elif fusable and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU):
            x = linear_relu(x, m, rows=rows_last and i + 2 == len(mods))
            i += 2
        elif fusable:
            x = linear_act(x, m, False)
            i += 1
        else:
            x = m(x)
            i += 1
    return x


class _ActorCritic(Predictor):
    """Shared interface: network → (actor logits, critic value)."""

    def trunk(self, x, prescaled: bool = False):
        """Shared network output. prescaled: x already holds obs / 255 (the HIP store / gather
        fold NormalizeImg in, bit-identical to it), so a leading NormalizeImg is skipped."""
        net = self.network
        if not isinstance(net, nn.Sequential):
            return net(x)
        if prescaled and len(net) and isinstance(net[0], NormalizeImg):
            net = net[1:]
        return fused_trunk(net, x)

    def trunk_frames_ok(self, frames, B: int) -> bool:
        """trunk_frames applies: a Sequential trunk [NormalizeImg,] Conv2d(+ReLU) ... on the GPU
        whose first convolution ops.conv_x6_u8 takes for B samples of `frames`."""
        net = self.network
        if not (CONV_X6_U8 and CONV_X6 and isinstance(net, nn.Sequential) and len(net) > 2):
            return False
        i = 1 if isinstance(net[0], NormalizeImg) else 0
        conv = net[i]
        return (isinstance(conv, nn.Conv2d) and conv.bias is not None and conv.groups == 1 and
                conv.dilation == (1, 1) and tuple(conv.padding) == (0, 0) and
                conv.stride[0] == conv.stride[1] and conv.weight.is_cuda and
                ops.conv_x6_u8_ok(frames, conv.weight, conv.stride[0], B,
                                  wgrad=conv.weight.requires_grad))

    def trunk_frames(self, frames, idx):
        """trunk(frames[idx]) for u8 frame stacks (NormalizeImg folded into the first
        convolution's epilogue), the first Conv2d(+ReLU) reading the u8 rows in place."""
        net = self.network
        div = 255.0 if isinstance(net[0], NormalizeImg) else 1.0
        if isinstance(net[0], NormalizeImg):
            net = net[1:]
        conv = net[0]
        relu = isinstance(net[1], nn.ReLU)
        box = {"bias": conv.bias} if relu and CONV_DGRAD_RELU else None
        # the rollout (weights fixed): the weight's tap-order copy made once per rollout
        wn = (_contig_infer(conv.weight) if _IN_ROLLOUT[0] and not torch.is_grad_enabled()
              and not conv.weight.is_contiguous() else None)
        y = _ConvX6U8.apply(conv.weight, conv.bias, frames, idx, conv.stride[0], relu, div, box,
                            wn)
        if box is not None:
            y._ocppo_cbox = box
        return fused_trunk(net[2 if relu else 1:], y)

    def _head(self, lin, h):
        if isinstance(lin, nn.Linear) and lin.bias is not None and h.is_cuda and \
                h.dtype == torch.float32:
            return linear_act(h, lin, False)
        return lin(h)

    def get_value(self, x, prescaled: bool = False):
        return self._head(self.critic, self.trunk(x, prescaled))

    def heads(self, hidden):
        """(actor logits, critic value) from the trunk output; under autograd on the GPU one
        _Heads function (fused HIP backward), else the two head Linears. With the fused path
        the trunk layer that produced `hidden` leaves its ReLU mask and bias gradient to _Heads,
        so `hidden` must feed nothing but these two heads in the graph being differentiated
        (true for the PPO loss of ppo_atari_oc.py:566-605; set FUSED_HEADS_BWD = False for
        extra losses on the trunk output)."""
        if heads_ok(hidden, self.actor, self.critic):
            box = getattr(hidden, "_ocppo_box", None)
            return _Heads.apply(hidden, self.actor.weight, self.actor.bias, self.critic.weight,
                                self.critic.bias, box)
        return self._head(self.actor, hidden), self._head(self.critic, hidden)

    def logits_and_value(self, x, prescaled: bool = False):
        return self.heads(self.trunk(x, prescaled))

    def get_action_and_value(self, x, action=None):
        """(action [B] i64, log_prob [B], entropy [B], value [B, 1]) like the reference."""
        logits, value = self.logits_and_value(x)
        if action is None:
            noise = torch.empty_like(logits, dtype=torch.float32).exponential_()
            ent = torch.empty(logits.shape[0], dtype=torch.float32, device=logits.device)
            act, lp, _ = ops.categorical_sample(logits.detach().float().contiguous(), noise,
                                                entropy_out=ent)
            if torch.is_grad_enabled() and logits.requires_grad:
                lp, ent = ops.categorical_logprob_entropy(logits.float(), act)
            return act, lp, ent, value
        lp, ent = ops.categorical_logprob_entropy(logits.float(), action)
        return action, lp, ent, value


class PPODefault(_ActorCritic):
    """NatureCNN agent (architectures/ppo.py:15-57)."""

    def __init__(self, envs, device=None, normalize=True):
        super().__init__()
        self.device = device
        dims = tuple(envs.observation_space.shape)
        self.network = nn.Sequential(
            layer_init(nn.Conv2d(dims[0], 32, 8, stride=4)),
            nn.ReLU(),
            layer_init(nn.Conv2d(32, 64, 4, stride=2)),
            nn.ReLU(),
            layer_init(nn.Conv2d(64, 64, 3, stride=1)),
            nn.ReLU(),
        )
        if normalize:
            self.network.insert(0, NormalizeImg())
        self.network.append(nn.Flatten())
        with torch.no_grad():
            feat_dim = self.network(torch.zeros((1,) + dims)).flatten().shape[0]
        self.network.append(layer_init(nn.Linear(feat_dim, 512)))
        self.network.append(nn.ReLU())
        self.actor = layer_init(nn.Linear(512, envs.action_space.n), std=0.01)
        self.critic = layer_init(nn.Linear(512, 1), std=1)


class PPObj(_ActorCritic):
    """Object-centric MLP agent (architectures/ppo.py:60-95): a per-frame Linear encoder on the
    last (feature) dim, Flatten over the frame stack, a Linear decoder, actor and critic heads."""

    def __init__(self, envs, device=None, encoder_dims=(128, 64), decoder_dims=(32,)):
        super().__init__()
        self.device = device
        dims = tuple(envs.observation_space.shape)
        layers = nn.ModuleList()
        in_dim = dims[-1]
        for l in encoder_dims:
            layers.append(layer_init(nn.Linear(in_dim, l)))
            layers.append(nn.ReLU())
            in_dim = l
        layers.append(nn.Flatten())
        in_dim *= int(np.prod(dims[:-1], dtype=int))
        l = in_dim
        for l in decoder_dims:
            layers.append(layer_init(nn.Linear(in_dim, l)))
            layers.append(nn.ReLU())
            in_dim = l
        self.network = nn.Sequential(*layers)
        self.actor = layer_init(nn.Linear(l, envs.action_space.n), std=0.01)
        self.critic = layer_init(nn.Linear(l, 1), std=1)
        self._flat = len(encoder_dims) * 2  # index of the Flatten in self.network

    # The encoder acts on each stacked frame alone (Linear on the last dim), so the rollout can
    # encode only the newest frame per step and keep the rest in a cache (ops.frame_cache_shift).
    @property
    def encoding_dim(self) -> int:
        return self.network[self._flat - 2].out_features

    def encode(self, x):
        """Per-frame encoder output: [..., F] -> [..., E]."""
        return fused_trunk(self.network[:self._flat], x)

    def decode(self, enc):
        """Flatten + decoder on the stacked frame encodings [B, W, E] -> hidden [B, H];
        decode(encode(x)) == trunk(x)."""
        return fused_trunk(self.network[self._flat:], enc)


class CartPoleAgent(_ActorCritic):
    """The tanh-MLP agent of cleanrl/ppo.py:100-126 (config 1), separate actor/critic trunks.

    Exposed through the same logits_and_value interface; `network` is the identity so the
    actor/critic Sequentials see the raw observation, as in the reference.
    """

    def __init__(self, envs, device=None):
        super().__init__()
        self.device = device
        n = int(np.array(envs.observation_space.shape).prod())
        self.critic = nn.Sequential(
            layer_init(nn.Linear(n, 64)), nn.Tanh(), layer_init(nn.Linear(64, 64)), nn.Tanh(),
            layer_init(nn.Linear(64, 1), std=1.0))
        self.actor = nn.Sequential(
            layer_init(nn.Linear(n, 64)), nn.Tanh(), layer_init(nn.Linear(64, 64)), nn.Tanh(),
            layer_init(nn.Linear(64, envs.action_space.n), std=0.01))
        self.network = nn.Identity()

    def trunk(self, x, prescaled: bool = False):
        """The raw observation, flattened per sample ([B, 4] from the rollout's [B, 1, 4])."""
        return x.reshape(x.shape[0], -1)


class Space:
    """Minimal gym-like space (shape / n) for constructing agents without gymnasium."""

    def __init__(self, shape=(), n=None):
        self.shape = tuple(shape)
        self.n = n


class EnvSpec:
    """`envs`-like object exposing observation_space / action_space (what the agents read)."""

    def __init__(self, obs_shape, n_actions):
        self.observation_space = Space(obs_shape)
        self.action_space = Space((), n_actions)
        self.single_observation_space = self.observation_space
        self.single_action_space = self.action_space


def make_agent(architecture: str, obs_shape, n_actions, device=None, encoder_dims=(256, 512, 1024, 512),
               decoder_dims=(512,)):
    """Architecture switch of ppo_atari_oc.py:435-440 for the supported agents."""
    spec = EnvSpec(obs_shape, n_actions)
    if architecture == "PPO_OBJ":
        return PPObj(spec, device, tuple(encoder_dims), tuple(decoder_dims))
    if architecture == "PPO":
        return PPODefault(spec, device)
    if architecture == "CARTPOLE_MLP":
        return CartPoleAgent(spec, device)
    raise NotImplementedError(f"Architecture {architecture} is not supported by oc_cleanrl_amd "
                              "(supported: PPO_OBJ, PPO, CARTPOLE_MLP)")
