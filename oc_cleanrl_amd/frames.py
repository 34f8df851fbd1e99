"""Frame-deduplicated PPObj minibatch forward/backward (obs_mode "obj", PPO_OBJ agent).

The update of ppo_atari_oc.py:566 runs `agent.get_action_and_value(b_obs[mb_inds], ...)`, and
PPObj's encoder (architectures/ppo.py:60-84) is a Linear stack on the last dim, i.e. on every
stacked frame alone. The W frames of a stored observation obs[t, n] are frames of env n's own
timeline (slot k = the frame of step t-(W-1)+k, clipped to the latest reset), so a minibatch of M
samples holds only ~0.69·M·W distinct frames when it is a random quarter of the batch (W = 4).

Per minibatch the trainer therefore
  1. gathers the C distinct frames once                    (HIP `ocppo_frames_gather`),
  2. runs the encoder on C rows instead of M·W             (hipBLASLt, autograd),
  3. expands the C encodings to the [M, W, E] decoder input (HIP `ocppo_frames_expand`),
and in the backward pass sums each frame's slot gradients back onto its row
(HIP `ocppo_frames_scatter`, fixed order, deterministic). The rows are the same frames, so the
forward is identical to encoding every slot; only the f32 summation order of the encoder's
weight gradients differs (the uses of one frame are summed first).

The plan (which frames each minibatch needs) depends only on the epoch permutations, so it is
built on the host from the shuffle (`FramePlanner`), as a superset that ignores resets (a reset
only maps a slot onto a later frame of the same window, which is in the set already), and copied
to the device with the permutation; every minibatch gets the same fixed capacity `cap` (padding
ids -1 encode to rows whose gradient is exactly zero), so the update stays graph-capturable.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


class FramePlanner:
    """Host-side plan of the distinct frames of every minibatch of an iteration.

    Layout of one plan (int32, one contiguous pinned buffer so it is ONE H2D copy):
      uniq  [J, cap]           timeline ids of the distinct frames of minibatch j, ascending,
                               padded with -1 (J = epochs x minibatches)
      pos_of[J, (T+W-1)*N]     row of each timeline id in minibatch j's encoding
      inv   [E, T*N]           position of each sample in epoch e's permutation
    Timeline id of env n's frame of step s (s in [-(W-1), T-1]): u = (s + W - 1) * N + n.
    """

    def __init__(self, T: int, N: int, W: int, M: int, epochs: int, num_minibatches: int,
                 cap: int | None = None, margin: int = 64, align: int = 2048,
                 extra_caps: tuple = (11520,)):
        self.T, self.N, self.W, self.M = T, N, W, M
        self.E, self.nmb = epochs, num_minibatches
        self.J = epochs * num_minibatches
        self.B = T * N
        self.U = (T + W - 1) * N
        self.margin, self.align, self.extra_caps = margin, align, tuple(extra_caps)
        self.cap = cap
        self.counts = np.zeros(self.J, np.int64)

    def size(self, cap: int) -> int:
        return self.J * cap + self.J * self.U + self.E * self.B

    def views(self, buf, cap: int):
        """(uniq [J, cap], pos_of [J, U], inv [E, B]) views of a flat int32 buffer."""
        J, U = self.J, self.U
        uniq = buf[:J * cap].reshape(J, cap)
        pos_of = buf[J * cap:J * cap + J * U].reshape(J, U)
        inv = buf[J * cap + J * U:self.size(cap)].reshape(self.E, self.B)
        return uniq, pos_of, inv

    def cap_for(self, counts) -> int:
        """Capacity for the largest minibatch + `margin` rows: the smallest multiple of `align`
        or entry of `extra_caps` that holds it. hipBLASLt's f32 tiles quantise the encoder's
        fwd+bwd time in rows on gfx950 (tools/exp_dedup_rows.py, encoder 12->256->512->1024->512:
        10240 / 11264 / 11520 / 11776 / 12032 / 12288 rows -> 710 / 837 / 781 / 905 / 906 / 800 us),
        so between the multiples of 2048 only 11520 pays. At config 2 the largest of an
        iteration's 16 minibatches is 11357 +- 40 distinct frames (max 11470 over 300 iterations),
        so 11520 holds it; a later overflow re-sizes the plan (trainer._alloc_plan)."""
        need = int(counts.max()) + self.margin
        cands = sorted({c for c in self.extra_caps if c >= need} |
                       {-(-need // self.align) * self.align})
        return min(max(cands[0], self.align), self.M * self.W)

    def plan(self, perm: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """perm [E*B] (the epochs' shuffles, ppo_atari_oc.py:561) -> (used [J, U] bool,
        inv [E, B] int32); sets self.counts (distinct frames per minibatch).

        Frame (s, n) is used by minibatch k of epoch e iff one of the samples t in
        [s, s+W-1] of env n is in it: with mb[t, n] = inv_e[t*N + n] // M that is an OR of W
        shifted copies of (mb == k) along t -- a few [T+W-1, N] array passes per minibatch."""
        T, N, W, M, J, U, B = self.T, self.N, self.W, self.M, self.J, self.U, self.B
        inv = np.empty((self.E, B), np.int32)
        ar = np.arange(B, dtype=np.int32)
        used = np.zeros((J, T + W - 1, N), bool)
        for e in range(self.E):
            inv[e, perm[e * B:(e + 1) * B]] = ar
            mb = (inv[e] // M).reshape(T, N)
            for k in range(self.nmb):
                eq = mb == k
                u = used[e * self.nmb + k]
                for i in range(W):  # frame row s' = s + W - 1 is used by sample t = s' - i
                    u[i:i + T] |= eq
        used = used.reshape(J, U)
        self.counts = np.count_nonzero(used, axis=1)
        return used, inv

    def fill(self, buf: np.ndarray, cap: int, used, inv) -> None:
        """Write a plan into the flat int32 buffer laid out for capacity `cap`."""
        uniq, po, iv = self.views(buf, cap)
        uniq.fill(-1)
        for j in range(self.J):
            nz = np.flatnonzero(used[j])
            uniq[j, :len(nz)] = nz
        np.cumsum(used, axis=1, dtype=np.int32, out=po)
        po -= 1  # row of a used id; unused ids are never looked up
        iv[...] = inv


# The encoder's last ReLU backward (and its bias-gradient partials) inside the frame scatter
# (ops.frames_scatter_relu) when enc is the ReLU output of an in-place-grad Linear (its box).
FUSED_SCATTER_RELU = True
# ... reading that layer's ReLU mask as the row-major bitmask its forward GEMM wrote
# (ops.linear_x6(..., mbits="rows")): 1 bit instead of the 4-B output element per (frame, column)
SCATTER_MBITS = True


def _rows_bits(box):
    """The row-major ReLU bitmask in an encoder box, else None (the scatter reads the output)."""
    mb = box.get("mbits") if box is not None else None
    return mb[0] if mb is not None and mb[1] == "rows" else None


class _FramesExpand(torch.autograd.Function):
    """h [M, W, E] = enc[pos_of[slot frame ids]]; backward = deterministic per-frame slot sum.
    When enc carries the producing _LinearAct's box (agents.linear_act: ReLU output, grads in
    place), the backward also applies that layer's ReLU mask and leaves its bias-gradient
    partials in the box: the layer's own backward then runs only dX / dW (single consumer: enc
    feeds nothing but this expand)."""

    @staticmethod
    def forward(ctx, enc, pos_of, perm, dones, uniq, inv, mb, T, N, W, box=None):
        fuse = (FUSED_SCATTER_RELU and box is not None and not box["premasked"] and
                enc.shape[-1] % 4 == 0)
        if fuse:
            box["premasked"] = True
            ctx.save_for_backward(uniq, inv, dones, enc)
        else:
            ctx.save_for_backward(uniq, inv, dones)
        ctx.box = box if fuse else None
        ctx.geom = (int(mb), T, N, W, perm.numel())
        return ops.timed("frames_expand", lambda: ops.frames_expand(enc, pos_of, perm, dones,
                                                                    T, N, W))

    @staticmethod
    def backward(ctx, dh):
        mb, T, N, W, M = ctx.geom
        dh = dh.contiguous().view(M, W, -1)
        if ctx.box is not None:
            uniq, inv, dones, enc = ctx.saved_tensors
            box = ctx.box
            gp, part = ops.timed("frames_scatter_relu", lambda: ops.frames_scatter_relu(
                dh, uniq, inv, mb, dones, T, N, W, out=enc, mbits=_rows_bits(box)))
            box["dbp"] = part
            return gp, None, None, None, None, None, None, None, None, None, None
        uniq, inv, dones = ctx.saved_tensors
        denc = ops.timed("frames_scatter", lambda: ops.frames_scatter(dh, uniq, inv, mb, dones,
                                                                      T, N, W))
        return denc, None, None, None, None, None, None, None, None, None, None


# The decoder's Linear+ReLU reading its input rows straight from the distinct-frame encodings
# (frames_expand never materialised): forward and weight gradient gather the rows through an
# [M, W] row table (ocppo_gemm_x6_gather), dX goes to the frame scatter as before.
FUSED_DECODE_GATHER = True
# ... its dX reading the weight's pre-split planes. Off: once the planes were really read
# (round 5: the backward reads them from ctx, not from the forward thread's scope) they measured
# slower than the in-kernel split at config 2 (979.0 / 962.8k vs 986.0 / 982.7k env steps/s,
# tools/ab_toggle.py, profiles/r05/ab_decoder_dx_planes.txt), so the trainer does not build them
DECODE_DX_PLANES = False


class _DecodeFrames(torch.autograd.Function):
    """hidden = relu(expand(enc) Wd^T + bd) (architectures/ppo.py:77-80 on the Flatten of the
    stacked frame encodings) without the [M, W * E] copy: idx = frames_expand_index(...) holds
    each (sample, slot)'s source row; the forward is W K-splits of gemm_x6 whose A rows are
    gathered through idx (split k = stack slot k) + the combine with bias / ReLU
    (ocppo_sum_splits_act); backward: dX = g' Wd on gemm_x6 -> the frame scatter (with the last
    encoder layer's ReLU backward when enc carries its box, as _FramesExpand), dW = g'^T
    expand(enc) with the rows gathered again (mode 2) + the split-K combine, which also runs the
    heads-loss finish when one is pending. g' = the grad masked by the fused heads (box
    premasked, bias grad already written) or masked here."""

    @staticmethod
    def forward(ctx, enc, w, b, pos_of, perm, dones, uniq, inv, mb, T, N, W, enc_box, box,
                idx=None):
        from . import agents

        E = enc.shape[1]
        if idx is None:  # else made by the frame gather's launch (_GatherLinear1's index)
            idx = ops.timed("frames_expand_index",
                            lambda: ops.frames_expand_index(pos_of, perm, dones, T, N, W))
        out = ops.linear_x6_split(enc, w, b, True, W, planes=agents._planes(w, "fwd"),
                                  gather=(idx, E))
        fuse = (FUSED_SCATTER_RELU and enc_box is not None and not enc_box["premasked"] and
                E % 4 == 0)
        if fuse:
            enc_box["premasked"] = True
        ctx.save_for_backward(enc, idx, uniq, inv, dones, out)
        ctx.params, ctx.box, ctx.enc_box = (w, b), box, (enc_box if fuse else None)
        # the dX planes are read here: the weight_planes() scope is the forward thread's, and
        # autograd runs this node's backward on its device thread
        ctx.pdx = agents._planes(w, "dx") if DECODE_DX_PLANES else None
        ctx.geom = (int(mb), T, N, W, perm.numel())
        return out

    @staticmethod
    def backward(ctx, g):
        from . import agents

        enc, idx, uniq, inv, dones, out = ctx.saved_tensors
        w, b = ctx.params
        box = ctx.box
        mb, T, N, W, M = ctx.geom
        g = g.contiguous()
        if box["premasked"]:
            gp = g
        else:
            gp = torch.ops.aten.threshold_backward(g, out, 0)
            torch.sum(gp, 0, out=b.grad)
        dh = agents._dx(gp, w, True, ctx.pdx).view(M, W, -1)
        if ctx.enc_box is not None:
            denc, part = ops.timed("frames_scatter_relu", lambda: ops.frames_scatter_relu(
                dh, uniq, inv, mb, dones, T, N, W, out=enc, mbits=_rows_bits(ctx.enc_box)))
            ctx.enc_box["dbp"] = part
        else:
            denc = ops.timed("frames_scatter", lambda: ops.frames_scatter(dh, uniq, inv, mb, dones,
                                                                          T, N, W))
        S = agents._x6_splits(M, w.shape[0], w.shape[1])[0]
        wpart = ops.dw_x6_parts_gather(gp, enc, idx, S)
        fin = box.get("finish")
        if fin is not None and fin.pending:
            ops.timed(f"sum_splits_fin_{S}x{w.shape[0]}x{w.shape[1]}",
                      lambda: ops.sum_splits(wpart, w.grad, finish=fin))
            fin.run()  # no-op: the combine took it
        else:
            ops.timed(f"sum_splits_{S}x{w.shape[0]}x{w.shape[1]}",
                      lambda: ops.sum_splits(wpart, w.grad))
        return (denc,) + (None,) * 14


def _decode_gather_ok(agent, enc, M: int, W: int) -> bool:
    """The decoder is one Linear+ReLU on the Flatten of the W frame encodings, with FlatAdam-owned
    grads on the gemm_x6 route, at shapes ocppo_gemm_x6_gather takes (128 x 128 tiles; one split
    per stack slot; <= 1024 rows per weight-gradient split)."""
    from . import agents

    net = agent.network
    flat = getattr(agent, "_flat", None)
    if not (FUSED_DECODE_GATHER and agents.X6_FWD_SPLITK and flat is not None and
            torch.is_grad_enabled() and enc.is_cuda and enc.dtype == torch.float32 and
            len(net) == flat + 3 and isinstance(net[flat], torch.nn.Flatten) and
            isinstance(net[flat + 1], torch.nn.Linear) and isinstance(net[flat + 2], torch.nn.ReLU)):
        return False
    lin = net[flat + 1]
    C, E = enc.shape
    H = lin.out_features
    return (lin.bias is not None and lin.in_features == W * E and agents.x6_route(lin.weight)
            and agents._direct(lin.weight) and agents._direct(lin.bias)
            and lin.weight.is_contiguous() and lin.weight.data_ptr() % 16 == 0
            and lin.bias.data_ptr() % 16 == 0 and enc.is_contiguous() and enc.data_ptr() % 16 == 0
            and decode_gather_shape_ok(M, H, E, W))


# K-split counts ocppo_sum_splits_act combines (the gathered forward runs one split per slot)
DECODE_SPLITS = (1, 2, 4, 8, 16)


def decode_gather_shape_ok(M: int, H: int, E: int, W: int) -> bool:
    """The shape part of _decode_gather_ok: the forward's W K-splits (one per stack slot) must be a
    split count the combine takes, the tiles 128 x 128, the weight gradient's splits even over
    32-row steps with <= 1024 rows each."""
    from . import agents

    if W not in DECODE_SPLITS or M % 128 or H % 128 or E % 128 or (M // 32) % W:
        return False
    st = agents._x6_splits(M, H, W * E)
    return (st is not None and st[1] == ops.X6_AUTO and (M // 32) % st[0] == 0
            and M // st[0] <= 1024 and W * (M // 128) * (H // 128) >= 256)


def _decode_frames(agent, enc, pos_of, perm, dones, uniq, inv, mb, T, N, W, idx=None):
    lin = agent.network[agent._flat + 1]
    box = {"premasked": False, "bias": lin.bias}
    hidden = _DecodeFrames.apply(enc, lin.weight, lin.bias, pos_of, perm, dones, uniq, inv, mb,
                                 T, N, W, getattr(enc, "_ocppo_box", None), box, idx)
    hidden._ocppo_box = box
    return hidden


# The frame gather and the encoder's first Linear(+ReLU) as one HIP launch
# (ops.frames_gather_linear) when that layer has <= 16 inputs and FlatAdam-owned grads; its
# backward is the one-pass ReLU-backward + bias + weight gradient (ops.relu_bias_wgrad).
FUSED_GATHER_L1 = True
# ... which also makes the gathered decoder's [M, W] row table (ops.frames_gather_linear's index)
FUSED_INDEX_IN_GATHER = True


class _GatherLinear1(torch.autograd.Function):
    """h1 = relu(frames_gather(obs, uniq) @ W1^T + b1); backward = dW1 / db1 only (the frames
    need no gradient), written into the FlatAdam-owned grads. slot: a dict the next layer's
    backward may leave its weight-gradient step in ("run"); it then runs here, after this layer's
    rows launch, carrying this layer's finish in its split-K combine (no finish launch)."""

    @staticmethod
    def forward(ctx, w, b, obs, uniq, slot=None, index=None):
        # index = (pos_of, perm, dones, holder): the decoder's row table made by the same launch
        # (holder["idx"])
        if index is not None:
            x, h1, index[3]["idx"] = ops.timed(
                "frames_gather_linear",
                lambda: ops.frames_gather_linear(obs, uniq, w, b, relu=True, index=index[:3]))
        else:
            x, h1 = ops.timed("frames_gather_linear",
                              lambda: ops.frames_gather_linear(obs, uniq, w, b, relu=True))
        ctx.save_for_backward(x, h1)
        ctx.params, ctx.slot = (w, b), slot
        if slot is not None:
            # the next layer's dX may run this layer's backward in its epilogue
            # (ops.dx_x6_wgrad); it then marks the slot "done" and passes no gradient down
            slot["l1"] = (x, w, b)
            ctx.set_materialize_grads(False)
        return h1

    @staticmethod
    def backward(ctx, g):
        x, h1 = ctx.saved_tensors
        w, b = ctx.params
        if ctx.slot is not None:
            ctx.slot.pop("l1", None)
            if ctx.slot.pop("done", False) or g is None:
                # a weight-gradient step the next layer left here must still run (with no
                # finish to carry: this layer wrote nothing to finish)
                run = ctx.slot.pop("run", None)
                if run is not None:
                    run(None)
                return None, None, None, None, None, None
        g = g.contiguous()
        run = ctx.slot.pop("run", None) if ctx.slot is not None else None
        if run is None or g.shape[0] == 0:
            ops.timed(f"relu_bias_wgrad_{g.shape[0]}x{g.shape[1]}x{x.shape[1]}",
                      lambda: ops.relu_bias_wgrad(g, h1, x, dw=w.grad, db=b.grad))
            if run is not None:
                run(None)
            return None, None, None, None, None, None
        fin = ops.DeferredFinish(g.device)
        ops.timed(f"relu_bias_wgrad_{g.shape[0]}x{g.shape[1]}x{x.shape[1]}",
                  lambda: ops.relu_bias_wgrad(g, h1, x, dw=w.grad, db=b.grad, defer=fin))
        run(fin)
        fin.run()  # no-op when the combine took it
        return None, None, None, None, None, None


def _gather_l1_ok(agent, obs, split: int) -> bool:
    from .agents import _direct

    net = agent.network
    flat = getattr(agent, "_flat", 0)
    if not (FUSED_GATHER_L1 and torch.is_grad_enabled() and obs.is_cuda and flat >= 4
            and (split == 0 or split >= 2) and isinstance(net[0], torch.nn.Linear)
            and isinstance(net[1], torch.nn.ReLU) and net[0].bias is not None):
        return False
    l1 = net[0]
    return (l1.in_features == obs.shape[-1] <= 16 and l1.out_features % 4 == 0
            and l1.out_features <= 1024 and _direct(l1.weight) and _direct(l1.bias)
            and l1.weight.is_contiguous())


# The DP cut's leaf carries the box of the layer below it (_cut). Off only to show what the box
# buys (tests/test_dp_gpu.py: without it the split chain's arithmetic differs from the uncut one)
CUT_CARRIES_BOX = True


def _cut(low):
    """The leaf the layers above a DP cut read instead of `low`. It carries `low`'s box (the
    Linear+ReLU that produced it), so the first layer above the cut still takes that ReLU's
    backward and bias-gradient partials into its dX epilogue (agents._LinearAct, ops.dx_x6_relu):
    the same products in the same order as the uncut chain, the partials handed across the cut in
    the box. Without it the lower phase re-derives them with relu_bias_grad's row chunks, a
    different summation order of that layer's bias gradient (VERDICT r05 Weak 1)."""
    low_d = low.detach().requires_grad_()
    box = getattr(low, "_ocppo_box", None)
    if box is not None and CUT_CARRIES_BOX:
        low_d._ocppo_box = box
    return low_d


def minibatch_hidden(agent, obs, dones, uniq, pos_of, inv, perm, mb: int, split: int = 0):
    """Decoder output of PPObj for the samples `perm` (one minibatch) from the rollout obs
    [T+1, N, W, F] with each distinct frame encoded once; autograd flows to every parameter.
    `mb` is the minibatch's index within its epoch (inv is that epoch's inverse permutation).

    split > 0 cuts the autograd graph after agent.network[:split] (a prefix of the encoder) and
    returns (hidden, (low, low_detached)): a backward from the heads then stops at
    `low_detached`, and `torch.autograd.backward(low, low_detached.grad)` finishes it -- two
    phases, so the data-parallel trainer can all-reduce the gradients of the layers above the
    cut while the layers below it still run their backward."""
    from .agents import fused_trunk

    T1, N, W, _ = obs.shape
    T = T1 - 1
    cut = None
    if _gather_l1_ok(agent, obs, split):
        l1 = agent.network[0]
        # the second layer's weight gradient may wait for this layer's backward only when both
        # run in the same backward phase: a DP cut between them (split == 2) would all-reduce
        # that gradient (the buffer's tail) while the lower phase still writes it
        slot = {} if split == 0 or split >= 4 else None
        # the gathered decoder's row table from the same launch (used when the decoder takes
        # the gathered path below; an unused table costs the launch a few workgroups)
        hold = {}
        index = ((pos_of, perm, dones, hold)
                 if FUSED_INDEX_IN_GATHER and FUSED_DECODE_GATHER and torch.is_grad_enabled()
                 else None)
        h1 = _GatherLinear1.apply(l1.weight, l1.bias, obs, uniq, slot, index)
        if slot is not None:
            h1._ocppo_wslot = slot
        if split:
            low = fused_trunk(agent.network[2:split], h1)
            low_d = _cut(low)
            enc = fused_trunk(agent.network[split:agent._flat], low_d, rows_last=SCATTER_MBITS)
            cut = (low, low_d)
        else:
            enc = fused_trunk(agent.network[2:agent._flat], h1, rows_last=SCATTER_MBITS)
        if _decode_gather_ok(agent, enc, perm.numel(), W):
            hidden = _decode_frames(agent, enc, pos_of, perm, dones, uniq, inv, mb, T, N, W,
                                    idx=hold.get("idx"))
            return (hidden, cut) if split else hidden
        h = _FramesExpand.apply(enc.contiguous(), pos_of, perm, dones, uniq, inv, mb, T, N, W,
                                getattr(enc, "_ocppo_box", None))
        hidden = agent.decode(h)
        return (hidden, cut) if split else hidden
    x = ops.timed("frames_gather", lambda: ops.frames_gather(obs, uniq))
    if split:
        low = fused_trunk(agent.network[:split], x)
        low_d = _cut(low)
        enc = fused_trunk(agent.network[split:agent._flat], low_d)
        cut = (low, low_d)
    else:
        enc = agent.encode(x)
    h = _FramesExpand.apply(enc.contiguous(), pos_of, perm, dones, uniq, inv, mb, T, N, W,
                            getattr(enc, "_ocppo_box", None))
    hidden = agent.decode(h)
    return (hidden, cut) if split else hidden
