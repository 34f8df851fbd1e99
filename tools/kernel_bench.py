"""Per-kernel microbenchmark of libocppo_hip.so at the config sizes and at scaled sizes.

Each case builds its inputs on the GPU, captures `reps` back-to-back launches of ONE kernel into a
hipGraph, and times `rounds` replays with HIP events: mean launch duration = elapsed / (reps x
rounds). Algorithmic bytes per launch are the DESIGN.md figures, so GB/s = bytes / duration.

    python tools/kernel_bench.py                       # all kernels, config + scaled, JSON lines
    python tools/kernel_bench.py --kernel gae --size scaled --reps 20   # one case (for rocprofv3)

Scaled sizes are chosen to stream well past the 256 MiB Infinity Cache so that HBM, not the
on-die caches, bounds them.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from oc_cleanrl_amd import ops  # noqa: E402
from oc_cleanrl_amd.trainer import replay_time_us  # noqa: E402

HBM_PEAK_GBS = 8000.0
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA (= the f32 vector rate)

SIZES = {
    # name: {size: params}
    # GAE as the trainer runs it: advantages / returns + the 16-B sample records (ops.gae with
    # records); gae_plain without the records
    "gae": {"config": dict(T=128, N=128), "scaled": dict(T=128, N=262144)},
    "gae_plain": {"config": dict(T=128, N=128), "scaled": dict(T=128, N=262144)},
    "ppo_loss": {"config": dict(M=4096, A=6, B=16384), "scaled": dict(M=4 * 1024 * 1024, A=6, B=4 * 1024 * 1024)},
    "gather": {"config": dict(M=4096, B=16384, R=48), "scaled": dict(M=1 << 20, B=1 << 20, R=48)},
    # config-3 minibatch gather: u8 frame stacks -> f32 NHWC (NatureCNN input, 8192 rows)
    "gather_pixels": {"config": dict(M=8192, B=16384), "scaled": dict(M=16384, B=32768)},
    "rollout_store": {"config": dict(N=128, W=4, D=12), "scaled": dict(N=1 << 20, W=4, D=12)},
    "action_head": {"config": dict(N=128, A=6), "scaled": dict(N=4 * 1024 * 1024, A=6)},
    "env_step": {"config": dict(N=128, D=12), "scaled": dict(N=4 * 1024 * 1024, D=12)},
    "adv_stats": {"config": dict(M=4096, nmb=16, B=16384), "scaled": dict(M=16384, nmb=256, B=1 << 20)},
    "mb_prepare": {"config": dict(M=4096, nmb=16, B=16384), "scaled": dict(M=16384, nmb=256, B=1 << 20)},
    # the same from the five SoA arrays (the form before GAE packed 16-B sample records)
    "mb_prepare_soa": {"config": dict(M=4096, nmb=16, B=16384), "scaled": dict(M=16384, nmb=256, B=1 << 20)},
    "ppo_loss_prepared": {"config": dict(M=4096, A=6), "scaled": dict(M=4 * 1024 * 1024, A=6)},
    "policy_head": {"config": dict(N=128, H=512, A=6), "scaled": dict(N=262144, H=512, A=6)},
    # the two Linear->ReLU backward launches of one config-2 minibatch (dedup capacity 11520
    # encoder rows: layers 1024/512 -- the first layer (256) runs relu_bias_wgrad, the last
    # encoder layer's mask rides in frames_scatter_relu, the decoder's in heads_loss), and one
    # streaming-size launch
    "relu_bias_grad": {"config": dict(shapes=((11520, 1024), (11520, 512))),
                       "scaled": dict(shapes=((262144, 1024),))},
    # the first encoder layer's fused ReLU-backward + bias + weight gradient (F = 12 -> 256)
    "relu_bias_wgrad": {"config": dict(R=11520, N=256, K=12), "scaled": dict(R=262144, N=256, K=12)},
    # actor + critic heads' backward with the decoder's ReLU mask + bias grad (M = 4096, H = 512)
    "heads_bwd": {"config": dict(M=4096, H=512, A=6), "scaled": dict(M=262144, H=512, A=6)},
    # policy heads forward + fused PPO loss + heads backward (both launches: rows, then records)
    "heads_loss": {"config": dict(M=4096, H=512, A=6), "scaled": dict(M=262144, H=512, A=6)},
    # the dedup update's frame gather fused with the first encoder Linear+ReLU (F=12 -> 256) at
    # the frame capacity of config 2 (11520 distinct frames of a [129, 128, 4, 12] bf16 rollout)
    "frames_gather_linear": {"config": dict(T=128, N=128, W=4, F=12, C=11520, N1=256),
                             "scaled": dict(T=128, N=2048, W=4, F=12, C=184320, N1=256)},
    # relu_bias_grad with its in-launch last-arriver bias-gradient tail (conv layers; the
    # Linear layers at config run the deferred form above, ops.relu_bias_grad_partial)
    "relu_bias_grad_tail": {"config": dict(shapes=((12288, 512), (12288, 1024), (12288, 512))),
                            "scaled": dict(shapes=((262144, 1024),))},
    # the update's frame scatter with the last encoder layer's ReLU backward (config 2: a
    # 4096-sample minibatch of a [128, 128] rollout, W = 4, E = 512, the planner's 11520 rows):
    # mask from the forward's row-major bitmask; frames_scatter_relu_f32 reads the f32 output
    "frames_scatter_relu": {"config": dict(T=128, N=128, W=4, M=4096, E=512),
                            "scaled": dict(T=128, N=2048, W=4, M=65536, E=512)},
    "frames_scatter_relu_f32": {"config": dict(T=128, N=128, W=4, M=4096, E=512),
                                "scaled": dict(T=128, N=2048, W=4, M=65536, E=512)},
    # the rollout's last encoder layer writing the frame-encoding ring (M = 128 envs, 1024 -> 512)
    "cache_linear": {"config": dict(M=128, K=1024, E=512, W=4), "scaled": dict(M=8192, K=1024, E=512, W=4)},
    # the rollout decoder on the frame-encoding ring (128 envs, W*E = 4*512 -> 512, rot 1) and the
    # middle encoder layer (512 -> 1024): the LDS-staged f32-MFMA Linear kernel
    "decoder": {"config": dict(M=128, K=2048, N=512, seg=512), "scaled": dict(M=8192, K=2048, N=512, seg=512)},
    "encoder_mid": {"config": dict(M=128, K=512, N=1024), "scaled": dict(M=8192, K=512, N=1024)},
    # the rollout store of step t-1 + the first two encoder layers of step t (F=12 -> 256 -> 512)
    "store_encode": {"config": dict(N=128, W=4, F=12, N1=256, N2=512),
                     "scaled": dict(N=8192, W=4, F=12, N1=256, N2=512)},
    # the update GEMM on the bf16 matrix cores (exact-split f32): the middle encoder layer's
    # forward at the dedup capacity (x [11520, 512] -> [11520, 1024], bias + ReLU) and a large
    # square-ish product
    "gemm_x6": {"config": dict(M=11520, N=1024, K=512), "scaled": dict(M=8192, N=8192, K=4096)},
}

# useful flops per launch of the MFMA kernels (2 per multiply-add)
FLOPS = {
    "cache_linear": lambda p: 2 * p["M"] * p["K"] * p["E"],
    "decoder": lambda p: 2 * p["M"] * p["K"] * p["N"],
    "encoder_mid": lambda p: 2 * p["M"] * p["K"] * p["N"],
    # f32-equivalent flops (the bf16 MFMA work issued is 6x)
    "gemm_x6": lambda p: 2 * p["M"] * p["K"] * p["N"],
    "store_encode": lambda p: 2 * p["N"] * (p["F"] * p["N1"] + p["N1"] * p["N2"]),
}


def relu_bias_grad_bytes(shapes):
    """g + out in, gp out (f32 [R, N]) + db out, summed over the launches."""
    return sum(R * N * 12 + 4 * N for R, N in shapes)


def case_bytes(name: str, p: dict) -> float:
    """Algorithmic bytes per launch of a case (the DESIGN.md §4 figures; no GPU needed, so
    tools/summarize_profiles.py prices the PMC passes with the same numbers). ppo_loss gathers its
    records through the minibatch indices (8A+32 B per element + the 4-B index); the prepared
    form reads them contiguous (8A+32)."""
    if name == "gae":  # + log-prob 4 + action 8 in, the 16-B record out
        return 48 * p["T"] * p["N"] + 8 * p["N"]
    if name == "gae_plain":
        return 20 * p["T"] * p["N"] + 8 * p["N"]
    if name == "ppo_loss":
        return (8 * p["A"] + 36) * p["M"]
    if name == "ppo_loss_prepared":
        return (8 * p["A"] + 32) * p["M"]
    if name == "gather":
        return p["M"] * (8 + p["R"] * 6)
    if name == "gather_pixels":
        return p["M"] * (8 + 4 * 7056 * 5)
    if name == "rollout_store":
        N, W, D = p["N"], p["W"], p["D"]
        return N * ((W - 1) * D * 2 + D * 4 + W * D * 6 + 16)
    if name == "action_head":
        return p["N"] * (8 * p["A"] + 8 + 4 + 8)
    if name == "env_step":
        return p["N"] * (8 + p["D"] * 4 + 8 + 2 * 20)
    if name == "adv_stats":
        return 2 * p["nmb"] * p["M"] * 12
    if name in ("mb_prepare", "mb_prepare_soa"):
        return p["nmb"] * p["M"] * (8 + 2 * (8 + 16))
    if name == "policy_head":
        N, H, A = p["N"], p["H"], p["A"]
        return N * (4 * H + 4 * A + 16) + 4 * (A + 1) * (H + 1)
    if name in ("relu_bias_grad", "relu_bias_grad_tail"):
        return relu_bias_grad_bytes(p["shapes"])
    if name == "heads_loss":
        # h in + gp out; records (action 8 + 4 x 4) in; [Wa; Wc] + biases in; head grads out
        M, H, A = p["M"], p["H"], p["A"]
        return M * H * 8 + M * 24 + 4 * (A + 1) * (H + 1) + 4 * ((A + 1) * (H + 1) + H) + 36
    if name == "frames_gather_linear":  # frame id 4 + bf16 row in + f32 row out + f32 h out
        return p["C"] * (4 + p["F"] * (2 + 4) + 4 * p["N1"])
    if name == "cache_linear":  # ring form: x + W in, the fresh row written into one slot
        M, K, E = p["M"], p["K"], p["E"]
        return 4 * (M * K + E * (K + 1)) + 4 * M * E + 4 * M
    if name in ("decoder", "encoder_mid"):  # x + W + b in, y out
        M, K, N = p["M"], p["K"], p["N"]
        return 4 * (M * K + N * (K + 1) + M * N)
    if name == "store_encode":
        N, W, F, N1, N2 = p["N"], p["W"], p["F"], p["N1"], p["N2"]
        store = N * ((W - 1) * F * 2 + F * 4 + W * F * 6 + 8 + 4 + 24 + 4)
        return store + 4 * (N1 * (F + 1) + N2 * (N1 + 1)) + 4 * N * N2
    if name == "heads_bwd":
        M, H, A = p["M"], p["H"], p["A"]
        return M * H * 8 + M * (A + 1) * 4 + 2 * (A + 1) * H * 4 + H * 4 + (A + 1) * 4
    if name == "relu_bias_wgrad":
        R, N, K = p["R"], p["N"], p["K"]
        return R * N * 8 + R * K * 4 + N * (K + 1) * 4
    if name == "gemm_x6":  # x, W (+ bias) in, y out
        M, N, K = p["M"], p["N"], p["K"]
        return 4 * (M * K + N * (K + 1) + M * N)
    if name in ("frames_scatter_relu", "frames_scatter_relu_f32"):
        # dh [M, W, E] in; per frame: id 4 + the mask (1 bit or 4 B per element) in, gp out;
        # the bias-gradient partials (one row per 16 frames) out. C = the plan's capacity.
        M, W, E = p["M"], p["W"], p["E"]
        C = p.get("C") or _scatter_plan(p, None)[0]
        mask = E // 8 if name == "frames_scatter_relu" else 4 * E
        return 4 * M * W * E + C * (4 + 4 * E + mask) + 4 * E * -(-C // 16)
    raise KeyError(name)


_PLANS = {}


def _scatter_plan(p: dict, dev):
    """(C, uniq, inv, dones) of minibatch 0 of a seeded [T, N] rollout's first epoch (the trainer's
    FramePlanner, 4 minibatches of M); host arrays when dev is None."""
    key = (p["T"], p["N"], p["W"], p["M"], str(dev))
    if key not in _PLANS:
        import numpy as np

        from oc_cleanrl_amd.frames import FramePlanner

        T, N, W, M = p["T"], p["N"], p["W"], p["M"]
        B = T * N
        pl = FramePlanner(T, N, W, M, 1, B // M)
        perm = np.random.default_rng(0).permutation(B).astype(np.int64)
        used, inv = pl.plan(perm)
        cap = pl.cap_for(pl.counts)
        buf = np.zeros(pl.size(cap), np.int32)
        pl.fill(buf, cap, used, inv)
        uniq, _, iv = pl.views(buf, cap)
        dones = (np.random.default_rng(1).random((T + 1, N)) < 1 / 3500).astype(np.float32)
        if dev is None:
            return cap, uniq[0], iv[0], dones
        _PLANS[key] = (cap, torch.from_numpy(uniq[0].copy()).to(dev),
                       torch.from_numpy(iv[0].copy()).to(dev), torch.from_numpy(dones).to(dev))
    return _PLANS[key]


def make_case(name: str, p: dict, dev):
    """Returns (launch closure, algorithmic bytes per launch)."""
    g = torch.Generator(device=dev).manual_seed(0)
    f32 = torch.float32
    if name == "gae_plain":
        T, N = p["T"], p["N"]
        r = torch.randn(T, N, device=dev, generator=g)
        v = torch.randn(T, N, device=dev, generator=g)
        d = (torch.rand(T, N, device=dev, generator=g) < 0.01).float()
        nv, nd = torch.randn(N, device=dev, generator=g), torch.zeros(N, device=dev)
        adv, ret = torch.empty_like(r), torch.empty_like(r)
        return (lambda: ops.gae(r, v, d, nv, nd, 0.99, 0.95, adv, ret)), 20 * T * N + 8 * N
    if name == "gae":
        T, N = p["T"], p["N"]
        r = torch.randn(T, N, device=dev, generator=g)
        v = torch.randn(T, N, device=dev, generator=g)
        d = (torch.rand(T, N, device=dev, generator=g) < 0.01).float()
        nv, nd = torch.randn(N, device=dev, generator=g), torch.zeros(N, device=dev)
        lp = torch.randn(T, N, device=dev, generator=g)
        act = torch.randint(0, 6, (T, N), device=dev, generator=g)
        rec = ops.sample_records(T * N, dev)
        adv, ret = torch.empty_like(r), torch.empty_like(r)
        return (lambda: ops.gae(r, v, d, nv, nd, 0.99, 0.95, adv, ret, logprobs=lp, actions=act,
                                records=rec)), 48 * T * N + 8 * N
    if name == "ppo_loss":
        M, A, B = p["M"], p["A"], p["B"]
        logits = torch.randn(M, A, device=dev, generator=g)
        val = torch.randn(M, device=dev, generator=g)
        acts = torch.randint(0, A, (B,), device=dev, generator=g)
        lp, adv, ret, bv = (torch.randn(B, device=dev, generator=g) for _ in range(4))
        idx = torch.randperm(B, device=dev, generator=g)[:M]
        st = ops.minibatch_adv_stats(adv, idx, M)
        ws = ops.LossWorkspace(M, A, dev)
        dl, dv, stats = torch.empty_like(logits), torch.empty(M, device=dev), torch.empty(9, device=dev)
        fn = lambda: ops.ppo_loss_fwd_bwd(  # noqa: E731
            logits, val, acts, lp, adv, ret, bv, mb_inds=idx, adv_stats=st[0], clip_coef=0.1,
            ent_coef=0.01, vf_coef=0.5, norm_adv=True, clip_vloss=True, dlogits=dl, dvalue=dv,
            stats=stats, workspace=ws)
        return fn, (8 * A + 36) * M
    if name == "gather":
        M, B, R = p["M"], p["B"], p["R"]
        src = torch.randint(0, 200, (B, R), device=dev, generator=g).to(torch.bfloat16)
        idx = torch.randperm(B, device=dev, generator=g)[:M]
        out = torch.empty(M, R, device=dev)
        return (lambda: ops.gather_rows(src, idx, out)), M * (8 + R * 6)
    if name == "gather_pixels":
        M, B = p["M"], p["B"]
        src = torch.randint(0, 256, (B, 4, 84, 84), device=dev, generator=g).to(torch.uint8)
        idx = torch.randperm(B, device=dev, generator=g)[:M]
        out = torch.empty(M, 4, 84, 84, device=dev, memory_format=torch.channels_last)
        return (lambda: ops.gather_rows(src, idx, out)), M * (8 + 4 * 7056 * 5)
    if name == "rollout_store":
        N, W, D = p["N"], p["W"], p["D"]
        frame = torch.randint(0, 200, (N, D), device=dev, generator=g).float()
        rew, done = torch.randn(N, device=dev, generator=g), torch.zeros(N, device=dev)
        prev = torch.randint(0, 200, (N, W, D), device=dev, generator=g).to(torch.bfloat16)
        out = torch.empty_like(prev)
        net = torch.empty(N, W, D, device=dev)
        ro, do = torch.empty(N, device=dev), torch.empty(N, device=dev)
        fn = lambda: ops.rollout_store(frame, rew, done, prev, out, net, ro, do)  # noqa: E731
        return fn, N * ((W - 1) * D * 2 + D * 4 + W * D * 6 + 16)
    if name == "action_head":
        N, A = p["N"], p["A"]
        logits = torch.randn(N, A, device=dev, generator=g)
        noise = torch.empty(N, A, device=dev).exponential_(generator=g)
        act, lp = torch.empty(N, dtype=torch.int64, device=dev), torch.empty(N, device=dev)
        vi, vo = torch.randn(N, device=dev, generator=g), torch.empty(N, device=dev)
        fn = lambda: ops.categorical_sample(logits, noise, act, lp, None, vi, vo)  # noqa: E731
        return fn, N * (8 * A + 8 + 4 + 8)
    if name == "env_step":
        N, D = p["N"], p["D"]
        base = torch.zeros(1, dtype=torch.int64, device=dev)
        acts = torch.randint(0, 6, (N,), device=dev, generator=g)
        frame = torch.empty(N, D, device=dev)
        rew, done = torch.empty(N, device=dev), torch.empty(N, device=dev)
        ep = torch.zeros(N, 5, device=dev)
        fn = lambda: ops.synth_env_step(42, base, 0, acts, frame, rew, done, ep)  # noqa: E731
        return fn, N * (8 + D * 4 + 8 + 2 * 20)
    if name == "adv_stats":
        M, nmb, B = p["M"], p["nmb"], p["B"]
        adv = torch.randn(B, device=dev, generator=g)
        reps = (nmb * M + B - 1) // B
        perm = torch.cat([torch.randperm(B, device=dev, generator=g) for _ in range(reps)])[:nmb * M]
        out = torch.empty(nmb, 2, device=dev)
        return (lambda: ops.minibatch_adv_stats(adv, perm, M, out)), 2 * nmb * M * 12
    if name in ("mb_prepare", "mb_prepare_soa"):
        # mb_prepare: the trainer's form, from GAE's 16-B sample records (the records are made
        # here by ops.gae on a [T, B / T] rollout of the same arrays)
        M, nmb, B = p["M"], p["nmb"], p["B"]
        reps = (nmb * M + B - 1) // B
        perm = torch.cat([torch.randperm(B, device=dev, generator=g) for _ in range(reps)])[:nmb * M]
        acts = torch.randint(0, 6, (B,), device=dev, generator=g)
        lp, adv, ret, bv = (torch.randn(B, device=dev, generator=g) for _ in range(4))
        rec = None
        if name == "mb_prepare":
            T = 128
            rec = ops.sample_records(B, dev)
            z = torch.zeros(B // T, device=dev)
            ops.gae(torch.randn(T, B // T, device=dev, generator=g), bv.view(T, -1),
                    torch.zeros(T, B // T, device=dev), z, z, 0.99, 0.95, adv.view(T, -1),
                    ret.view(T, -1), logprobs=lp.view(T, -1), actions=acts.view(T, -1),
                    records=rec)
        out = ops.minibatch_prepare(perm, M, acts, lp, adv, ret, bv, records=rec)
        fn = lambda: ops.minibatch_prepare(perm, M, acts, lp, adv, ret, bv, out=out,  # noqa: E731
                                           records=rec)
        return fn, nmb * M * (8 + 2 * (8 + 16))
    if name == "ppo_loss_prepared":
        M, A = p["M"], p["A"]
        logits = torch.randn(M, A, device=dev, generator=g)
        val = torch.randn(M, device=dev, generator=g)
        acts = torch.randint(0, A, (M,), device=dev, generator=g)
        lp, adv, ret, bv = (torch.randn(M, device=dev, generator=g) for _ in range(4))
        st = torch.tensor([0.1, 1.3], device=dev)
        ws = ops.LossWorkspace(M, A, dev)
        dl, dv, stats = torch.empty_like(logits), torch.empty(M, device=dev), torch.empty(9, device=dev)
        fn = lambda: ops.ppo_loss_fwd_bwd(  # noqa: E731
            logits, val, acts, lp, adv, ret, bv, adv_stats=st, clip_coef=0.1, ent_coef=0.01,
            vf_coef=0.5, norm_adv=True, clip_vloss=True, dlogits=dl, dvalue=dv, stats=stats,
            workspace=ws)
        return fn, (8 * A + 32) * M
    if name == "policy_head":
        N, H, A = p["N"], p["H"], p["A"]
        hid = torch.relu(torch.randn(N, H, device=dev, generator=g))
        wa, ba = torch.randn(A, H, device=dev, generator=g) * 0.05, torch.zeros(A, device=dev)
        wc, bc = torch.randn(1, H, device=dev, generator=g), torch.zeros(1, device=dev)
        noise = torch.empty(N, A, device=dev).exponential_(generator=g)
        act, lp = torch.empty(N, dtype=torch.int64, device=dev), torch.empty(N, device=dev)
        vo = torch.empty(N, device=dev)
        fn = lambda: ops.policy_head_sample(hid, wa, ba, wc, bc, noise, act, lp, vo)  # noqa: E731
        return fn, N * (4 * H + 4 * A + 16) + 4 * (A + 1) * (H + 1)
    if name in ("relu_bias_grad", "relu_bias_grad_tail"):
        bufs = []
        for R, N in p["shapes"]:
            gg = torch.randn(R, N, device=dev, generator=g)
            out = torch.relu(torch.randn(R, N, device=dev, generator=g))
            bufs.append((gg, out, torch.empty_like(gg), torch.empty(N, device=dev)))

        def fn():
            for gg, out, gp, db in bufs:
                if name == "relu_bias_grad":
                    ops.relu_bias_grad_partial(gg, out, gp=gp)
                else:
                    ops.relu_bias_grad(gg, out, db=db, gp=gp)
        return fn, relu_bias_grad_bytes(p["shapes"])
    if name == "heads_loss":
        M, H, A = p["M"], p["H"], p["A"]
        hh = torch.relu(torch.randn(M, H, device=dev, generator=g))
        wa, ba = torch.randn(A, H, device=dev, generator=g) * 0.05, torch.zeros(A, device=dev)
        wc, bc = torch.randn(1, H, device=dev, generator=g) * 0.05, torch.zeros(1, device=dev)
        acts = torch.randint(0, A, (M,), device=dev, generator=g)
        lp, adv, ret, val = (torch.randn(M, device=dev, generator=g) for _ in range(4))
        st = torch.tensor([0.0, 1.0], device=dev)
        gp, dbh = torch.empty_like(hh), torch.empty(H, device=dev)
        dwa, dwc = torch.empty(A, H, device=dev), torch.empty(1, H, device=dev)
        dba, dbc, stats = torch.empty(A, device=dev), torch.empty(1, device=dev), torch.empty(9, device=dev)
        fn = lambda: ops.heads_loss_fwd_bwd(  # noqa: E731
            hh, wa, ba, wc, bc, acts, lp, adv, ret, val, adv_stats=st, clip_coef=0.1,
            ent_coef=0.01, vf_coef=0.5, norm_adv=True, clip_vloss=True, gp=gp, db_h=dbh, dwa=dwa,
            dwc=dwc, dba=dba, dbc=dbc, stats=stats)
        # h in + gp out; records (action 8 + 4 x 4) in; [Wa; Wc] + biases in; head grads out
        return fn, M * H * 8 + M * 24 + 4 * (A + 1) * (H + 1) + 4 * ((A + 1) * (H + 1) + H) + 36
    if name == "frames_gather_linear":
        T, N, W, F, C, N1 = p["T"], p["N"], p["W"], p["F"], p["C"], p["N1"]
        obs = torch.randint(0, 200, (T + 1, N, W, F), device=dev, generator=g).to(torch.bfloat16)
        U = (T + W - 1) * N
        uniq = torch.randperm(U, device=dev, generator=g)[:C].sort().values.to(torch.int32)
        w = torch.randn(N1, F, device=dev, generator=g) * F ** -0.5
        b = torch.randn(N1, device=dev, generator=g)
        x, h = torch.empty(C, F, device=dev), torch.empty(C, N1, device=dev)
        fn = lambda: ops.frames_gather_linear(obs, uniq, w, b, relu=True, x_out=x, h_out=h)  # noqa: E731
        return fn, case_bytes(name, p)
    if name in ("frames_scatter_relu", "frames_scatter_relu_f32"):
        T, N, W, M, E = p["T"], p["N"], p["W"], p["M"], p["E"]
        C, uniq, inv, dones = _scatter_plan(p, dev)
        dh = torch.randn(M, W, E, device=dev, generator=g)
        out = torch.relu(torch.randn(C, E, device=dev, generator=g))
        on = (out > 0).view(C, E // 32, 32).to(torch.int64) << torch.arange(32, device=dev)
        bits = on.sum(-1).to(torch.int32)  # bit 31 wraps into the sign: the same 32 bits
        gp = torch.empty(C, E, device=dev)
        if name == "frames_scatter_relu":
            fn = lambda: ops.frames_scatter_relu(dh, uniq, inv, 0, dones, T, N, W,  # noqa: E731
                                                 gp=gp, mbits=bits)
        else:
            fn = lambda: ops.frames_scatter_relu(dh, uniq, inv, 0, dones, T, N, W,  # noqa: E731
                                                 out=out, gp=gp)
        return fn, case_bytes(name, dict(p, C=C))
    if name == "cache_linear":
        M, K, E, W = p["M"], p["K"], p["E"], p["W"]
        x = torch.relu(torch.randn(M, K, device=dev, generator=g))
        w = torch.randn(E, K, device=dev, generator=g) * K ** -0.5
        b = torch.randn(E, device=dev, generator=g)
        enc = torch.randn(M, W, E, device=dev, generator=g)
        done = (torch.rand(M, device=dev, generator=g) < 1 / 3500).float()
        fn = lambda: ops.linear_cache_ring(x, w, b, enc, 1, done)  # noqa: E731
        return fn, 4 * (M * K + E * (K + 1)) + 4 * M * E + 4 * M
    if name in ("decoder", "encoder_mid"):
        M, K, N = p["M"], p["K"], p["N"]
        x = torch.relu(torch.randn(M, K, device=dev, generator=g))
        w = torch.randn(N, K, device=dev, generator=g) * K ** -0.5
        b = torch.randn(N, device=dev, generator=g)
        y = torch.empty(M, N, device=dev)
        ring = (p["seg"], 1) if "seg" in p else None
        fn = lambda: ops.linear_act(x, w, b, True, out=y, ring=ring)  # noqa: E731
        return fn, case_bytes(name, p)
    if name == "store_encode":
        N, W, F, N1, N2 = p["N"], p["W"], p["F"], p["N1"], p["N2"]
        frame = torch.randint(0, 210, (N, F), device=dev, generator=g).float()
        reward = torch.zeros(N, device=dev)
        done = (torch.rand(N, device=dev, generator=g) < 1 / 3500).float()
        prev = torch.zeros(N, W, F, dtype=torch.bfloat16, device=dev)
        out = torch.empty_like(prev)
        net = torch.empty(N, W, F, device=dev)
        dn, rw = torch.empty(N, device=dev), torch.empty(N, device=dev)
        ret = torch.zeros(N, dtype=torch.float64, device=dev)
        rms = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=dev)
        w1, b1 = torch.randn(N1, F, device=dev, generator=g) * 0.1, torch.zeros(N1, device=dev)
        w2, b2 = torch.randn(N2, N1, device=dev, generator=g) * 0.05, torch.zeros(N2, device=dev)
        y = torch.empty(N, N2, device=dev)
        fn = lambda: ops.store_linear2(frame, reward, done, prev, out, net, dn, rw, w1, b1, w2, b2,  # noqa: E731
                                       y, vecnorm_state=(ret, rms))
        store = N * ((W - 1) * F * 2 + F * 4 + W * F * 6 + 8 + 4 + 24 + 4)
        return fn, store + 4 * (N1 * (F + 1) + N2 * (N1 + 1)) + 4 * N * N2
    if name == "heads_bwd":
        M, H, A = p["M"], p["H"], p["A"]
        hh = torch.relu(torch.randn(M, H, device=dev, generator=g))
        dl, dv = torch.randn(M, A, device=dev, generator=g), torch.randn(M, device=dev, generator=g)
        wa, wc = torch.randn(A, H, device=dev, generator=g), torch.randn(H, device=dev, generator=g)
        gp, dbh = torch.empty_like(hh), torch.empty(H, device=dev)
        dwa, dwc = torch.empty(A, H, device=dev), torch.empty(1, H, device=dev)
        dba, dbc = torch.empty(A, device=dev), torch.empty(1, device=dev)
        fn = lambda: ops.heads_bwd(hh, dl, dv, wa, wc, True, gp, dbh, dwa, dwc, dba, dbc)  # noqa: E731
        return fn, M * H * 8 + M * (A + 1) * 4 + 2 * (A + 1) * H * 4 + H * 4 + (A + 1) * 4
    if name == "relu_bias_wgrad":
        R, N, K = p["R"], p["N"], p["K"]
        gg = torch.randn(R, N, device=dev, generator=g)
        out = torch.relu(torch.randn(R, N, device=dev, generator=g))
        x = torch.randn(R, K, device=dev, generator=g)
        dw, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
        fn = lambda: ops.relu_bias_wgrad(gg, out, x, dw, db)  # noqa: E731
        return fn, R * N * 8 + R * K * 4 + N * (K + 1) * 4
    if name == "gemm_x6":
        M, N, K = p["M"], p["N"], p["K"]
        x = torch.rand(M, K, device=dev, generator=g) * 2 - 1
        w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1) / K ** 0.5
        b = torch.randn(N, device=dev, generator=g) * 0.1
        y = torch.empty(M, N, device=dev)
        fn = lambda: ops.linear_x6(x, w, b, relu=True, out=y)  # noqa: E731
        return fn, case_bytes(name, p)
    raise KeyError(name)


def time_case(fn, reps=20, rounds=5, cold=False) -> float:
    """Mean launch duration (us): trainer.replay_time_us (cold = an L3 scrub before every
    launch, subtracted)."""
    return replay_time_us(fn, reps, rounds, cold=cold)


def run_case(name, size, dev, reps=20, rounds=5, cold=False) -> dict:
    fn, nbytes = make_case(name, SIZES[name][size], dev)
    assert nbytes == case_bytes(name, SIZES[name][size]), name
    us = time_case(fn, reps, rounds, cold)
    launches = len(SIZES[name][size].get("shapes", (None,)))
    us, nbytes = us / launches, nbytes / launches  # per launch (average over the launch mix)
    # (a cold figure is a difference of two timings: under a profiler with one round it can
    # come out <= 0; only the profile's counters matter there)
    gbs = nbytes / (us * 1e-6) / 1e9 if us > 0 else float("nan")
    r = {"kernel": name, "size": size, "cache": "cold" if cold else "warm",
         "params": SIZES[name][size], "mean_us": round(us, 3),
         "bytes": nbytes, "GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    if name in FLOPS:
        fl = FLOPS[name](SIZES[name][size])
        r.update(flops=fl, TFLOPs=round(fl / (us * 1e-6) / 1e12, 2),
                 mfma_frac=round(fl / (us * 1e-6) / 1e12 / MFMA_F32_PEAK_TFLOPS, 4))
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="all")
    ap.add_argument("--size", default="all", choices=["all", "config", "scaled"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--cold", action="store_true", help="L3 scrub before every launch")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    names = list(SIZES) if a.kernel == "all" else [a.kernel]
    sizes = ["config", "scaled"] if a.size == "all" else [a.size]
    for n in names:
        for s in sizes:
            print(json.dumps(run_case(n, s, dev, a.reps, a.rounds, a.cold)), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
