"""Benchmark: PPO actor-learner SPS + PPO updates/sec, ALE/Pong-v5 obj-mode (synthetic env), PPO_OBJ.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one PPO iteration of the reference loop (cleanrl/ppo_atari_oc.py:469-617) on every
rank: a T=128-step rollout of local_num_envs=128 envs (BASELINE config 2 per GPU; config 4 =
1024 envs over 8 GPUs), GAE, and update_epochs=4 x num_minibatches=4 minibatch updates with an
RCCL gradient all-reduce per minibatch when N > 1 (ppo_atari_multigpu semantics, weak scaling).
value = env steps of all ranks / max-over-ranks wall time of the K timed iterations.

Rank 0 prints ONE JSON line. Extra fields: `roofline` (dominant HIP kernel of this package, live
HIP-event timing over the timed region), `kernels` (every HIP kernel's mean launch duration and
algorithmic GB/s), `roofline_scaled` (N=1: the north-star kernels the timed path runs -- GAE, minibatch
prepare, the fused heads + loss pair -- and the rollout head and ReLU backward re-timed cold at
streaming sizes, where HBM rather than launch latency bounds them; same algorithmic-byte formulas,
tools/kernel_bench.py cases), `cpu_baseline` (the oracle's CPU port of
the same loop timed on this host, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
MFMA_F32_PEAK_TFLOPS = 157.3  # dense f32 MFMA (MI355X_MICROARCH.md; no xf32 on gfx950)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (the matrix rate ocppo_gemm_x6 runs on)
RIDGE = MFMA_F32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)  # flop/B where the two bounds meet
# HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE, separate passes) of
# the same launch shapes: tools/profile_round.sh -> tools/summarize_profiles.py
PMC_SUMMARY = ROOT / "profiles" / "r05" / "pmc_summary.json"
# in-situ HBM bytes of the bench's own gemm_x6 launches (all shapes, mean per dispatch):
# tools/pmc_bench.sh -> tools/pmc_bench_summary.py
PMC_BENCH = ROOT / "profiles" / "r05" / "pmc_bench.json"
PMC_KEYS = {"gemm_x6": "gemm_x6", "action_head": "policy_head_config", "gae": "gae_config",
            "ppo_loss": "ppo_loss_prepared_config", "relu_bias_grad": "relu_bias_grad_config",
            "cache_linear": "cache_linear_config", "store_encode": "store_encode_config",
            "heads_bwd": "heads_bwd_config", "relu_bias_wgrad": "relu_bias_wgrad_config",
            "heads_loss": "heads_loss_config", "decoder": "decoder_config",
            "encoder_mid": "encoder_mid_config", "mb_prepare": "mb_prepare_config",
            "frames_scatter_relu": "frames_scatter_relu_config"}


def pmc_traffic(key):
    try:
        if key == "gemm_x6":
            rec = json.loads(PMC_BENCH.read_text())["gemm_x6"]
            return rec.get("traffic_bytes"), str(PMC_BENCH.relative_to(ROOT))
        rec = json.loads(PMC_SUMMARY.read_text())["kernels"][key]
        return rec.get("traffic_bytes"), str(PMC_SUMMARY.relative_to(ROOT))
    except (OSError, KeyError, ValueError):
        return None, None


def kernel_bytes(tr) -> dict:
    """ALGORITHMIC bytes per launch of each timed HIP kernel."""
    N, T, M, A = tr.N, tr.T, tr.M, tr.A
    W, D = tr.obs_shape[0], int(torch.tensor(tr.obs_shape[1:]).prod())
    sb = tr.obs.element_size()
    fb = tr.env.frame.element_size()
    kb = {
        # read r, v, d [T,N] + next v/d [N]; write adv, ret [T,N] (+ with the sample records:
        # log-prob 4 + action 8 in, the 16-B record out)
        "gae": (48 if tr.records is not None else 20) * T * N + 8 * N,
        # logits 4A + value 4 + action 8 + old logprob/adv/return/value 16 in (contiguous,
        # prepared); dlogits 4A + dv 4 out
        "ppo_loss": (8 * A + 32) * M,
        # index 8 + row read (storage dtype) + f32 row write
        "gather": M * (8 + W * D * (sb + 4)),
        # prev slot (W-1 frames) + new frame + done in; slot + f32 net obs out; done row; fused
        # VecNormalize: reward in, ret f64 read/write (2 passes), reward out
        "rollout_store": N * ((W - 1) * D * sb + D * fb + W * D * (sb + 4) + 8 + 4 + 24 + 4),
        # hidden row + noise in; action i64 + logprob + value out (the A+1 weight rows are shared,
        # L2-resident: counted once per launch)
        "action_head": N * (4 * tr.H + 4 * A + 16) + 4 * (A + 1) * (tr.H + 1),
        # actions in; frame + reward + done + episode counters out (read-modify-write)
        "env_step": N * (8 + D * fb + 8 + 2 * 20),
        # perm index + 5 gathered per-sample values in, 5 written in minibatch order
        "mb_prepare": tr.E * tr.B * (8 + 2 * (8 + 16)),
        # fresh encoding row + done + W-1 shifted slots in; W slots out
        "frame_cache": (N * (4 + 4 * tr.enc_cache.shape[2] * (2 * tr.enc_cache.shape[1]))
                        if tr.enc_cache is not None else None),
    }
    if tr.rollout_fusion:
        lins = [m for m in tr.agent.network[:tr.agent._flat] if isinstance(m, torch.nn.Linear)]
        N1, N2 = lins[0].out_features, lins[1].out_features
        E, Kl = lins[-1].out_features, lins[-1].in_features
        # store (as rollout_store) + linear2: W1, W2 in, y [N, N2] out (the frame is counted once)
        kb["store_encode"] = kb["rollout_store"] + 4 * (N1 * (D + 1) + N2 * (N1 + 1)) + 4 * N * N2
        # x [N, K] + W [E, K] in; done row; ring: the fresh row into one slot (shift form: W-1
        # slots read, W written)
        kb["cache_linear"] = (4 * (N * Kl + E * (Kl + 1)) + 4 * N +
                              (4 * N * E if tr.cache_ring else 4 * N * E * (2 * W - 1)))
    if tr.rollout_fusion and len(lins) > 3:
        mid = lins[2]  # the first middle encoder layer, x [N, K] + W + b in, y out
        kb["encoder_mid"] = 4 * (N * mid.in_features + mid.out_features * (mid.in_features + 1) +
                                 N * mid.out_features)
    if tr.cache_ring:
        dec = tr.agent.network[tr.agent._flat + 1]
        kb["decoder"] = 4 * (N * dec.in_features + dec.out_features * (dec.in_features + 1) +
                             N * dec.out_features)
    if tr.fused_heads_loss:
        Hh, A1 = tr.H, tr.A + 1
        kb["heads_loss"] = (M * Hh * 8 + M * 24 + 4 * A1 * (Hh + 1) + 4 * (A1 * (Hh + 1) + Hh)
                            + 36)
    Hh = tr.agent.actor.in_features
    # heads' input h in + masked dh out [M, H]; dlogits + dv in; [Wa; Wc] in, dW + db out
    kb["heads_bwd"] = M * Hh * 8 + M * (A + 1) * 4 + 2 * (A + 1) * Hh * 4 + Hh * 4 + (A + 1) * 4
    if tr.frame_dedup:
        C, E = tr.planner.cap, tr.agent.encoding_dim
        F = D
        # frame id 4 + f32 row out (storage-dtype row in)
        kb["frames_gather"] = C * (4 + F * (sb + 4))
        # ... fused with the first encoder Linear+ReLU: + the f32 [C, N1] output (W1 from L2)
        N1 = tr.agent.network[0].out_features if hasattr(tr.agent, "network") else 0
        kb["frames_gather_linear"] = C * (4 + F * (sb + 4) + 4 * N1)
        # perm 8 + W x (dones 4 + pos_of 4) per sample; W encoded rows in, W rows out
        kb["frames_expand"] = M * (8 + 8 * W + 8 * W * E)
        # dh rows in, one row out per distinct frame
        kb["frames_scatter"] = 4 * M * W * E + C * (4 + 4 * E)
        # ... with the last encoder layer's ReLU backward: its mask in (the forward's row-major
        # bitmask, 1 bit per element, or its f32 output rows), its bias-gradient partials out
        from oc_cleanrl_amd import frames as _fr
        mask_b = E // 8 if _fr.SCATTER_MBITS and E % 32 == 0 else 4 * E
        kb["frames_scatter_relu"] = (4 * M * W * E + C * (4 + 4 * E + mask_b) +
                                     4 * E * -(-C // 16))
    return kb


def kernel_flops(tr) -> dict:
    """Useful flops per launch of the MFMA kernels (2 per multiply-add)."""
    fl = {}
    if tr.rollout_fusion:
        lins = [m for m in tr.agent.network[:tr.agent._flat] if isinstance(m, torch.nn.Linear)]
        fl["store_encode"] = 2 * tr.N * (lins[0].in_features * lins[0].out_features +
                                         lins[1].in_features * lins[1].out_features)
        fl["cache_linear"] = 2 * tr.N * lins[-1].in_features * lins[-1].out_features
        if len(lins) > 3:
            fl["encoder_mid"] = 2 * tr.N * lins[2].in_features * lins[2].out_features
    if tr.cache_ring:
        dec = tr.agent.network[tr.agent._flat + 1]
        fl["decoder"] = 2 * tr.N * dec.in_features * dec.out_features
    return fl


def gemm_x6_shape(name: str):
    """(M, N, K, splits, form) of an ops.gemm_x6 timer site `gemm_x6_{M}x{N}x{K}s{S}[m|w]`
    (form "m": the masked dX epilogue; "w": the lower layer's weight gradient in the epilogue)."""
    spec = name[len("gemm_x6_"):]
    form = spec[-1] if spec[-1] in "mw" else ""
    dims, S = spec.rstrip("mw").split("s")
    M, N, K = (int(v) for v in dims.split("x"))
    return M, N, K, int(S), form


def gemm_x6_bytes(name: str) -> int:
    """A [M, K] + B [N, K] f32 in, C [splits, M, N] f32 out (+ the [M, N] ReLU bitmask read,
    1 bit per element, and the bias-gradient partials written, in the masked dX form; the "w"
    form writes no C but reads the lower layer's f32 ReLU output [M, N] as its mask)."""
    M, N, K, S, form = gemm_x6_shape(name)
    if form == "w":
        return 4 * (M * K + N * K + M * N)
    return 4 * (M * K + N * K + S * M * N) + ((M * N) // 8 + 4 * N * (M // 128) if form == "m" else 0)


def mfma_bound(flops, nbytes) -> bool:
    """Arithmetic intensity (useful flops / algorithmic bytes) above the ridge point."""
    return bool(flops) and flops / nbytes > RIDGE


def roofline_of(name, k, flops, traffic, src):
    """The roofline record of one timed kernel: MFMA-bound when its arithmetic intensity is above
    the ridge point (timed warm: its operands are cache-resident in the iteration too), else
    HBM-bound, timed cold (an L3 scrub before every replayed launch: the operands come from HBM,
    never from Infinity-Cache hits; trainer.replay_time_us)."""
    rec = {"kernel": name, "bytes_per_launch": k["bytes"], "traffic": traffic,
           "traffic_source": src}
    if name == "gemm_x6":
        # f32 products as six bf16 piece products on the bf16 matrix cores: the MFMA work issued
        # is 6 x the f32-equivalent flops, against the dense bf16 peak
        f32e = flops / (k["mean_us"] * 1e-6) / 1e12
        rec.update(bound="mfma", mean_launch_us=k["mean_us"], cache="warm",
                   achieved=round(6 * f32e, 2), peak=MFMA_BF16_PEAK_TFLOPS, unit="TFLOP/s",
                   frac=round(6 * f32e / MFMA_BF16_PEAK_TFLOPS, 5), flops_per_launch=6 * flops,
                   f32_equivalent_tflops=round(f32e, 2), launches_per_iter=k["launches_per_iter"],
                   shapes=k.get("shapes"))
    elif mfma_bound(flops, k["bytes"]):
        ach = flops / (k["mean_us"] * 1e-6) / 1e12
        rec.update(bound="mfma", mean_launch_us=k["mean_us"], cache="warm",
                   achieved=round(ach, 2), peak=MFMA_F32_PEAK_TFLOPS, unit="TFLOP/s",
                   frac=round(ach / MFMA_F32_PEAK_TFLOPS, 5), flops_per_launch=flops)
    else:
        us = k.get("cold_us", k["mean_us"])
        ach = round(k["bytes"] / (us * 1e-6) / 1e9, 2)
        rec.update(bound="hbm", mean_launch_us=us, warm_launch_us=k["mean_us"],
                   cache="cold" if "cold_us" in k else "warm", achieved=ach, peak=HBM_PEAK_GBS,
                   unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 5))
    return rec


def relu_bias_grad_bytes(name: str):
    """relu_bias_grad_{R}x{N}[_norelu]: g (+ out in, gp out) f32 [R, N] + db [N] out;
    relu_bias_grad_bits_{R}x{N}: g in, gp out f32 [R, N], the mask 1 bit per element, db out."""
    spec = name[len("relu_bias_grad_"):]
    if spec.startswith("bits_"):
        R, N = (int(v) for v in spec[len("bits_"):].split("x"))
        return R * N * 8 + R * N // 8 + 4 * N
    relu = not spec.endswith("_norelu")
    R, N = (int(v) for v in spec.replace("_norelu", "").split("x"))
    return R * N * (12 if relu else 4) + 4 * N


def relu_bias_wgrad_bytes(name: str):
    """relu_bias_wgrad_{R}x{N}x{K}: g + out f32 [R, N] and x f32 [R, K] in, dw [N, K] + db out."""
    R, N, K = (int(v) for v in name[len("relu_bias_wgrad_"):].split("x"))
    return R * N * 8 + R * K * 4 + N * (K + 1) * 4


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, gpus: int, port: int, script=None) -> list:
    """The torch.distributed.run command that starts `gpus` ranks of this script with the same
    arguments (one process per GPU; the ranks read RANK / LOCAL_RANK / WORLD_SIZE from the env,
    as under the driver's own launch)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            str(script or ROOT / "bench.py"), *argv]


def needs_launch(gpus: int, env=os.environ) -> bool:
    """--gpus N > 1 outside a torch.distributed launch: start the ranks as a child."""
    return gpus > 1 and "WORLD_SIZE" not in env


DEADLINE_S = 540.0  # whole-run bound, under the driver's 600 s per run


def launch(argv, gpus: int, script=None, deadline_s: float | None = None) -> int:
    """Run the N ranks as ONE child process tree (not an exec), before this process makes any GPU
    call. Rank 0's JSON line is forwarded to stdout as it arrives; anything else the ranks print
    on stdout (gloo's connection chatter) goes to stderr, so stdout holds the line alone.
    Returns the child's exit code. The ranks write their phases under a status directory
    (oc_cleanrl_amd.watch); if the tree outlives `deadline_s` (the ranks' own watchdogs did not
    end it), it is killed as a whole and an error line naming every rank's phase is printed
    instead, exit code 3."""
    import shutil
    import signal
    import subprocess
    import tempfile
    import threading

    from oc_cleanrl_amd.watch import behind, read_status

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    status = tempfile.mkdtemp(prefix="ocppo_watch_")
    env["OCPPO_WATCH_DIR"] = status
    env["OCPPO_RUN_ID"] = os.path.basename(status)  # the ranks' run token (watch.run_token)
    t0 = time.monotonic()
    p = subprocess.Popen(launcher_cmd(argv, gpus, free_port(), script), env=env,
                         stdout=subprocess.PIPE, text=True, bufsize=1, start_new_session=True)
    sent = []

    def forward():
        for line in p.stdout:
            dst = sys.stdout if line.startswith("{") else sys.stderr
            if dst is sys.stdout:
                sent.append(line)
            dst.write(line)
            dst.flush()

    reader = threading.Thread(target=forward, daemon=True)
    reader.start()
    try:
        rc = p.wait(timeout=deadline_s)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        ranks = read_status(status)
        rec = {"metric": None, "value": None, "n_gpus": gpus, "error": "launcher deadline",
               "elapsed_s": round(time.monotonic() - t0, 1),
               "ranks": {str(k): v["phase"] for k, v in sorted(ranks.items())},
               "behind": behind(ranks)}
        print(json.dumps(rec), file=sys.stderr if sent else sys.stdout, flush=True)
        sent.append("deadline")
        rc = 3
    reader.join(timeout=5)
    if rc != 0 and not sent:  # the ranks died without a line: say where they were
        ranks = read_status(status)
        print(json.dumps({"metric": None, "value": None, "n_gpus": gpus,
                          "error": f"ranks exited with code {rc}",
                          "ranks": {str(k): v["phase"] for k, v in sorted(ranks.items())},
                          "failed": {str(k): v["failed"] for k, v in sorted(ranks.items())
                                     if v.get("failed")},
                          "behind": behind(ranks)}), flush=True)
    shutil.rmtree(status, ignore_errors=True)
    return rc


def replica_check(tr, world: int, device) -> dict:
    """Every rank's parameter checksum after the timed iterations, gathered on every rank and
    asserted equal: the replica invariant of ppo_atari_multigpu.py:360-377 (identical init, the
    same all-reduced gradient, the same Adam step)."""
    mine = tr.param_checksum()
    sums = [mine]
    if world > 1:
        sums = [None] * world
        dist.all_gather_object(sums, mine)
    equal = all(s == sums[0] for s in sums)
    if not equal:
        raise SystemExit(f"DP replicas diverged: parameter checksums {sums}")
    return {"param_checksums": [f"{s:016x}" for s in sums], "equal": equal}


def own_stdout():
    """A private handle on this process's stdout for the one JSON line, with fd 1 itself sent to
    stderr for the rest of the run: native libraries print there (RCCL's version banner at
    communicator init), and the line must be the only thing on stdout."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 5),
                    help="BASELINE config: 2 = Pong obj PPO_OBJ (the headline; 4 = 2 per GPU), "
                         "3 = Breakout dqn-pixels NatureCNN, 256 envs, 1 = ppo.py CartPole-v1 "
                         "(4 envs; its CPU leg is the reference's own CPU path), 5 = "
                         "dqn_atari_oc.py SpaceInvaders obj, 1M-row HBM replay (a step = 1000 "
                         "global steps)")
    ap.add_argument("--envs-per-gpu", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-iterations", type=int, default=3)
    ap.add_argument("--no-cpu-blocks", action="store_true",
                    help="skip the per-block CPU timings (GAE, minibatch update, config-3 estimate)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--sync-metrics", dest="lag_metrics", action="store_false",
                    help="read each iteration's metrics with a host sync at its end (default: "
                         "lagged one iteration, trainer.train_iteration(lag=True))")
    ap.add_argument("--no-scaled", action="store_true", help="skip roofline_scaled")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only for the "
                         "N = 2 rehearsal with ranks sharing one GPU)")
    ap.add_argument("--dp-exchange", action="store_true",
                    help="N = 1: run the DP exchange path over a 1-rank group (its structure cost)")
    ap.add_argument("--device-index", type=int, default=None,
                    help="GPU of this rank (default LOCAL_RANK; 0 for the shared-GPU rehearsal)")
    ap.add_argument("--set", action="append", default=[], metavar="FIELD=VALUE",
                    help="override an Args field (experiments; e.g. --set rollout_frame_cache=0)")
    ap.add_argument("--deadline", type=float, default=DEADLINE_S,
                    help="whole-run bound in s: a rank past it (or the self-launch parent, 30 s "
                         "later) ends the run with an error line naming every rank's phase")
    ap.add_argument("--stall", type=float, default=120.0,
                    help="bound in s on one timed iteration (warm-up iterations, which capture "
                         "the graphs: 2.5x; init and rendezvous: 300 s)")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="torch.distributed timeout in s (process-group collectives)")
    ap.add_argument("--rehearse-stall", type=int, default=None, metavar="RANK",
                    help="CPU rehearsal of the fail-fast path (gloo, no GPU): the ranks run "
                         "all-reduce iterations and RANK stops before its second one")
    opt = ap.parse_args()
    if needs_launch(opt.gpus):
        # nothing has touched the GPU yet in this process
        raise SystemExit(launch(sys.argv[1:], opt.gpus, deadline_s=opt.deadline + 30))
    line_out = own_stdout()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    watch = rank_watch(opt, rank, world, line_out)
    try:
        run_rank(opt, rank, world, line_out, watch)
    except BaseException as e:  # noqa: BLE001 -- every failure ends with a line naming its phase
        if isinstance(e, SystemExit) and not e.code:
            raise
        import traceback

        traceback.print_exc()
        watch.fire(f"{type(e).__name__}: {e}",
                   exit_code=e.code if isinstance(e, SystemExit) and isinstance(e.code, int) else 1)
    watch.stop()


def emit_error(rec: dict, rank: int, world: int, line_out):
    """The error line: on rank 0's stdout handle (the bench line's place), else on stderr."""
    line = json.dumps({"metric": None, "value": None, "n_gpus": world, **rec})
    print(line, file=line_out if rank == 0 else sys.stderr, flush=True)


def rank_watch(opt, rank: int, world: int, line_out):
    """This rank's RankWatch: status files in the launcher's directory (or one per master port
    under the driver's own torch.distributed.run launch), the run's deadline, the error line as
    its last word."""
    from oc_cleanrl_amd.watch import RankWatch

    status = os.environ.get("OCPPO_WATCH_DIR") or (
        f"/tmp/ocppo_watch_{os.environ.get('MASTER_PORT', os.getpid())}")
    return RankWatch(rank, world, status, stall_s=opt.stall, deadline_s=opt.deadline,
                     on_fire=lambda rec: emit_error(rec, rank, world, line_out))


def rehearse_stall(opt, rank: int, world: int, line_out, watch):
    """--rehearse-stall R: the fail-fast path on CPU. gloo process group with the bench's
    timeout; iterations of one all-reduce each, every rank naming its phase; rank R stops before
    its second all-reduce, the others wait in it until a watchdog ends the run."""
    from datetime import timedelta

    watch.phase("init", stall_s=300.0)
    dist.init_process_group("gloo", timeout=timedelta(seconds=opt.dist_timeout))
    t = torch.ones(1024)
    for i in range(opt.steps):
        watch.phase(f"timed {i}")
        if rank == opt.rehearse_stall and i == 1:
            while True:  # stuck before its collective: the others wait inside theirs
                time.sleep(1.0)
        watch.phase(f"timed {i} all-reduce")
        dist.all_reduce(t)
    watch.phase("report")
    if rank == 0:
        print(json.dumps({"rehearsal": "no stall", "value": float(t[0])}), file=line_out,
              flush=True)
    dist.destroy_process_group()


DQN_STEPS_PER_BENCH_STEP = 1000


def dqn_roofline(tr) -> dict:
    """The dominant kernels of the config-5 step: the acting Q-trunk (agents.fused_trunk over the
    env's W frame rows: the first two layers in one launch, then one launch per layer), run once
    per global step. At M = W rows every weight is used for 2 W flops, far below the ridge: a
    weight stream, HBM-bound by nature. achieved = the trunk's weight + bias bytes (+ the
    activations) per step / the trunk's launches' device time, timed by replaying exactly those
    launches in a hipGraph (trainer.replay_time_us): warm as the loop runs them (the 8.9 MB of
    weights stay Infinity-Cache resident between steps), and cold after an L3 scrub."""
    import torch.nn as nn

    from oc_cleanrl_amd.agents import fused_trunk
    from oc_cleanrl_amd.trainer import replay_time_us

    net = tr.q.network[:-1]
    x = tr.net_obs

    def trunk():
        with torch.no_grad():
            fused_trunk(net, x)

    warm = replay_time_us(trunk, reps=64, rounds=5)
    cold = replay_time_us(trunk, reps=16, rounds=5, cold=True)
    rows = x.numel() // x.shape[-1]  # encoder rows: every frame of every env's stack
    nbytes = 0
    for m in net:
        if isinstance(m, nn.Flatten):
            rows = x.shape[0]  # decoder rows: one per env
        elif isinstance(m, nn.Linear):
            nbytes += 4 * (m.weight.numel() + m.bias.numel() +
                           rows * (m.in_features + m.out_features))
    return {"kernel": "acting Q-trunk (linear2_rows + linear_rows launches, one step)",
            "bound": "hbm", "achieved": round(nbytes / (cold * 1e-6) / 1e9, 1),
            "achieved_warm": round(nbytes / (warm * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(nbytes / (cold * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": None, "bytes": nbytes, "launch_us_cold": round(cold, 2),
            "launch_us_warm": round(warm, 2), "per": "global step"}


def run_dqn(opt, rank: int, world: int, line_out, watch):
    """BASELINE config 5: the training phase of dqn_atari_oc.py:341-400 on one GPU (obj mode,
    1 env, a 1M-transition HBM replay; acting, env step, store, replay add every global step, a
    batch-32 TD update every 4, the target copy every 1000, as replayed hipGraph chunks). One bench
    step = DQN_STEPS_PER_BENCH_STEP global steps, all past learning_starts. The CPU leg is the
    same loop on CPU torch (oracle/cpu_learner.time_cpu_dqn)."""
    from oc_cleanrl_amd.dqn import DQNArgs, DQNTrainer

    if world != 1:
        raise SystemExit("--config 5 is a one-GPU configuration")
    watch.phase("init", stall_s=300.0)
    dev = torch.device("cuda:0" if opt.device_index is None else f"cuda:{opt.device_index}")
    torch.cuda.set_device(dev)
    envs = opt.envs_per_gpu or 1
    args = DQNArgs(env_id="ALE/SpaceInvaders-v5", obs_mode="obj", num_envs=envs,
                   buffer_size=1_000_000, learning_starts=1000, total_timesteps=10_000_000,
                   save_model=False, cuda_graphs=not opt.no_graphs)
    for kv in opt.set:
        k, v = kv.split("=", 1)
        cur = getattr(args, k)
        setattr(args, k, (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v))
    tr = DQNTrainer(args, dev, log=False)
    K = DQN_STEPS_PER_BENCH_STEP
    watch.phase("warmup", stall_s=600.0)
    tr.steps(args.learning_starts + opt.warmup * K)
    torch.cuda.synchronize(dev)
    watch.phase("timed")
    t0 = time.perf_counter()
    for i in range(opt.steps):
        tr.steps(K)
        watch.beat()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    m = tr.metrics()
    watch.phase("report", stall_s=max(opt.deadline, 600.0))
    roofline = dqn_roofline(tr) if not opt.no_kernel_timing else None
    cpu = None
    if not opt.no_cpu_baseline:
        from oracle.cpu_learner import host_info, time_cpu_dqn, usable_threads

        threads = usable_threads()
        # the same 1M-transition replay as the GPU side (host numpy rows)
        r = time_cpu_dqn(steps=opt.cpu_iterations * 1000, threads=threads, num_envs=envs,
                         buffer_size=args.buffer_size)
        cpu = {"value": round(r["sps"], 1), "unit": "env steps/s", "cores": threads,
               "kind": "port", "updates_per_sec": round(r["updates_per_sec"], 2),
               "sample": f"{r['steps']} global steps of dqn_atari_oc.py:341-400 (QNetworkObj, "
                         f"{envs} env, {args.buffer_size}-transition replay, batch-32 TD update "
                         f"every 4 steps) on CPU torch, {r['seconds']:.1f} s", "host": host_info()}
    steps = opt.steps * K
    line = {
        "metric": "env steps/sec + DQN updates/sec, dqn_atari_oc.py SpaceInvaders-v5 obj, 1 MI355X",
        "value": round(steps * envs / dt, 1), "unit": "env steps/s", "n_gpus": 1,
        "steps": opt.steps, "warmup": opt.warmup, "ms_per_step": round(1e3 * dt / opt.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (device-resident SpaceInvaders-obj env; random-init Q-network)",
        "config": {"workload": "dqn_atari_oc.py SpaceInvaders-v5 obj (BASELINE config 5)",
                   "global_steps_per_step": K, "num_envs": envs, "replay_rows": tr.rb.size,
                   "replay_obs_dtype": str(tr.obs_dtype).replace("torch.", ""),
                   "replay_bytes": tr.rb.obs.numel() * tr.rb.obs.element_size(),
                   "batch_size": args.batch_size, "train_frequency": args.train_frequency,
                   "cuda_graphs": tr._graphable(), "parallelism": "dp1"},
        "updates_per_sec": round(steps / args.train_frequency / dt, 2),
        "us_per_global_step": round(dt / steps * 1e6, 3),
        "td_loss": m["losses/td_loss"],
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), file=line_out, flush=True)


def run_rank(opt, rank: int, world: int, line_out, watch):
    """One rank of the bench (the whole run at N = 1)."""
    if opt.rehearse_stall is not None:
        return rehearse_stall(opt, rank, world, line_out, watch)
    if opt.config == 5:
        return run_dqn(opt, rank, world, line_out, watch)
    from datetime import timedelta

    from oc_cleanrl_amd.args import Args, finalize
    from oc_cleanrl_amd import gemm_table
    from oc_cleanrl_amd.trainer import PPOTrainer

    watch.phase("init", stall_s=300.0)
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != opt.gpus:
        raise SystemExit(f"--gpus {opt.gpus} under a launch of WORLD_SIZE={world}")
    device = torch.device(f"cuda:{local_rank if opt.device_index is None else opt.device_index}")
    torch.cuda.set_device(device)
    timeout = timedelta(seconds=opt.dist_timeout)
    if world > 1:
        if opt.backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
    elif opt.dp_exchange:
        # the data-parallel step structure (per-minibatch graphs around an RCCL all-reduce of the
        # flat gradient buffer, /world folded into Adam) over a 1-rank group: what N > 1 runs,
        # minus the xGMI transfer
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        dist.init_process_group(opt.backend, rank=0, world_size=1, timeout=timeout,
                                **({"device_id": device} if opt.backend == "nccl" else {}))
        opt.set.append("dp_exchange=1")

    if opt.config == 1:
        from oc_cleanrl_amd.ppo import PPO_DEFAULTS

        envs = opt.envs_per_gpu or 4
        args = Args(**{**PPO_DEFAULTS, "num_envs": envs * world, "cuda_graphs": not opt.no_graphs,
                       "save_model": False})
        opt.no_kernel_timing = True
    elif opt.config == 3:
        envs = opt.envs_per_gpu or 256
        # the reference's torch_deterministic=True default: the NatureCNN convolutions run on
        # this package's implicit GEMMs (agents._ConvX6 / _ConvX6U8: no MIOpen, no atomics), so
        # the determinism costs nothing (MIOpen's deterministic solutions are naive kernels:
        # 0.9k env steps/s, profiles/r05/c3_deterministic_miopen.txt)
        args = Args(env_id="ALE/Breakout-v5", obs_mode="dqn", architecture="PPO",
                    num_envs=envs * world, num_steps=128, total_timesteps=10_000_000,
                    cuda_graphs=not opt.no_graphs, save_model=False, torch_deterministic=True)
    else:
        envs = opt.envs_per_gpu or 128
        args = Args(env_id="ALE/Pong-v5", obs_mode="obj", architecture="PPO_OBJ",
                    num_envs=envs * world, num_steps=128, num_features=12,
                    total_timesteps=10_000_000, cuda_graphs=not opt.no_graphs, save_model=False)
    for kv in opt.set:
        k, v = kv.split("=", 1)
        cur = getattr(args, k)
        setattr(args, k, (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v))
    args = finalize(args, world)
    tr = PPOTrainer(args, device, rank, world, kernel_timing=not opt.no_kernel_timing, log=False)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)

    # every iteration's metrics (the reference's per-iteration scalars) are collected inside the
    # timed region; lagged: gathered on the device behind the iteration's work and read by the
    # host one iteration later, the last one flushed before the closing barrier
    for i in range(opt.warmup):
        watch.phase(f"warmup {i}", stall_s=2.5 * opt.stall)
        tr.train_iteration(collect_metrics=True, lag=opt.lag_metrics)
    tr.flush_metrics()
    watch.phase("barrier")
    barrier()
    t0 = time.perf_counter()
    for i in range(opt.steps):
        watch.phase(f"timed {i}")
        tr.train_iteration(collect_metrics=True, lag=opt.lag_metrics)
    tr.flush_metrics()
    watch.phase("barrier")
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    watch.phase("replica check")
    replicas = replica_check(tr, world, device)
    # after the timed region, the kernel timer's replays, the scaled cases and the CPU legs
    watch.phase("report", stall_s=max(opt.deadline, 600.0))

    env_steps = opt.steps * args.num_steps * args.local_num_envs * world
    updates = opt.steps * args.update_epochs * args.num_minibatches
    kb = kernel_bytes(tr) if opt.config != 1 else {}
    kf = kernel_flops(tr) if opt.config != 1 else {}
    kernels = {}
    if not opt.no_kernel_timing:
        # HBM-bound sites (no flops, or below the ridge) are also timed cold
        cold = {n for n in tr.timer.sites
                if not n.startswith("gemm_x6_") and not mfma_bound(kf.get(n), kb.get(n) or 1)}
        for name, us in tr.timer.measure(cold=cold).items():
            n = tr.timer.per_iter.get(name, 0)
            nbytes = kb.get(name) or (relu_bias_grad_bytes(name)
                                      if name.startswith("relu_bias_grad_") else
                                      relu_bias_wgrad_bytes(name)
                                      if name.startswith("relu_bias_wgrad_") else
                                      gemm_x6_bytes(name) if name.startswith("gemm_x6_") else None)
            kernels[name] = {"mean_us": round(us, 3), "launches_per_iter": n,
                             "us_per_iter": round(us * n, 2)}
            if name in tr.timer.cold_us:
                kernels[name]["cold_us"] = round(tr.timer.cold_us[name], 3)
            if nbytes:
                kernels[name].update(bytes=nbytes, GBps=round(nbytes / (us * 1e-6) / 1e9, 2))
                if "cold_us" in kernels[name]:
                    kernels[name]["GBps_cold"] = round(
                        nbytes / (kernels[name]["cold_us"] * 1e-6) / 1e9, 2)
    # one kernel, several launch shapes per minibatch: aggregate them (average bytes per launch
    # over average launch duration = total bytes / total time)
    parts = [k for k in kernels if k.startswith("relu_bias_grad_") and "bytes" in kernels[k]]
    if parts:
        n = sum(kernels[k]["launches_per_iter"] for k in parts)
        t = sum(kernels[k]["us_per_iter"] for k in parts)
        b = sum(kernels[k]["bytes"] * kernels[k]["launches_per_iter"] for k in parts)
        kernels["relu_bias_grad"] = {"mean_us": round(t / n, 3), "launches_per_iter": n,
                                     "us_per_iter": round(t, 2), "bytes": round(b / n),
                                     "GBps": round(b / (t * 1e-6) / 1e9, 2),
                                     "shapes": sorted(k[len("relu_bias_grad_"):] for k in parts)}
        if all("cold_us" in kernels[k] for k in parts):
            tc = sum(kernels[k]["cold_us"] * kernels[k]["launches_per_iter"] for k in parts)
            kernels["relu_bias_grad"].update(cold_us=round(tc / n, 3),
                                             GBps_cold=round(b / (tc * 1e-6) / 1e9, 2))
        for k in parts:
            kernels[k].pop("GBps", None)  # counted in the aggregate
            kernels[k].pop("GBps_cold", None)
    # the update GEMMs on ocppo_gemm_x6: one kernel, a dozen launch shapes per minibatch ->
    # total f32-equivalent flops over total time (the bf16 MFMA work issued is 6x that)
    parts = [k for k in kernels if k.startswith("gemm_x6_") and "bytes" in kernels[k]]
    if parts:
        n = sum(kernels[k]["launches_per_iter"] for k in parts)
        t = sum(kernels[k]["us_per_iter"] for k in parts)
        b = sum(kernels[k]["bytes"] * kernels[k]["launches_per_iter"] for k in parts)
        fl = 0
        for k in parts:
            M, N, K, _, _ = gemm_x6_shape(k)
            fl += 2 * M * N * K * kernels[k]["launches_per_iter"]
        kernels["gemm_x6"] = {"mean_us": round(t / n, 3), "launches_per_iter": n,
                              "us_per_iter": round(t, 2), "bytes": round(b / n),
                              "GBps": round(b / (t * 1e-6) / 1e9, 2),
                              "shapes": sorted(k[len("gemm_x6_"):] for k in parts)}
        kf["gemm_x6"] = fl / n
        for k in parts:
            kernels[k].pop("GBps", None)  # counted in the aggregate
    timed = [k for k in kernels if "GBps" in kernels[k]]
    recs = []
    for name in sorted(timed, key=lambda k: -kernels[k]["us_per_iter"]):
        # the PMC passes replay config 2's launch shapes: no traffic figure for other configs
        traffic, src = pmc_traffic(PMC_KEYS.get(name, "")) if opt.config == 2 else (None, None)
        recs.append(roofline_of(name, kernels[name], kf.get(name), traffic, src))
    # the dominant kernel of this package by device time per iteration; also the dominant
    # HBM-bound one when that is a different kernel
    roofline = recs[0] if recs else None
    roofline_hbm = next((r for r in recs if r["bound"] == "hbm"), None)

    scaled = None
    if rank == 0 and world == 1 and not opt.no_scaled and opt.config == 2:
        from tools.kernel_bench import run_case

        # the north-star kernels the timed path runs (GAE, minibatch prepare = adv-norm stats,
        # the fused heads + loss pair) and the largest HBM streams of the iteration, at streaming
        # sizes, every launch after an L3 scrub (cold)
        scaled = {}
        for name in ("gae", "heads_loss", "mb_prepare", "policy_head", "relu_bias_grad",
                     "frames_scatter_relu"):
            r = run_case(name, "scaled", device, reps=10, rounds=5, cold=True)
            traffic, _ = pmc_traffic(f"{name}_scaled")
            scaled[name] = {"params": r["params"], "mean_us": r["mean_us"], "cache": r["cache"],
                            "bytes": r["bytes"], "achieved": r["GBps"], "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": r["frac"], "traffic": traffic}
            torch.cuda.empty_cache()

    cpu = None
    if rank == 0 and world == 1 and not opt.no_cpu_baseline and opt.config == 1:
        # config 1 is the reference's CPU path: its loop on this host (oracle CartPole dynamics)
        from oracle.cpu_learner import host_info, time_cpu_cartpole

        r = time_cpu_cartpole(iterations=opt.cpu_iterations * 20, threads=1)
        cpu = {"value": round(r["sps"], 1), "unit": "env steps/s", "cores": 1, "kind": "port",
               "updates_per_sec": round(r["updates_per_sec"], 2),
               "sample": f"{r['iterations']} iterations of cleanrl/ppo.py's loop (4 CartPole-v1 "
                         f"envs x 128 steps, 16 minibatch updates of 128) on CPU torch, 1 thread, "
                         f"{r['seconds']:.1f} s",
               "host": host_info()}
    if rank == 0 and world == 1 and not opt.no_cpu_baseline and opt.config == 3:
        # config 3's CPU leg: ONE whole iteration of the oracle's port (256 pixel envs x 128
        # steps of the NatureCNN + 4 x 4 minibatch updates of 8192) on every usable host thread
        # (about 30 s on the box's 16 threads), not an extrapolation
        from oracle.cpu_learner import host_info, time_cpu_baseline, usable_threads

        threads = usable_threads()
        r = time_cpu_baseline(iterations=1, threads=threads, num_envs=256, num_steps=128,
                              n_actions=4, pixels=True)
        cpu = {"value": round(r["sps"], 1), "unit": "env steps/s", "cores": threads,
               "kind": "port", "updates_per_sec": round(r["updates_per_sec"], 3),
               "sample": f"1 PPO iteration of config 3 (256 Breakout-pixel envs x 128 steps, "
                         f"NatureCNN, 16 minibatch updates of 8192) on CPU torch, "
                         f"{r['seconds']:.1f} s",
               "host": host_info()}
    if rank == 0 and world == 1 and not opt.no_cpu_baseline and opt.config == 2:
        # CPU baseline leg (the oracle's port of the reference loop), on every host core this
        # process may use (its CPU affinity capped by the cgroup quota)
        from oracle.cpu_learner import host_info, time_cpu_baseline, time_cpu_blocks, usable_threads

        threads = usable_threads()
        r = time_cpu_baseline(iterations=opt.cpu_iterations, threads=threads, num_envs=128,
                              num_steps=128)
        cpu = {"value": round(r["sps"], 1), "unit": "env steps/s", "cores": threads,
               "kind": "port",
               "updates_per_sec": round(r["updates_per_sec"], 3),
               "sample": f"{opt.cpu_iterations} PPO iterations of config 2 (128 envs x 128 steps, "
                         f"16 minibatch updates of 4096) on CPU torch, {r['seconds']:.1f} s",
               "host": host_info()}
        if not opt.no_cpu_blocks:
            cpu["blocks"] = time_cpu_blocks(threads)

    if rank == 0:
        sps = env_steps / dt
        line = {
            "metric": "env steps/sec (SPS) + PPO updates/sec, ALE/Pong-v5 obj-mode, 1/2/4/8 MI355X"
                      if opt.config == 2 else
                      "env steps/sec (SPS) + PPO updates/sec, ALE/Breakout-v5 dqn pixels, 1 MI355X"
                      if opt.config == 3 else
                      "env steps/sec (SPS) + PPO updates/sec, CartPole-v1 (ppo.py), 1 MI355X",
            "value": round(sps, 1),
            "unit": "env steps/s",
            "n_gpus": world,
            "steps": opt.steps,
            "warmup": opt.warmup,
            "ms_per_step": round(1e3 * dt / opt.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (device-resident Pong-obj env; random-init PPObj)" if opt.config == 2
                    else "synthetic (device-resident 84x84 u8 frames; random-init NatureCNN)"
                    if opt.config == 3 else
                    "device CartPole-v1 env (gymnasium 0.28.1 dynamics restated); random-init agent",
            "config": {"workload": "ppo_atari_oc.py Pong-v5 obj PPO_OBJ (BASELINE config 2 per GPU)"
                       if opt.config == 2 else
                       "ppo_atari_oc.py Breakout-v5 dqn NatureCNN (BASELINE config 3)"
                       if opt.config == 3 else "ppo.py CartPole-v1, 4 envs (BASELINE config 1)",
                       "local_num_envs": args.local_num_envs, "num_envs": args.num_envs,
                       "num_steps": args.num_steps, "num_features": args.num_features,
                       "minibatch_size": args.local_minibatch_size,
                       "update_epochs": args.update_epochs,
                       "num_minibatches": args.num_minibatches,
                       "obs_storage": str(tr.obs_dtype).replace("torch.", ""),
                       "cuda_graphs": args.cuda_graphs,
                       "metrics": ("every iteration, lagged one iteration (device gather + "
                                   "non-blocking copy; the host reads them while the next "
                                   "iteration runs; the last flushed inside the timed region)"
                                   if opt.lag_metrics else "every iteration, host sync at its end"),
                       "torch_deterministic": args.torch_deterministic,
                       "gemm_table": (str(gemm_table.TABLE.relative_to(ROOT))
                                      if tr.gemm_table else None),
                       "update_gemm": ("ocppo_gemm_x6: f32 operands split exactly into three "
                                       "bf16 pieces, six piece products accumulated in f32 on "
                                       "the bf16 matrix cores (error vs f64 at or below "
                                       "hipBLASLt's f32 GEMM, tests/test_gemm_gpu.py); "
                                       "products it does not tile on hipBLASLt f32"
                                       if args.x6_gemm else "hipBLASLt f32"),
                       **({"convolutions": "ocppo_conv_x6 / ocppo_conv_x6_u8: implicit GEMMs "
                           "on the exact three-piece bf16 products (forward with bias + ReLU, "
                           "weight gradient, data gradient; the first layer reads the u8 frame "
                           "stacks through the minibatch indices), deterministic"}
                          if opt.config == 3 else {}),
                       "conv_benchmark": args.conv_benchmark,
                       "sampling_noise": {
                           "kernel": "the reference's stream: Categorical.sample's per-step [N, A] "
                                     "Exp(1) draws on the device generator (torch's Philox "
                                     "exponential_ restated), the rollout's T draws made by one "
                                     "HIP launch at its start; bitwise torch's draws "
                                     "(tests/test_kernels_gpu.py, tests/test_trainer_gpu.py)",
                           "head": "the reference's stream drawn inside each step's sampling "
                                   "kernel",
                           "torch": "the reference's stream from torch's exponential_, one "
                                    "launch per step",
                           "rollout": "one [T, N, A] Exp(1) draw per rollout (not the "
                                      "reference's stream)"}[args.sampling_noise],
                       "parallelism": f"dp{world}",
                       **({"dist_backend": opt.backend} if world > 1 else {}),
                       **({"dp_exchange": tr.dp_form,
                           "dp_overlap": bool(args.dp_overlap)} if tr.dp else {})},
            "replicas": replicas,
            "updates_per_sec": round(updates / dt, 2),
            "roofline": roofline,
            "roofline_hbm": roofline_hbm if roofline_hbm is not roofline else None,
            "rooflines_top": recs[:6],
            "roofline_scaled": scaled,
            "kernels": kernels,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), file=line_out, flush=True)
    tr.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
