"""Summarise a tools/profile_round.sh capture into profiles/<tag>/:
  bench_kernel_stats.csv  (rocprofv3 --kernel-trace --stats of the bench command, as written)
  pmc_summary.json        (mean FETCH_SIZE / WRITE_SIZE per dispatch of each case's kernel)

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch. On gfx950 FETCH_SIZE counts half the
bytes of 16-B/lane coalesced streaming reads (MI355X_MICROARCH.md §HBM), so `fetch_bytes_x2` is
the calibrated read figure for such reads; WRITE_SIZE is exact for 16-B/lane streaming stores.

    python tools/summarize_profiles.py gpurun_out/prof_r01b profiles/r01b
"""
import csv
import json
import shutil
import sys
from pathlib import Path

csv.field_size_limit(1 << 30)
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from tools.kernel_bench import SIZES  # noqa: E402

from tools.kernel_bench import case_bytes  # noqa: E402

# kernels of each case (name substrings); a case's counters are summed over them per launch
KERNEL_SUBSTR = {
    "policy_head": ("policy_head_fast_kernel",),
    "gae": ("ocppo::gae",),  # gae_kernel (LDS) / gae_stream_kernel by width
    "ppo_loss_prepared": ("ocppo::ppo_loss",),  # _small / _vec / tile forms by size
    "rollout_store": ("rollout_store_kernel",),
    "gather": ("gather_rows_kernel",),
    "gather_pixels": ("gather_rows_cl4_u8_kernel",),
    "relu_bias_grad": ("relu_bias_grad_kernel",),
    "relu_bias_grad_tail": ("relu_bias_grad_kernel",),
    "relu_bias_wgrad": ("relu_bias_wgrad_rows_kernel", "relu_bias_wgrad_finish_kernel"),
    "heads_bwd": ("heads_bwd_kernel",),
    "heads_loss": ("heads_loss_kernel", "heads_loss_finish_kernel"),
    # the records form (minibatch_prepare_rec_kernel; at >= 2^20 samples + its stats launch)
    "mb_prepare": ("minibatch_prepare", "adv_stats_kernel"),
    "mb_prepare_soa": ("minibatch_prepare_kernel",),
    "gae_plain": ("ocppo::gae",),
    "cache_linear": ("linear_rows_kernel",),
    "store_encode": ("store_linear2_kernel",),
    "decoder": ("linear_rows_kernel",),
    "encoder_mid": ("linear_rows_kernel",),
    "gemm_x6": ("gemm_x6_kernel",),
    "frames_scatter_relu": ("frames_scatter_relu_kernel",),
    "frames_scatter_relu_f32": ("frames_scatter_relu_kernel",),
}


def algorithmic_bytes(name, size):
    """Algorithmic bytes per launch: kernel_bench's formulas (needs no GPU); a multi-shape case
    (relu_bias_grad) is averaged over its launch mix like kernel_bench's per-launch figures."""
    p = SIZES[name][size]
    return case_bytes(name, p) / len(p.get("shapes", (None,)))


def mean_counter(path: Path, substrs):
    """Per-launch counter: the mean over dispatches of each kernel, summed over the kernels."""
    rows = list(csv.DictReader(open(path)))
    total, n = 0.0, []
    for sub in substrs:  # a kernel a case does not launch at this size adds nothing
        vals = [float(r["Counter_Value"]) for r in rows if sub in r["Kernel_Name"]]
        if vals:
            total += sum(vals) / len(vals)
        n.append(len(vals))
    return (total if any(n) else None), n


def main(src, dst):
    src, dst = Path(src), Path(dst)
    dst.mkdir(parents=True, exist_ok=True)
    stats = next((src / "bench").glob("*kernel_stats.csv"), None)
    if stats:
        shutil.copy(stats, dst / "bench_kernel_stats.csv")
    out = {"note": __doc__.strip().splitlines()[4].strip() + " " +
           __doc__.strip().splitlines()[5].strip(), "kernels": {}}
    for d in sorted(src.glob("pmc_*_FETCH_SIZE")):
        tag = d.name[len("pmc_"):-len("_FETCH_SIZE")]
        name, size = tag.rsplit("_", 1)
        sub = KERNEL_SUBSTR[name]
        f, nf = mean_counter(next(d.glob("*counter_collection.csv")), sub)
        wdir = src / f"pmc_{tag}_WRITE_SIZE"
        w, nw = mean_counter(next(wdir.glob("*counter_collection.csv")), sub)
        alg = algorithmic_bytes(name, size)
        rec = {"kernel_match": sub, "params": SIZES[name][size], "dispatches": [nf, nw],
               "FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w,
               "fetch_bytes_x2": round(2 * 1024 * f) if f is not None else None,
               "write_bytes": round(1024 * w) if w is not None else None,
               "algorithmic_bytes": alg}
        if f is not None and w is not None and alg:
            rec["traffic_bytes"] = rec["fetch_bytes_x2"] + rec["write_bytes"]
            rec["traffic_over_algorithmic"] = round(rec["traffic_bytes"] / alg, 3)
        out["kernels"][tag] = rec
    json.dump(out, open(dst / "pmc_summary.json", "w"), indent=1)
    for k, v in out["kernels"].items():
        print(k, v.get("traffic_bytes"), v["algorithmic_bytes"], v.get("traffic_over_algorithmic"))


if __name__ == "__main__":
    main(*sys.argv[1:3])
