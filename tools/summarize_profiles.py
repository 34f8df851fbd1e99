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
from tools.kernel_bench import SIZES, make_case  # noqa: E402,F401

KERNEL_SUBSTR = {
    "policy_head": "policy_head_fast_kernel",
    "gae": "ocppo::gae",  # gae_kernel (LDS) / gae_stream_kernel by width
    "ppo_loss_prepared": "ocppo::ppo_loss",  # _small / _vec / tile forms by size
    "rollout_store": "rollout_store_kernel",
    "gather": "gather_rows_kernel",
    "relu_bias_grad": "relu_bias_grad_kernel",
    "relu_bias_wgrad": "relu_bias_wgrad_kernel",
    "heads_bwd": "heads_bwd_kernel",
}


def algorithmic_bytes(name, size):
    """Algorithmic bytes per launch: the kernel_bench formulas (needs no GPU for these)."""
    p = SIZES[name][size]
    if name == "gae":
        return 20 * p["T"] * p["N"] + 8 * p["N"]
    if name == "ppo_loss_prepared":
        return (8 * p["A"] + 32) * p["M"]
    if name == "policy_head":
        return p["N"] * (4 * p["H"] + 4 * p["A"] + 16) + 4 * (p["A"] + 1) * (p["H"] + 1)
    if name == "rollout_store":
        return p["N"] * ((p["W"] - 1) * p["D"] * 2 + p["D"] * 4 + p["W"] * p["D"] * 6 + 16)
    if name == "gather":
        return p["M"] * (8 + p["R"] * 6)
    if name == "relu_bias_grad":  # average over the launch mix
        return sum(R * N * 12 + 4 * N for R, N in p["shapes"]) / len(p["shapes"])
    if name == "heads_bwd":
        M, H, A = p["M"], p["H"], p["A"]
        return M * H * 8 + M * (A + 1) * 4 + 2 * (A + 1) * H * 4 + H * 4 + (A + 1) * 4
    if name == "relu_bias_wgrad":
        return p["R"] * p["N"] * 8 + p["R"] * p["K"] * 4 + p["N"] * (p["K"] + 1) * 4
    return None


def mean_counter(path: Path, substr: str):
    vals = []
    for row in csv.DictReader(open(path)):
        if substr in row["Kernel_Name"]:
            vals.append(float(row["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


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
