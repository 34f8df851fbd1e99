"""Summarise tools/pmc_bench.sh: mean FETCH_SIZE / WRITE_SIZE (KiB) per dispatch of every kernel
of the bench run, and the calibrated HBM traffic per dispatch (FETCH_SIZE x2 for 16-B/lane reads,
MI355X_MICROARCH.md §HBM, + WRITE_SIZE, in bytes). `gemm_x6` aggregates every ocppo::gemm_x6
dispatch (all its launch shapes, as the bench's roofline record does).

    python tools/pmc_bench_summary.py gpurun_out/pmc_bench_r04 > profiles/r04/pmc_bench.json
"""
import csv
import glob
import json
import sys
from collections import defaultdict

csv.field_size_limit(1 << 30)


def load(d, ctr):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/{ctr}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != ctr:
                continue
            name = r["Kernel_Name"]
            vals[name].append(float(r["Counter_Value"]))
    return vals


def short(name):
    s = name.split("(")[0]
    return s.replace("void ", "").strip()


def main():
    d = sys.argv[1]
    fetch, write = load(d, "FETCH_SIZE"), load(d, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes) "
                     "over `bench.py --steps 3 --warmup 2 --no-kernel-timing`",
           "kernels": {}}
    agg = defaultdict(lambda: [0.0, 0.0, 0, 0])
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name, []), write.get(name, [])
        rec = {"dispatches": max(len(f), len(w)),
               "FETCH_SIZE_KiB": sum(f) / len(f) if f else None,
               "WRITE_SIZE_KiB": sum(w) / len(w) if w else None}
        if f and w:
            rec["traffic_bytes"] = round(1024 * (2 * rec["FETCH_SIZE_KiB"] + rec["WRITE_SIZE_KiB"]))
        out["kernels"][short(name)[:120]] = rec
        if "gemm_x6" in name:
            a = agg["gemm_x6"]
            a[0] += sum(f)
            a[1] += sum(w)
            a[2] += len(f)
            a[3] += len(w)
    if "gemm_x6" in agg:
        a = agg["gemm_x6"]
        fk, wk = a[0] / max(a[2], 1), a[1] / max(a[3], 1)
        out["gemm_x6"] = {"dispatches": a[2], "FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk,
                          "traffic_bytes": round(1024 * (2 * fk + wk))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
