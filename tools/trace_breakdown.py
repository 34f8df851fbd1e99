"""Per-iteration kernel-time breakdown of a rocprofv3 --kernel-trace of bench.py: only the
dispatches inside the last `--iters` iterations are counted (found from the policy-head launch
count: T per iteration), so warm-up, capture and eager iterations are excluded.

    python tools/trace_breakdown.py <dir with *_kernel_trace.csv> [--iters 10] [--T 128]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--marker", default="policy_head")
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    first = marks[-a.iters * a.T]  # first rollout step of the timed window
    win = rows[first:]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    per = defaultdict(lambda: [0, 0])
    for r in win:
        name = r["Kernel_Name"]
        name = name if len(name) < 70 else name[:67] + "..."
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[name][0] += 1
        per[name][1] += d
    busy = sum(v[1] for v in per.values())
    print(f"window: {a.iters} iterations, wall {1e-6 * (t1 - t0) / a.iters:.3f} ms/iter, "
          f"kernel busy {1e-6 * busy / a.iters:.3f} ms/iter")
    for name, (n, d) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{1e-6 * d / a.iters:8.3f} ms/it {n / a.iters:8.1f} calls/it {1e-3 * d / n:8.2f} us  {name}")


if __name__ == "__main__":
    main()
