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
    # phase split: the rollout runs from the first launch after an iteration's last Adam launch
    # to the GAE launch; the update from the GAE launch to the last Adam launch
    gae = [i for i, r in enumerate(win) if "gae" in r["Kernel_Name"]]
    adam = [i for i, r in enumerate(win) if "adam_kernel" in r["Kernel_Name"]]
    roll, upd, rbusy = [], [], []
    for g in gae:
        prev = [i for i in adam if i < g]
        nxt = [i for i in adam if i > g]
        if not prev or not nxt:
            continue
        lo = prev[-1] + 1
        hi = max(i for i in adam if i < (min(j for j in gae if j > g) if any(j > g for j in gae)
                                          else len(win)))
        roll.append(int(win[g]["Start_Timestamp"]) - int(win[lo]["Start_Timestamp"]))
        rbusy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win[lo:g]))
        upd.append(int(win[hi]["End_Timestamp"]) - int(win[g]["Start_Timestamp"]))
    if roll:
        n = len(roll)
        print(f"phases ({n} whole iterations): rollout {1e-6 * sum(roll) / n:.3f} ms "
              f"({1e-3 * sum(roll) / n / a.T:.2f} us/step, kernel busy "
              f"{1e-3 * sum(rbusy) / n / a.T:.2f} us/step), update {1e-6 * sum(upd) / n:.3f} ms")
    for name, (n, d) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{1e-6 * d / a.iters:8.3f} ms/it {n / a.iters:8.1f} calls/it {1e-3 * d / n:8.2f} us  {name}")


if __name__ == "__main__":
    main()
