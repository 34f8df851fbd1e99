"""Compare two rocprofv3 --stats kernel summaries (per-kernel total time per iteration).

    python tools/compare_stats.py A_kernel_stats.csv B_kernel_stats.csv --iters 7
"""
import argparse
import csv


def load(p):
    return {r["Name"]: r for r in csv.DictReader(open(p))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--iters", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    o = ap.parse_args()
    A, B = load(o.a), load(o.b)
    names = set(A) | set(B)
    f = lambda d, n, k: float(d[n][k]) if n in d else 0.0  # noqa: E731
    rows = sorted(names, key=lambda n: -max(f(A, n, "TotalDurationNs"), f(B, n, "TotalDurationNs")))
    ta = sum(f(A, n, "TotalDurationNs") for n in names) / o.iters / 1e3
    tb = sum(f(B, n, "TotalDurationNs") for n in names) / o.iters / 1e3
    print(f"total us/iter  A {ta:9.1f}   B {tb:9.1f}")
    for n in rows[:o.top]:
        print(f"A {f(A, n, 'TotalDurationNs') / o.iters / 1e3:8.1f}us x{f(A, n, 'Calls') / o.iters:6.1f} "
              f"({f(A, n, 'AverageNs') / 1e3:6.2f})  B {f(B, n, 'TotalDurationNs') / o.iters / 1e3:8.1f}us "
              f"x{f(B, n, 'Calls') / o.iters:6.1f} ({f(B, n, 'AverageNs') / 1e3:6.2f})  {n[:90]}")


if __name__ == "__main__":
    main()
