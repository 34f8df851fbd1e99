#!/usr/bin/env bash
# Kernel breakdown of the config-5 DQN bench (tools/dqn_bench.py): rocprofv3 --kernel-trace --stats.
#   bash tools/prof_dqn.sh TAG
set -euo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/dqn_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o d \
  -- python3 $R/tools/dqn_bench.py --steps 4000 --warmup 1000 > $OUT/bench.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"]) / 1e6:8.2f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"]) / 1e3:7.2f} us  {r["Name"][:90]}')
PY
rm -f $OUT/*/*kernel_trace.csv $OUT/*kernel_trace.csv 2>/dev/null || true
