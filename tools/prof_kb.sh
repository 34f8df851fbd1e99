#!/usr/bin/env bash
# Per-kernel device durations (rocprofv3 --kernel-trace --stats) of kernel_bench cases, one run
# per case, into gpurun_out/kb_<tag>/; prints each case's kernel averages.
#   bash tools/prof_kb.sh TAG "heads_loss config" "gae config" ...
set -euo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/kb_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for case in "$@"; do
  set -- $case
  d="$OUT/${1}_${2}"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k \
    -- python3 "$R/tools/kernel_bench.py" --kernel "$1" --size "$2" --reps 20 --rounds 5 \
    > "$d.log" 2>&1
  python3 - "$d" "$1 $2" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/k_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    if int(r["Calls"]) >= 20:
        print(f"{sys.argv[2]:24s} {float(r['AverageNs']) / 1e3:8.2f} us  x{r['Calls']:>5s}  {r['Name'][:90]}")
PY
  rm -f "$d"/*/*kernel_trace.csv "$d"/*kernel_trace.csv 2>/dev/null || true
done
