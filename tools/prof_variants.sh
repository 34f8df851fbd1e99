#!/usr/bin/env bash
# rocprofv3 kernel durations of one kernel_bench case for several library variants:
#   bash tools/prof_variants.sh TAG KERNEL SIZE lib1.so lib2.so ...   ("-" = the product library)
set -euo pipefail
TAG=$1; K=$2; S=$3; shift 3
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pv_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  name=$(basename "$lib" .so)
  d="$OUT/$name"
  if [ "$lib" = "-" ]; then unset OCPPO_LIB; name=product; d="$OUT/product"; else export OCPPO_LIB="$R/$lib"; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k \
    -- python3 "$R/tools/kernel_bench.py" --kernel "$K" --size "$S" --reps 20 --rounds 5 > "$d.log" 2>&1
  python3 - "$d" "$name" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/k_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if int(r["Calls"]) >= 20:
        print(f"{sys.argv[2]:20s} {float(r['AverageNs']) / 1e3:8.2f} us  {r['Name'][:80]}")
PY
  rm -f "$d"/*/*kernel_trace.csv 2>/dev/null || true
done
