#!/usr/bin/env bash
# Round-5 closing profiles: rocprofv3 --kernel-trace --stats of the bench command (the line's
# kernel timer on: its replays included), and clean traces (timer off) of configs 2 and 3
#   bash tools/r05_profiles.sh TAG
set -euo pipefail
TAG=$1
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-scaled \
  > "$OUT/bench.log" 2>&1
rm -f "$OUT"/bench/*kernel_trace.csv
echo "bench stats done"
bash "$R/tools/prof_clean.sh" "$TAG"
echo "clean config 2 done"
bash "$R/tools/prof_c3.sh" "$TAG"
echo "clean config 3 done"
