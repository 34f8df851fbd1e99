#!/usr/bin/env bash
# Clean per-kernel breakdown of the headline bench: rocprofv3 --kernel-trace --stats of bench.py
# with the per-kernel timer (and its replays) off. Usage: tools/prof_clean.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/clean_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o b \
  -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-scaled --no-kernel-timing \
  "$@" > $OUT/bench.log 2>&1
python3 $R/tools/trace_breakdown.py $OUT > $OUT/breakdown.txt
rm -f $OUT/b_kernel_trace.csv
