#!/usr/bin/env bash
# Clean per-kernel breakdown of the config-3 bench (NatureCNN pixels): rocprofv3 --kernel-trace
# of bench.py --config 3 without the per-kernel timer. Usage: tools/prof_c3.sh TAG
set -euo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c3_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o b \
  -- python3 $R/bench.py --config 3 --steps 4 --warmup 2 --no-cpu-baseline --no-scaled \
  --no-kernel-timing > $OUT/bench.log 2>&1
python3 $R/tools/trace_breakdown.py $OUT --iters 3 > $OUT/breakdown.txt
rm -f $OUT/b_kernel_trace.csv
