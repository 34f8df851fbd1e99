#!/usr/bin/env bash
# Clean per-kernel summary of the config-5 bench (DQN): rocprofv3 --kernel-trace --stats of
# bench.py --config 5 without the per-kernel timer. Usage: tools/prof_c5.sh TAG
set -euo pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c5_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o b \
  -- python3 $R/bench.py --config 5 --no-cpu-baseline --no-scaled --no-kernel-timing \
  > $OUT/bench.log 2>&1
rm -f $OUT/b_kernel_trace.csv
