#!/usr/bin/env bash
# rocprofv3 kernel stats of the headline bench + phase timing. Usage: prof_bench.sh TAG [bench args]
set -euo pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pb_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/phase_timing.py > $OUT/phase.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o b \
  -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-scaled "$@" > $OUT/bench.log 2>&1
rm -f $OUT/b_kernel_trace.csv
