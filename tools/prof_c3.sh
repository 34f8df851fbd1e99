#!/usr/bin/env bash
# Config 3 (Breakout pixels, NatureCNN, 256 envs): bench line + rocprofv3 kernel stats.
set -euo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --config 3 --steps 5 --warmup 2 > $R/gpurun_out/c3_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3prof -o b -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-kernel-timing > $R/gpurun_out/c3prof.log 2>&1
rm -f $R/gpurun_out/c3prof/b_kernel_trace.csv
