#!/usr/bin/env bash
# Round-5: which MIOpen convolution solutions config 3 gets with torch_deterministic=True (the
# reference default), and what they cost: one short bench line + a rocprofv3 stats pass of it
#   bash tools/r05_c3det.sh
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3det
timeout -k 10 400 python3 bench.py --config 3 --no-cpu-baseline --no-scaled --no-kernel-timing \
  --steps 2 --warmup 1 --set torch_deterministic=1 > gpurun_out/c3det/line_det.json 2> gpurun_out/c3det/line_det.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c3det/prof -o c3det -- \
  python3 bench.py --config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 2 --warmup 1 \
  --set torch_deterministic=1 > gpurun_out/c3det/prof.log 2>&1
