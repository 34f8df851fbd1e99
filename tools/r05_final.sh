#!/usr/bin/env bash
# Round-5 final evidence: full GPU suite, then bench lines of configs 2 / 3 (+ 1, 5) and a rocprof
# stats pass of the config-3 line
#   bash tools/r05_final.sh tests|lines|c3prof
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
case "$1" in
  tests)
    timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/final/gpu_tests.log 2>&1 ;;
  lines)
    timeout -k 10 300 python3 bench.py > gpurun_out/final/bench_line.json 2> gpurun_out/final/bench_line.err
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled --steps 40 > gpurun_out/final/plain_1.json 2>/dev/null
    timeout -k 10 300 python3 bench.py --config 3 > gpurun_out/final/bench_line_config3.json 2> gpurun_out/final/c3.err ;;
  c3prof)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/c3prof -o c3 -- \
      python3 bench.py --config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 5 \
      > gpurun_out/final/c3prof.log 2>&1 ;;
esac
