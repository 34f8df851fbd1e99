#!/usr/bin/env bash
# End-of-round evidence on the GPU box: rocprofv3 --kernel-trace --stats of the bench command,
# the full GPU parity suite, and the bench lines of configs 2 and 3 (each step time-limited).
#   bash tools/round_close.sh r01f
set -euo pipefail
TAG=$1
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-scaled \
  > "$OUT/bench.log" 2>&1
echo "bench trace done"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
echo "gpu tests done"
timeout -k 10 300 python3 bench.py > gpurun_out/bench_line.json 2> gpurun_out/bench_line.err
timeout -k 10 300 python3 bench.py --config 3 > gpurun_out/bench_line_config3.json 2> gpurun_out/bench_line_config3.err
timeout -k 10 300 python3 bench.py --config 1 > gpurun_out/bench_line_config1.json 2> gpurun_out/bench_line_config1.err
echo "bench lines done"
