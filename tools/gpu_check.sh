#!/usr/bin/env bash
# One GPU-box pass: the GPU parity suite, the config-2 bench line, and the 2-rank DP rehearsal
# (bench.py --gpus 2 starts its own torch.distributed.run child; gloo, both ranks on GPU 0).
#   bash tools/gpu_check.sh TAG [pytest -k expression]
set -euo pipefail
TAG=$1
K=${2:-}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "$K" > "$OUT/gpu_tests.log" 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1
fi
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled > "$OUT/bench_line.json" 2> "$OUT/bench_line.err"
head -c 400 "$OUT/bench_line.json"; echo
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --device-index 0 --steps 5 --warmup 2 \
  --no-kernel-timing > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.err"
head -c 300 "$OUT/bench_gpus2.json"; echo
