#!/usr/bin/env bash
# End-of-round evidence pass on one GPU box (run from the repo root via gpurun):
#   the GPU parity suite, the bench lines of configs 2 (default: headline, with the CPU leg and
#   the scaled rooflines), 1 and 3, and the 2-rank self-launch rehearsal; each step time-boxed,
#   chained so that a failure ends the call.
#   bash tools/round_evidence.sh TAG
set -euo pipefail
TAG=${1:-r04}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/evidence_$TAG"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench_line.json" 2> "$OUT/bench_line.err"
head -c 300 "$OUT/bench_line.json"; echo
timeout -k 10 300 python3 bench.py --config 1 > "$OUT/bench_line_config1.json" 2> "$OUT/bench_line_config1.err"
head -c 200 "$OUT/bench_line_config1.json"; echo
timeout -k 10 400 python3 bench.py --config 3 --no-cpu-baseline > "$OUT/bench_line_config3.json" \
  2> "$OUT/bench_line_config3.err"
head -c 200 "$OUT/bench_line_config3.json"; echo
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --device-index 0 --steps 5 --warmup 2 \
  --no-kernel-timing > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.err"
head -c 200 "$OUT/bench_gpus2.json"; echo
