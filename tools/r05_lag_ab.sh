#!/usr/bin/env bash
# Round-5: the lagged-metrics test, then default bench lines with lagged vs synchronous metrics,
# interleaved (three pairs)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lag
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_trainer_gpu.py -k "lagged or metrics" > gpurun_out/lag/test.log 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled > gpurun_out/lag/lag_$i.json 2>/dev/null
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled --sync-metrics > gpurun_out/lag/sync_$i.json 2>/dev/null
done
