#!/usr/bin/env bash
# A/B helper on the GPU box: focused GPU tests (pytest -k PATTERN), then the config-2 bench N
# times (kernel timings of the matching kernels printed), then the clean rocprof breakdown.
#   bash tools/ab_bench.sh TAG "pytest -k pattern" N
set -euo pipefail
TAG=$1; PAT=$2; N=${3:-2}
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "$PAT" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/ab_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ab_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/ab_tests_$TAG.log
for i in $(seq 1 "$N"); do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-scaled > gpurun_out/ab_${TAG}_${i}.json 2>/dev/null
  python3 - "gpurun_out/ab_${TAG}_${i}.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["ms_per_step"])
PY
done
bash tools/prof_clean.sh "$TAG"
head -32 "gpurun_out/clean_$TAG/breakdown.txt"
