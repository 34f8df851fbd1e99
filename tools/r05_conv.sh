#!/usr/bin/env bash
# Round-5: the NatureCNN convolutions on ocppo_conv_x6 -- kernel tests, the config-3 golden,
# and config-3 bench lines with the reference's torch_deterministic default and without it
#   bash tools/r05_conv.sh [tests|lines|all]
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/conv
what=${1:-all}
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread \
    tests/test_conv_gpu.py tests/test_config3_golden_gpu.py > gpurun_out/conv/tests.log 2>&1
fi
if [ "$what" = lines ] || [ "$what" = all ]; then
  for det in 1 0; do
    timeout -k 10 300 python3 bench.py --config 3 --no-cpu-baseline --no-scaled --steps 10 \
      --set torch_deterministic=$det > gpurun_out/conv/line_det$det.json 2> gpurun_out/conv/line_det$det.err
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/conv/prof -o c3 -- \
    python3 bench.py --config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 5 \
    --set torch_deterministic=1 > gpurun_out/conv/prof.log 2>&1
fi
