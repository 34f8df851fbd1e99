#!/usr/bin/env bash
# Round-5: conv kernel tests (+ the config-3 golden) + one config-3 line at torch_deterministic=1
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/conv
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_conv_gpu.py tests/test_config3_golden_gpu.py "tests/test_trainer_gpu.py::test_pixel_rollout_reads_the_u8_stacks" > gpurun_out/conv/tests_iter.log 2>&1
timeout -k 10 300 python3 bench.py --config 3 --no-cpu-baseline --no-scaled --steps 10 \
  --set torch_deterministic=1 > gpurun_out/conv/line_iter.json 2> gpurun_out/conv/line_iter.err
