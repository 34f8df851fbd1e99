#!/bin/bash
# Config 3: the first layer's ReLU backward + bias gradient inside the image-staged weight gradient
# (agents.U8_WGRAD_RELU): tests, an A/B in the bench, the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3c
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py "tests/test_trainer_gpu.py::test_pixel_natureccn_iteration" > gpurun_out/c3c/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py agents.U8_WGRAD_RELU 1 $Q > gpurun_out/c3c/on_$p.json 2> gpurun_out/c3c/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py agents.U8_WGRAD_RELU 0 $Q > gpurun_out/c3c/off_$p.json 2> gpurun_out/c3c/off_$p.err
done
bash tools/prof_c3.sh r06c > /dev/null 2>&1
