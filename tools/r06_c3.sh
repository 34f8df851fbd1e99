#!/bin/bash
# Config 3 with the image-staged first convolution: its tests, an A/B of ops.CONV_U8_IMG in the
# bench (no CPU leg: timed separately), the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py "tests/test_trainer_gpu.py::test_pixel_natureccn_iteration" "tests/test_trainer_gpu.py::test_pixel_rollout_reads_the_u8_stacks" > gpurun_out/c3/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_U8_IMG 1 $Q > gpurun_out/c3/on_$p.json 2> gpurun_out/c3/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_U8_IMG 0 $Q > gpurun_out/c3/off_$p.json 2> gpurun_out/c3/off_$p.err
done
bash tools/prof_c3.sh r06a > /dev/null 2>&1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider "tests/test_trainer_gpu.py::test_rollout_flatten_linear_reads_the_nhwc_activation" > gpurun_out/c3/tests2.log 2>&1
