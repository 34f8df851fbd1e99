#!/bin/bash
# Config 3: the image-staged first-layer weight gradient (ocppo_conv_x6_u8 tile 8): tests, an A/B
# of ops.CONV_U8_IMG_WGRAD in the bench, the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3b
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py "tests/test_trainer_gpu.py::test_pixel_natureccn_iteration" > gpurun_out/c3b/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_U8_IMG_WGRAD 1 $Q > gpurun_out/c3b/on_$p.json 2> gpurun_out/c3b/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_U8_IMG_WGRAD 0 $Q > gpurun_out/c3b/off_$p.json 2> gpurun_out/c3b/off_$p.err
done
bash tools/prof_c3.sh r06b > /dev/null 2>&1
