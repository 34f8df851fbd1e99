#!/bin/bash
# Config 3: the rollout's flattened Linear on the HIP f32-MFMA rows kernel (agents.HIP_FLAT_INFER):
# tests, an A/B in the bench, the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3d
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py "tests/test_trainer_gpu.py::test_pixel_natureccn_iteration" "tests/test_trainer_gpu.py::test_rollout_flatten_linear_reads_the_nhwc_activation" > gpurun_out/c3d/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py agents.HIP_FLAT_INFER 1 $Q > gpurun_out/c3d/on_$p.json 2> gpurun_out/c3d/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py agents.HIP_FLAT_INFER 0 $Q > gpurun_out/c3d/off_$p.json 2> gpurun_out/c3d/off_$p.err
done
bash tools/prof_c3.sh r06d > /dev/null 2>&1
