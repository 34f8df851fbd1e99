#!/bin/bash
# Config 3: the rollout's 64-channel convolutions on ocppo_conv_x6 tile 7 (K steps split over the
# waves of a workgroup): tests, A/B of ops.CONV_FWD_ROWS, the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3f
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py tests/test_trainer_gpu.py tests/test_abi.py > gpurun_out/c3f/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_FWD_ROWS 1 $Q > gpurun_out/c3f/on_$p.json 2> gpurun_out/c3f/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_FWD_ROWS 0 $Q > gpurun_out/c3f/off_$p.json 2> gpurun_out/c3f/off_$p.err
done
bash tools/prof_c3.sh r06f > /dev/null 2>&1
