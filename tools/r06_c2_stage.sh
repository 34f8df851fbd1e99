#!/bin/bash
# Config 2: the staging copies on a copy stream (trainer.STAGE_ON_SIDE_STREAM): tests, interleaved
# A/B in the bench (40-step lines)
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c2s
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_trainer_gpu.py tests/test_config2_golden_gpu.py tests/test_dp_gpu.py tests/test_frames_gpu.py > gpurun_out/c2s/tests.log 2>&1
Q="--no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5"
for p in 1 2 3; do
  timeout -k 10 300 python3 tools/ab_toggle.py trainer.STAGE_ON_SIDE_STREAM 1 $Q > gpurun_out/c2s/on_$p.json 2> gpurun_out/c2s/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py trainer.STAGE_ON_SIDE_STREAM 0 $Q > gpurun_out/c2s/off_$p.json 2> gpurun_out/c2s/off_$p.err
done
