#!/bin/bash
# Config 5: the DQN train step's target forward on a side stream (dqn.TARGET_SIDE_STREAM): tests,
# interleaved A/B in the bench
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c5
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_dqn_gpu.py tests/test_replay_gpu.py > gpurun_out/c5/tests.log 2>&1
Q="--config 5 --no-cpu-baseline --no-scaled --no-kernel-timing"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py dqn.TARGET_SIDE_STREAM 1 $Q > gpurun_out/c5/on_$p.json 2> gpurun_out/c5/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py dqn.TARGET_SIDE_STREAM 0 $Q > gpurun_out/c5/off_$p.json 2> gpurun_out/c5/off_$p.err
done
