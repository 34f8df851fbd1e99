#!/usr/bin/env bash
# Full GPU parity suite + DQN config-5 line + headline bench line, each step time-limited.
set -euo pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python3 tools/dqn_bench.py > gpurun_out/dqn_bench.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1
