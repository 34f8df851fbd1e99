#!/bin/bash
# Config 3: the convolution forwards' ReLU bitmask read by the backward's ReLU pass (agents.CONV_RELU_BITS):
# tests, interleaved A/B in the bench, the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3m
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py tests/test_trainer_gpu.py tests/test_abi.py tests/test_kernels_gpu.py > gpurun_out/c3m/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  for t in agents.CONV_RELU_BITS; do
    timeout -k 10 300 python3 tools/ab_toggle.py $t 1 $Q > gpurun_out/c3m/${t}_on_$p.json 2> gpurun_out/c3m/${t}_on_$p.err
    timeout -k 10 300 python3 tools/ab_toggle.py $t 0 $Q > gpurun_out/c3m/${t}_off_$p.json 2> gpurun_out/c3m/${t}_off_$p.err
  done
done
bash tools/prof_c3.sh r06m > /dev/null 2>&1
