#!/bin/bash
# Config 3: the last convolution's ReLU backward + bias gradient in the flattened Linear's dX epilogue
# (agents.CONV_RELU_IN_FLAT_DX): tests, interleaved A/B in the bench, the clean trace
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3i
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py tests/test_trainer_gpu.py > gpurun_out/c3i/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  for t in agents.CONV_RELU_IN_FLAT_DX; do
    timeout -k 10 300 python3 tools/ab_toggle.py $t 1 $Q > gpurun_out/c3i/${t}_on_$p.json 2> gpurun_out/c3i/${t}_on_$p.err
    timeout -k 10 300 python3 tools/ab_toggle.py $t 0 $Q > gpurun_out/c3i/${t}_off_$p.json 2> gpurun_out/c3i/${t}_off_$p.err
  done
done
bash tools/prof_c3.sh r06i > /dev/null 2>&1
