#!/bin/bash
# Config 3: the conv1 weight copy cached per rollout, the data gradients' flipped weights by one gather,
# and the fused heads-loss for the NatureCNN trunk (A/B of trainer.FUSED_HEADS_LOSS_ANY_TRUNK)
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3e
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py tests/test_config3_golden_gpu.py tests/test_trainer_gpu.py > gpurun_out/c3e/tests.log 2>&1
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py trainer.FUSED_HEADS_LOSS_ANY_TRUNK 1 $Q > gpurun_out/c3e/on_$p.json 2> gpurun_out/c3e/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py trainer.FUSED_HEADS_LOSS_ANY_TRUNK 0 $Q > gpurun_out/c3e/off_$p.json 2> gpurun_out/c3e/off_$p.err
done
bash tools/prof_c3.sh r06e > /dev/null 2>&1
