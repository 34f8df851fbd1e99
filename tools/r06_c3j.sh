#!/bin/bash
# Config 3: the data gradients' tile (ops.CONV_DGRAD_TILE: 0 = the rule's choice, 2 = 128 x 64,
# 3 = 64 x 64), interleaved in the bench
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3j
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  for t in 0 2 3; do
    timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_DGRAD_TILE $t $Q > gpurun_out/c3j/t${t}_$p.json 2> gpurun_out/c3j/t${t}_$p.err
  done
done
