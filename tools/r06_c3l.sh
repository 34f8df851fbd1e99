#!/bin/bash
# Config 3: the conv2 data gradient's pre-split class weights on the 128 x 128 tile (whose
# pre-split instance spills 9 VGPRs) on / off (ops.CONV_DGRAD_PLANES_128), interleaved in the bench
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3l
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2 3; do
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_DGRAD_PLANES_128 1 $Q > gpurun_out/c3l/on_$p.json 2> gpurun_out/c3l/on_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_DGRAD_PLANES_128 0 $Q > gpurun_out/c3l/off_$p.json 2> gpurun_out/c3l/off_$p.err
done
