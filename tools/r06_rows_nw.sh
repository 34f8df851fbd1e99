#!/bin/bash
# The rollout convolutions' few-rows kernel (ocppo_conv_x6 tile 7): waves per workgroup 4 / 8 / 16
# (variant builds -DOCPPO_ROWS_NW), with and without the pre-split weight planes, kernel times and
# the config-3 bench in one box session
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rows
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for n in 4 8 16; do
  export OCPPO_LIB=$R/tools/variants/rows_nw$n.so
  timeout -k 10 120 python3 tools/exp_conv_rows.py > gpurun_out/rows/kb_nw$n.json 2> gpurun_out/rows/kb_nw$n.err
  timeout -k 10 300 python3 tools/ab_toggle.py agents.CONV_ROWS_PLANES 1 $Q > gpurun_out/rows/c3_nw${n}_planes.json 2> gpurun_out/rows/c3_nw${n}_planes.err
  timeout -k 10 300 python3 tools/ab_toggle.py agents.CONV_ROWS_PLANES 0 $Q > gpurun_out/rows/c3_nw${n}_noplanes.json 2> gpurun_out/rows/c3_nw${n}_noplanes.err
done
