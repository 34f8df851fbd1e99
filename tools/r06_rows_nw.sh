#!/bin/bash
# The rollout convolutions' few-rows kernel (ocppo_conv_x6 tile 7): 4 (the shipped library) / 8 / 16
# waves per workgroup (variant builds -DOCPPO_ROWS_NW), kernel times and the config-3 bench,
# interleaved in one box session
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rows
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  for n in 4 8 16; do
    if [ $n = 4 ]; then export OCPPO_LIB=$R/oc_cleanrl_amd/lib/libocppo_hip.so; else export OCPPO_LIB=$R/tools/variants/rows_nw$n.so; fi
    [ $p = 1 ] && timeout -k 10 120 python3 tools/exp_conv_rows.py > gpurun_out/rows/kb_nw$n.json 2> gpurun_out/rows/kb_nw$n.err
    timeout -k 10 300 python3 bench.py $Q > gpurun_out/rows/c3_nw${n}_$p.json 2> gpurun_out/rows/c3_nw${n}_$p.err
  done
done
