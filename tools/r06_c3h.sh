#!/bin/bash
# Config 3: A/B of agents.CONV_ROWS_PLANES (the rollout convolutions' weight planes) in the bench
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3h
Q="--config 3 --no-cpu-baseline --no-scaled --no-kernel-timing --steps 10 --warmup 3"
for p in 1 2; do
  timeout -k 10 300 python3 tools/ab_toggle.py agents.CONV_ROWS_PLANES 0 $Q > gpurun_out/c3h/off_$p.json 2> gpurun_out/c3h/off_$p.err
  timeout -k 10 300 python3 tools/ab_toggle.py agents.CONV_ROWS_PLANES 1 $Q > gpurun_out/c3h/on_$p.json 2> gpurun_out/c3h/on_$p.err
done
