#!/bin/bash
# Config 2: re-check of the tuning flags measured in earlier rounds, at this round's tree: each
# flipped against the default, interleaved with default runs, 40-step lines
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c2f
Q="--no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5"
for p in 1 2; do
  timeout -k 10 200 python3 bench.py $Q > gpurun_out/c2f/default_$p.json 2> gpurun_out/c2f/default_$p.err
  for t in agents.X6_PIPE=0 agents.X6_FWD_SPLITK=0 frames.DECODE_DX_PLANES=1 trainer.ADAM_WRITES_PLANES=1 agents.DEFER_WGRAD_AFTER_FIRST_LAYER=0 frames.FUSED_INDEX_IN_GATHER=0; do
    timeout -k 10 200 python3 tools/ab_toggle.py ${t%=*} ${t#*=} $Q > gpurun_out/c2f/${t%=*}_$p.json 2> gpurun_out/c2f/${t%=*}_$p.err
  done
done
