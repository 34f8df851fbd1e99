#!/usr/bin/env bash
# heads_loss experiments: rows per workgroup sweep, the loss-math probe build, a rocprof split.
set -e
cd $GRAFT_REPO_ROOT
for r in 16 32; do
  OCPPO_HL_ROWS=$r timeout -k 10 120 python3 tools/kernel_bench.py --kernel heads_loss --size config --reps 20 --rounds 5 > gpurun_out/hl_$r.json 2>/dev/null
  OCPPO_LIB=$GRAFT_REPO_ROOT/oc_cleanrl_amd/lib/probe_loss.so OCPPO_HL_ROWS=$r timeout -k 10 120 python3 tools/kernel_bench.py --kernel heads_loss --size config --reps 20 --rounds 5 > gpurun_out/hl_probe_$r.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
OCPPO_HL_ROWS=16 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hlprof -o hl -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --kernel heads_loss --size config --reps 20 --rounds 5 > /dev/null 2>&1
