#!/usr/bin/env bash
# heads_loss experiments: rows per workgroup sweep, the loss-math probe build, a rocprof split.
# The geometry is compile-time (OCPPO_HL_ROWS / OCPPO_HL_GRID): build the variants on the CPU first,
#   for r in 16 32; do python tools/build_variant.py oc_cleanrl_amd/lib/hl_rows_$r.so -DOCPPO_HL_ROWS=$r; done
#   python tools/build_variant.py oc_cleanrl_amd/lib/probe_loss_32.so -DOCPPO_LOSS_PROBE -DOCPPO_HL_ROWS=32
set -e
cd $GRAFT_REPO_ROOT
for r in 16 32; do
  OCPPO_LIB=$GRAFT_REPO_ROOT/oc_cleanrl_amd/lib/hl_rows_$r.so timeout -k 10 120 python3 tools/kernel_bench.py --kernel heads_loss --size config --reps 20 --rounds 5 > gpurun_out/hl_$r.json 2>/dev/null
done
OCPPO_LIB=$GRAFT_REPO_ROOT/oc_cleanrl_amd/lib/probe_loss_32.so timeout -k 10 120 python3 tools/kernel_bench.py --kernel heads_loss --size config --reps 20 --rounds 5 > gpurun_out/hl_probe_32.json 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hlprof -o hl -- python3 $GRAFT_REPO_ROOT/tools/kernel_bench.py --kernel heads_loss --size config --reps 20 --rounds 5 > /dev/null 2>&1
