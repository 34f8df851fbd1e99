#!/usr/bin/env bash
# Round-5: frame-scatter shape variants (tools/variants/sc_F_G.so: F frames per workgroup, G frame
# groups) against the in-tree build, kernel_bench warm + cold
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for lib in oc_cleanrl_amd/lib/libocppo_hip.so tools/variants/sc_*.so; do
  for c in "" --cold; do
    OCPPO_LIB=$lib timeout -k 10 240 python3 tools/kernel_bench.py --kernel frames_scatter_relu $c \
      | python3 -c "import sys,json; [print(sys.argv[1], d['size'], d['cache'], d['mean_us'], d['frac']) for d in map(json.loads, sys.stdin)]" "$lib"
  done
done
