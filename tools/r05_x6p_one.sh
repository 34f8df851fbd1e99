#!/usr/bin/env bash
# Round-5 gemm_x6 probe timing on a few config-2 shapes for each library build
#   bash tools/r05_x6p_one.sh TILES LIB...   (LIB "-" = the in-tree build)
set -euo pipefail
TILES=$1; shift
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  if [ "$lib" = "-" ]; then name=product; unset OCPPO_LIB; else export OCPPO_LIB=$PWD/$lib; fi
  for shp in dx,4096,512,2048 fwd,11520,1024,512 fwd,11520,512,1024; do
    timeout -k 10 200 python3 tools/exp_gemm_x6.py --tiles "$TILES" --reps 20 --only $shp \
      > gpurun_out/x6p_one.log 2>&1
    python3 - "$name" <<'PY'
import json, sys
for ln in open("gpurun_out/x6p_one.log"):
    if not ln.startswith("{"):
        continue
    r = json.loads(ln)
    if r["kind"] != "total":
        print(sys.argv[1], r["kind"], r["M"], r["N"], r["K"], " ".join(f"{t}:{v[0]}" for t, v in r["ours"].items()))
PY
  done
done
