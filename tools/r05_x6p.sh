#!/usr/bin/env bash
# Round-5 gemm_x6 variant timing: exp_gemm_x6 over the config-2 shapes for each library build
#   bash tools/r05_x6p.sh TAG TILES LIB...   (LIB "-" = the in-tree build)
set -euo pipefail
TAG=$1; TILES=$2; shift 2
cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  if [ "$lib" = "-" ]; then name=product; unset OCPPO_LIB; else export OCPPO_LIB=$PWD/$lib; fi
  timeout -k 10 400 python3 tools/exp_gemm_x6.py --tiles "$TILES" --reps 20 \
    --out gpurun_out/x6p_${TAG}_$name.jsonl > gpurun_out/x6p_${TAG}_$name.log 2>&1
  python3 - gpurun_out/x6p_${TAG}_$name.jsonl "$name" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    r = json.loads(ln)
    if r["kind"] == "total":
        continue
    print(sys.argv[2], r["kind"], r["M"], r["N"], r["K"], " ".join(f"{t}:{v[0]}" for t, v in r["ours"].items()))
PY
done
