#!/usr/bin/env bash
# x6 main-loop variants (experiment): each prebuilt exp_lib/<name>.so timed at the config-2 update
# shapes with the shipped variants (24, 56), one JSON file per build.
#   bash tools/exp_x6_variants.sh OUTDIR name1 name2 ...
set -euo pipefail
OUT=$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  OCPPO_LIB="exp_lib/$v.so" timeout -k 10 240 python3 tools/exp_gemm_x6.py --tiles 24,56 --reps 30 \
    --out "$OUT/$v.jsonl" > "$OUT/$v.log" 2>&1
  tail -1 "$OUT/$v.jsonl"
done
