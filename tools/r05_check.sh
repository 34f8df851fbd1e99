#!/usr/bin/env bash
# Round-5 GPU check: a pytest subset (-k PATTERN, or "all" for the whole GPU suite), then the
# config-2 bench in the listed forms (each a `name:args` pair), every step time-boxed.
#   bash tools/r05_check.sh TAG "pytest -k pattern" [name:"bench args" ...]
set -euo pipefail
TAG=$1; PAT=$2; shift 2
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/check_$TAG
mkdir -p "$OUT"
if [ "$PAT" != "none" ]; then
  K=(); [ "$PAT" != "all" ] && K=(-k "$PAT")
  timeout -k 10 900 python3 -u -m pytest tests -m gpu "${K[@]}" -x -q --timeout 300 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing \
    --steps 40 --warmup 5 $args > "$OUT/$name.json" 2> "$OUT/$name.err" || {
      echo "$name failed"; tail -20 "$OUT/$name.err"; tail -2 "$OUT/$name.json"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
    "$OUT/$name.json" "$name"
done
