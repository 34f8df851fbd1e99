#!/usr/bin/env bash
# Round-5: interleaved in-bench A/B of a module-level switch (tools/ab_toggle.py), N pairs
#   bash tools/r05_toggle_ab.sh module.NAME N [bench args...]
set -euo pipefail
T=$1; N=$2; shift 2
cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 "$N"); do
  for v in 1 0; do
    timeout -k 10 300 python3 tools/ab_toggle.py "$T" $v --no-cpu-baseline --no-scaled \
      --no-kernel-timing --steps 40 --warmup 5 "$@" > gpurun_out/ab_$v.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/ab_$v.json "$T" $v
  done
done
