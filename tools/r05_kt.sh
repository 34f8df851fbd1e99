#!/usr/bin/env bash
# Round-5: config-2 bench with in-graph kernel timing, N runs; prints the value and the named
# kernels' in-situ mean durations
#   bash tools/r05_kt.sh N kernel[,kernel...] [bench args...]
set -euo pipefail
N=$1; K=$2; shift 2
cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled --steps 20 "$@" \
    > gpurun_out/kt_$i.json 2> gpurun_out/kt_$i.err
  python3 - gpurun_out/kt_$i.json "$K" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("kernels", {})
print(d["value"], d["ms_per_step"], {k: ks.get(k, {}).get("mean_us") for k in sys.argv[2].split(",")})
PY
done
