#!/usr/bin/env bash
# Round-5: config-5 bench A/B of a module switch (tools/ab_toggle.py), N pairs
#   bash tools/r05_dqn_ab.sh module.NAME N
set -euo pipefail
T=$1; N=$2
cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 "$N"); do
  for v in 1 0; do
    timeout -k 10 300 python3 tools/ab_toggle.py "$T" $v --config 5 --no-cpu-baseline \
      --no-kernel-timing --steps 10 --warmup 2 > gpurun_out/dab_$v.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/dab_$v.json "$T" $v
  done
done
