#!/usr/bin/env bash
# Round-5: interleaved in-bench A/B of a module-level value (tools/ab_toggle.py), N pairs
#   bash tools/r05_value_ab.sh module.NAME A B N [bench args...]
set -euo pipefail
T=$1; A=$2; B=$3; N=$4; shift 4
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vab
for i in $(seq 1 "$N"); do
  for v in $A $B; do
    timeout -k 10 300 python3 tools/ab_toggle.py "$T" $v --no-cpu-baseline --no-scaled \
      --steps 40 --warmup 5 "$@" > gpurun_out/vab/ab_${v}_$i.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels',{}); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {n: v['us_per_iter'] for n, v in k.items() if 'sum_splits_db' in n or '512x256' in n or '256x512' in n})" gpurun_out/vab/ab_${v}_$i.json "$T" $v
  done
done
