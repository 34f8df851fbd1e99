#!/usr/bin/env bash
# Round-5: config-3 lines with the forward tile rule's workgroup threshold (ops.CONV_FWD_MIN_UNITS)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fu
for i in 1 2; do
  for v in 512 256; do
    timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_FWD_MIN_UNITS $v --config 3 --no-cpu-baseline \
      --no-scaled --steps 10 > gpurun_out/fu/u_${v}_$i.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels',{}); print(sys.argv[2], d['value'], d['ms_per_step'], {n: v['mean_us'] for n, v in k.items() if n.startswith('conv_x6_256') or n.startswith('conv_x6_u8_256')})" gpurun_out/fu/u_${v}_$i.json $v
  done
done
