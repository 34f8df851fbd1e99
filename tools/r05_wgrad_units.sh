#!/usr/bin/env bash
# Round-5: config-3 lines with the convolution weight gradients' split target (ops.CONV_WGRAD_UNITS)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wu
for i in 1 2; do
  for v in 2048 1024 4096; do
    timeout -k 10 300 python3 tools/ab_toggle.py ops.CONV_WGRAD_UNITS $v --config 3 --no-cpu-baseline \
      --no-scaled --steps 10 > gpurun_out/wu/u_${v}_$i.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels',{}); print(sys.argv[2], d['value'], d['ms_per_step'], {n: v['mean_us'] for n, v in k.items() if 'wgrad' in n})" gpurun_out/wu/u_${v}_$i.json $v
  done
done
