#!/usr/bin/env bash
# Round-5: clean kernel traces of the plain and the DP-exchange (own RCCL, overlap on / off)
# config-2 iterations, then the decoder-dX-planes A/B.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/prof_clean.sh r05plain
head -3 gpurun_out/clean_r05plain/breakdown.txt
bash tools/prof_clean.sh r05dp --dp-exchange
head -3 gpurun_out/clean_r05dp/breakdown.txt
bash tools/prof_clean.sh r05dpnoov --dp-exchange --set dp_overlap=0
head -3 gpurun_out/clean_r05dpnoov/breakdown.txt
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python3 tools/ab_toggle.py frames.DECODE_DX_PLANES $v --no-cpu-baseline \
      --no-scaled --no-kernel-timing --steps 40 --warmup 5 > gpurun_out/ab_ddx_$v.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ddx', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/ab_ddx_$v.json $v
  done
done
