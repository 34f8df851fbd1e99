#!/usr/bin/env bash
# Config-2 bench with PyTorch TunableOp restricted to hipBLASLt solutions: pass 1 tunes every GEMM
# shape during the eager warm-up and writes the table, pass 2 only reads it (no tuning).
#   bash tools/tunable_bench.sh
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_hl.csv
S=$(date +%s)
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-scaled \
  --no-kernel-timing > gpurun_out/tun1.json 2> gpurun_out/tun1.err
echo "pass 1 (tuning) wall $(( $(date +%s) - S )) s"; ls gpurun_out/ | grep -i tunable || true
python3 -c "import json; d=json.load(open('gpurun_out/tun1.json')); print(d['value'], d['ms_per_step'])"
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled \
  --no-kernel-timing > gpurun_out/tun2.json 2> gpurun_out/tun2.err
python3 -c "import json; d=json.load(open('gpurun_out/tun2.json')); print(d['value'], d['ms_per_step'])"
unset PYTORCH_TUNABLEOP_ENABLED
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing \
  > gpurun_out/tun0.json 2>/dev/null
python3 -c "import json; d=json.load(open('gpurun_out/tun0.json')); print('default', d['value'], d['ms_per_step'])"
