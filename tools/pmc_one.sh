#!/usr/bin/env bash
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs, --kernel-trace only) of ONE
# kernel_bench case, into gpurun_out/prof_<tag>/ like tools/profile_round.sh:
#   bash tools/pmc_one.sh relu_bias_wgrad config r01f
set -euo pipefail
K=$1; S=$2; TAG=$3
REPO="$GRAFT_REPO_ROOT"
OUT="$REPO/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc "$ctr" --kernel-trace --output-format csv \
    -d "$OUT/pmc_${K}_${S}_${ctr}" -o pmc \
    -- python3 "$REPO/tools/kernel_bench.py" --kernel "$K" --size "$S" --reps 5 --rounds 1 \
    > "$OUT/pmc_${K}_${S}_${ctr}.log" 2>&1
done
echo "pmc $K $S done"
