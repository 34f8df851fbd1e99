#!/usr/bin/env bash
# Round profile capture on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the bench command (per-kernel durations)
#   2. PMC passes (FETCH_SIZE, WRITE_SIZE separately, --kernel-trace only) of the north-star
#      kernels at config and scaled sizes, one kernel_bench case per run, every launch after an
#      L3 scrub (--cold: the scrub's own reduction kernel is filtered out by kernel name).
# Outputs under gpurun_out/prof_<tag>/; copy the summaries into profiles/ afterwards.
set -euo pipefail
TAG=${1:-r03}
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
REPO="$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench \
  -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-scaled \
  > "$OUT/bench.log" 2>&1
echo "bench trace done"
for case in "gae config" "gae scaled" "heads_loss config" "heads_loss scaled" \
            "mb_prepare config" "mb_prepare scaled" "policy_head config" "policy_head scaled" \
            "relu_bias_grad config" "relu_bias_grad scaled" "relu_bias_wgrad config" \
            "cache_linear config" "store_encode config" "decoder config" "encoder_mid config" \
            "frames_scatter_relu config" "frames_scatter_relu scaled"; do
  set -- $case
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc "$ctr" --kernel-trace --output-format csv \
      -d "$OUT/pmc_${1}_${2}_${ctr}" -o pmc \
      -- python3 "$REPO/tools/kernel_bench.py" --kernel "$1" --size "$2" --reps 5 --rounds 1 --cold \
      > "$OUT/pmc_${1}_${2}_${ctr}.log" 2>&1
  done
  echo "pmc $1 $2 done"
done
