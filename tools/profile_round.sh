#!/usr/bin/env bash
# Round profile capture on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the bench command (per-kernel durations)
#   2. PMC passes (FETCH_SIZE, WRITE_SIZE separately, --kernel-trace only) of the north-star
#      kernels at config and scaled sizes, one kernel_bench case per run.
# Outputs under gpurun_out/prof_<tag>/; copy the summaries into profiles/ afterwards.
set -euo pipefail
TAG=${1:-r02}
OUT="$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG"
REPO="$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o bench \
  -- python3 "$REPO/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-scaled \
  > "$OUT/bench.log" 2>&1
echo "bench trace done"
for case in "policy_head config" "gae config" "ppo_loss_prepared config" \
            "gae scaled" "ppo_loss_prepared scaled" "policy_head scaled" "rollout_store scaled" \
            "gather scaled" "relu_bias_grad config" "relu_bias_grad scaled" \
            "relu_bias_wgrad config" "heads_bwd config" "heads_loss config" "heads_loss scaled" \
            "cache_linear config" "store_encode config" "gather_pixels config" \
            "decoder config" "encoder_mid config"; do
  set -- $case
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 240 rocprofv3 --pmc "$ctr" --kernel-trace --output-format csv \
      -d "$OUT/pmc_${1}_${2}_${ctr}" -o pmc \
      -- python3 "$REPO/tools/kernel_bench.py" --kernel "$1" --size "$2" --reps 5 --rounds 1 \
      > "$OUT/pmc_${1}_${2}_${ctr}.log" 2>&1
  done
  echo "pmc $1 $2 done"
done
