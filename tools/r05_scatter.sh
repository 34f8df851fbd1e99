#!/usr/bin/env bash
# Round-5: the frame scatter with the encoder's last ReLU backward, bitmask vs f32 mask:
# kernel_bench (warm and after an L3 scrub) at config and scaled sizes, then the PMC traffic
# passes of both forms (tools/pmc_one.sh; --cold like tools/profile_round.sh)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/scatter_r05
mkdir -p "$OUT"
for k in frames_scatter_relu frames_scatter_relu_f32; do
  timeout -k 10 240 python3 tools/kernel_bench.py --kernel $k > "$OUT/$k.jsonl"
  timeout -k 10 240 python3 tools/kernel_bench.py --kernel $k --cold > "$OUT/${k}_cold.jsonl"
done
cat "$OUT"/*.jsonl
REPO="$GRAFT_REPO_ROOT"
P="$REPO/gpurun_out/prof_r05s"
mkdir -p "$P"
cd /tmp && export TMPDIR=/tmp
for k in frames_scatter_relu frames_scatter_relu_f32; do
  for sz in config scaled; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 120 rocprofv3 --pmc "$ctr" --kernel-trace --output-format csv \
        -d "$P/pmc_${k}_${sz}_${ctr}" -o pmc \
        -- python3 "$REPO/tools/kernel_bench.py" --kernel "$k" --size "$sz" --reps 5 --rounds 1 --cold \
        > "$P/pmc_${k}_${sz}_${ctr}.log" 2>&1
    done
    echo "pmc $k $sz done"
  done
done
