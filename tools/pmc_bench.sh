#!/usr/bin/env bash
# In-situ HBM traffic of the bench's own kernels: two rocprofv3 PMC passes (FETCH_SIZE, then
# WRITE_SIZE: they do not fit one pass) over a short bench run (graphs replayed, kernel timer off),
# then tools/pmc_bench_summary.py -> gpurun_out/pmc_bench_<tag>/summary.json (mean per dispatch of
# every kernel name; the gemm_x6 aggregate the bench's roofline quotes).
#   bash tools/pmc_bench.sh r04
set -euo pipefail
TAG=${1:-r04}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc_bench_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc "$ctr" --kernel-trace --output-format csv -d "$OUT/$ctr" -o pmc \
    -- python3 "$R/bench.py" --steps 3 --warmup 2 --no-kernel-timing --no-cpu-baseline --no-scaled \
    > "$OUT/$ctr.log" 2>&1
  echo "pmc $ctr done"
done
cd "$R"
python3 tools/pmc_bench_summary.py "$OUT" > "$OUT/summary.json"
echo "summary written"
