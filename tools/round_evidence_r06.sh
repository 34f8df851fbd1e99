#!/usr/bin/env bash
# Round-6 evidence pass on one GPU box (run from the repo root via gpurun), each step time-boxed
# and chained so that a failure ends the call:
#   part "tests": the whole GPU parity suite
#   part "lines": the bench lines of config 2 (default: the headline, with the CPU leg, scaled
#     rooflines and in-graph kernel timing), 1, 3 and 5, the config-2 DP-exchange forms at world
#     1 (the package's RCCL exchange with and without the overlap split, torch's collectives), and
#     the 2-rank self-launch rehearsal (gloo, one GPU)
#   part "all": lines, then the rocprofv3 --kernel-trace --stats summary of the default bench command
#   bash tools/round_evidence_r06.sh TAG tests|lines|all
set -euo pipefail
TAG=${1:-r06}
PART=${2:-lines}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/evidence_$TAG"
mkdir -p "$OUT"
cd "$R"
line() {  # name, timeout, bench args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
    "$OUT/$name.json" "$name"
}
if [ "$PART" = "tests" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
  exit 0
fi
line bench_line 400
line bench_line_config1 300 --config 1
line bench_line_config3 400 --config 3
line bench_line_config5 400 --config 5
Q="--no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5"
line plain_1 240 $Q
line dp_rccl_1 240 $Q --dp-exchange
line bench_gpus2_gloo_rehearsal 300 --gpus 2 --backend gloo --device-index 0 --steps 5 --warmup 2 \
  --no-kernel-timing
if [ "$PART" = "all" ]; then
  # the rocprofv3 summary of the default bench command (the line's kernel timing cross-check)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o b \
    -- python3 "$R/bench.py" > "$OUT/prof_default.log" 2>&1
  rm -f "$OUT/prof_default/b_kernel_trace.csv"
fi
