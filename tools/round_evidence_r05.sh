#!/usr/bin/env bash
# Round-5 evidence pass on one GPU box (run from the repo root via gpurun), each step time-boxed
# and chained so that a failure ends the call:
#   part "tests": the whole GPU parity suite
#   part "lines": the bench lines of config 2 (default: the headline, with the CPU leg, scaled
#     rooflines and in-graph kernel timing), 1, 3 and 5, the config-2 DP-exchange forms at world
#     1 (the package's RCCL exchange with and without the overlap split, torch's collectives), and
#     the 2-rank self-launch rehearsal (gloo, one GPU)
#   bash tools/round_evidence_r05.sh TAG tests|lines
set -euo pipefail
TAG=${1:-r05}
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
line bench_line_config3 400 --config 3 --no-cpu-baseline
line bench_line_config5 400 --config 5
Q="--no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5"
for pass in 1 2; do
  line plain_$pass 240 $Q
  line dp_rccl_$pass 240 $Q --dp-exchange
  line dp_rccl_noov_$pass 240 $Q --dp-exchange --set dp_overlap=0
  line dp_torch_$pass 240 $Q --dp-exchange --set dp_collectives=torch
done
line bench_gpus2_gloo_rehearsal 300 --gpus 2 --backend gloo --device-index 0 --steps 5 --warmup 2 \
  --no-kernel-timing
