#!/usr/bin/env bash
# Round-5 A/B on one GPU box: the config-2 line in the plain, DP-exchange (eager collectives),
# DP-exchange (captured collectives) and per-step-noise forms, each time-boxed, each line kept.
#   bash tools/r05_dp_ab.sh TAG [extra bench args...]
set -euo pipefail
TAG=$1; shift || true
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/dpab_$TAG
mkdir -p "$OUT"
B="python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5 $*"
run() {  # name, extra args
  local name=$1; shift
  timeout -k 10 240 $B "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
    "$OUT/$name.json" "$name"
}
for pass in 1 2; do  # noqa
  run plain_$pass
  run dp_eager_$pass --dp-exchange
  run dp_graph_$pass --dp-exchange --set dp_graph_collectives=1
  run noise_$pass --set per_step_noise=1
done
