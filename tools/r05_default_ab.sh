#!/usr/bin/env bash
# Round-5: the default bench line's timed region with and without the in-graph kernel timer and
# with a longer warm-up (is the default line's gap to the 40-step lines the timer or the warm-up?)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for spec in "kt:" "nokt:--no-kernel-timing" "kt_w10:--warmup 10" "nokt_w10:--no-kernel-timing --warmup 10"; do
    name=${spec%%:*}; args=${spec#*:}
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-scaled $args > gpurun_out/dab_$name.json 2>/dev/null
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['steps'], d['warmup'])" gpurun_out/dab_$name.json $name
  done
done
