#!/usr/bin/env bash
# Config 3 SPS under the convolution-algorithm modes (deterministic MIOpen vs not, Find on/off).
set -euo pipefail
R=$GRAFT_REPO_ROOT
for s in "torch_deterministic=0" "torch_deterministic=0 --set conv_benchmark=1"; do
  timeout -k 10 400 python3 $R/bench.py --config 3 --steps 3 --warmup 2 --no-kernel-timing --set $s > $R/gpurun_out/c3m.log 2>&1
  echo "$s $(tail -n 1 $R/gpurun_out/c3m.log | cut -c1-200)"
done
