#!/bin/bash
# heads_loss at config: fewer, larger row ranges per workgroup (OCPPO_HL_ROWS 16 / 32 / 64 ->
# 256 / 128 / 64 records of 16 KB), PMC traffic and time of the rows + finish pair, and the bench
set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/hl
for v in base hl32 hl64; do
  if [ $v = base ]; then export OCPPO_LIB=$R/oc_cleanrl_amd/lib/libocppo_hip.so; else export OCPPO_LIB=$R/tools/variants/$v.so; fi
  timeout -k 10 120 python3 tools/kernel_bench.py --kernel heads_loss --size config > gpurun_out/hl/kb_$v.txt 2>&1
  timeout -k 10 120 python3 tools/kernel_bench.py --kernel heads_loss --size config --cold > gpurun_out/hl/kb_cold_$v.txt 2>&1
  bash tools/pmc_one.sh heads_loss config hl_$v > /dev/null 2>&1
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5 > gpurun_out/hl/line_$v.json 2> gpurun_out/hl/line_$v.err
done
unset OCPPO_LIB
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_dqn_gpu.py tests/test_cartpole_gpu.py tests/test_replay_gpu.py > gpurun_out/hl/tests_small_fwd.log 2>&1
timeout -k 10 300 python3 bench.py --config 5 > gpurun_out/hl/line_c5.json 2> gpurun_out/hl/line_c5.err
timeout -k 10 300 python3 bench.py --config 1 > gpurun_out/hl/line_c1.json 2> gpurun_out/hl/line_c1.err
