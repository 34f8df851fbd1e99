#!/usr/bin/env bash
# Build the shipped GEMM solution table (PyTorch TunableOp, hipBLASLt solutions only) for the
# fixed shapes of the benchmarked configs: configs 2 (PPObj) and 3 (NatureCNN) and the config-5
# DQN; every run appends its shapes to the same file. Copy the result to
# oc_cleanrl_amd/tuning/tunableop_gfx950.csv.
#   bash tools/tune_gemms.sh
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_gfx950.csv
export OCPPO_GEMM_TABLE=0  # tune from scratch, not from the shipped table
rm -f gpurun_out/tunableop_gfx950*.csv
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing --steps 3 \
  > /dev/null 2> gpurun_out/tune_c2.err && echo "c2 tuned"
timeout -k 10 600 python3 bench.py --config 3 --no-cpu-baseline --no-scaled --no-kernel-timing \
  --steps 2 > /dev/null 2> gpurun_out/tune_c3.err && echo "c3 tuned"
timeout -k 10 400 python3 tools/dqn_bench.py --steps 2000 --warmup 500 > /dev/null \
  2> gpurun_out/tune_dqn.err && echo "dqn tuned"
wc -l gpurun_out/tunableop_gfx950*.csv
