#!/usr/bin/env bash
# PMC instruction mix of the fused loss at the scaled size (one counter set per run).
set -euo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
KCASE=${1:-ppo_loss_prepared}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc_a -o p -- python3 $R/tools/kernel_bench.py --kernel $KCASE --size scaled --reps 3 --rounds 1 > $R/gpurun_out/pmc_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_b -o p -- python3 $R/tools/kernel_bench.py --kernel $KCASE --size scaled --reps 3 --rounds 1 > $R/gpurun_out/pmc_b.log 2>&1 || echo "pass b failed"
