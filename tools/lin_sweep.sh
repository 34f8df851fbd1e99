set -e
cd $GRAFT_REPO_ROOT
for cfg in "1 0 0" "1 1 0" "1 1 4" "1 1 2" "1 0 4"; do
  set -- $cfg
  OCPPO_LIN_STAGE=$1 OCPPO_LIN_PIPE=$2 OCPPO_LIN_CH=$3 timeout -k 10 120 python3 tools/exp_rollout_linear.py > gpurun_out/lin_s$1_p$2_c$3.log 2>&1
  OCPPO_LIN_STAGE=$1 OCPPO_LIN_PIPE=$2 OCPPO_LIN_CH=$3 timeout -k 10 100 python3 tools/kernel_bench.py --kernel cache_linear --size config >> gpurun_out/lin_s$1_p$2_c$3.log 2>&1
done
OCPPO_LIN_STAGE=1 OCPPO_LIN_PIPE=1 timeout -k 10 200 python3 -m pytest tests/test_kernels_gpu.py -q -x -k "linear" --timeout 60 --timeout-method thread > gpurun_out/lin_tests.log 2>&1
