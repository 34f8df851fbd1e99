set -e
cd $GRAFT_REPO_ROOT
for sm in 8 16; do
  OCPPO_LIN_SMAX=$sm timeout -k 10 120 python3 tools/exp_rollout_linear.py > gpurun_out/lin_sm$sm.log 2>&1
  OCPPO_LIN_SMAX=$sm timeout -k 10 100 python3 tools/kernel_bench.py --kernel cache_linear --size config >> gpurun_out/lin_sm$sm.log 2>&1
done
OCPPO_LIN_SMAX=16 timeout -k 10 200 python3 -m pytest tests/test_kernels_gpu.py -q -x -k "linear" --timeout 60 --timeout-method thread > gpurun_out/lin_tests.log 2>&1
