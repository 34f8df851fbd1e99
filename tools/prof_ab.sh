set -euo pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pc1 -o b -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-scaled --no-kernel-timing > $R/gpurun_out/pc1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pc0 -o b -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-scaled --no-kernel-timing --set rollout_frame_cache=0 > $R/gpurun_out/pc0.log 2>&1
