#!/bin/bash
# SQ-counter passes over the two 11520-row gemm_x6 forms the config-2 update
# spends most in: the 128 x 128 tile (variant 24) on [11520 x 1024] from K = 512 (720 tiles) and
# the mixed tile (56) on [11520 x 512] from K = 1024 (360 tiles)
set -eo pipefail
bash tools/pmc_gemm.sh t24_fwd_11520_1024_512 fwd,11520,1024,512 24 > gpurun_out/pmc_t24.txt 2>&1
bash tools/pmc_gemm.sh t56_fwd_11520_512_1024 fwd,11520,512,1024 56 > gpurun_out/pmc_t56.txt 2>&1
bash tools/pmc_gemm.sh t24_dx_11520_1024_512 dx,11520,1024,512 24 > gpurun_out/pmc_t24dx.txt 2>&1
timeout -k 10 120 python3 tools/exp_gemm_x6.py --only fwd,11520,1024,512 --tiles 24 --reps 20 > gpurun_out/time_t24.txt 2>&1
timeout -k 10 120 python3 tools/exp_gemm_x6.py --only fwd,11520,512,1024 --tiles 56 --reps 20 > gpurun_out/time_t56.txt 2>&1
bash tools/prof_clean.sh r06a > /dev/null 2>&1
timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5 > gpurun_out/r06_plain.json 2> gpurun_out/r06_plain.err
timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-scaled --no-kernel-timing --steps 40 --warmup 5 --dp-exchange > gpurun_out/r06_dp.json 2> gpurun_out/r06_dp.err
