#!/bin/bash
# the convolution gathers (GATH 3-7 of ocppo_gemm.hip) with every computed
# index checked against its extent, once, on the GPU box. The variant library is built here (CPU)
# beforehand:
#   python tools/build_variant.py tools/variants/x6_bounds.so --only ocppo_gemm.hip -DOCPPO_X6_BOUNDS
# then, on the box:
#   bash tools/run_bounds_check.sh > profiles/r06/bounds_check.log
set -o pipefail
export OCPPO_LIB=tools/variants/x6_bounds.so
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_conv_gpu.py \
  tests/test_trainer_gpu.py::test_pixel_natureccn_iteration \
  tests/test_config3_golden_gpu.py
