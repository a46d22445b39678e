#!/bin/bash
# Deferred-collect v2 (ABC_DEFER_V2: per-lane queue reservation, fp64 member
# sums in the resolve) against the default, on the GPU box.  Build the
# variant here first:
#   bash tools/build_variant.sh ab/libdeferv2.so abc_local.hip -DABC_DEFER_V2=1
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
ABCGPU_LIB=ab/libdeferv2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "local" \
  tests/test_gpu_rows.py::test_c5_local_fit_default_k > gpurun_out/defer_v2_tests.log 2>&1 \
  || { echo "v2 tests failed"; tail -30 gpurun_out/defer_v2_tests.log; exit 1; }
tail -2 gpurun_out/defer_v2_tests.log
bash tools/ab_local_fit.sh ab/libdeferv2.so
