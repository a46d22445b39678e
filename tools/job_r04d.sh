#!/bin/bash
# Round-4 job d: the staged user-model path after the accept-tail and
# proposal changes -- parity (fused / fallbacks / kernels / multirank), the
# tail probe (HEAD's abc_fused.hip vs the tree), the c2 user-model run.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r04d
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_fallbacks.py tests/test_gpu_kernels.py tests/test_gpu_multirank.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/tests.log
for L in ab/libfused_head.so pyabc_amd/libabcgpu.so; do
  echo "== $L"; ABCGPU_LIB=$L timeout -k 5 120 python3 -u tools/probes/user_tail_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04dcm -o run -- python3 -u tools/probes/custom_model_c2.py 20 > $O/custom20.log 2>&1 || { echo "custom probe failed"; tail -5 $O/custom20.log; exit 1; }
find /tmp/r04dcm -name "*kernel_stats.csv" -exec cp {} $O/custom_model_kernel_stats.csv \;
grep model $O/custom20.log | cut -c1-400
