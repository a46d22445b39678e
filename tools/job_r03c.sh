set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_fallbacks.py tests/test_stochastic.py tests/test_gpu_api.py tests/test_gpu_e2e.py > gpurun_out/tests_c.log 2>&1 || { tail -30 gpurun_out/tests_c.log; exit 1; }
tail -2 gpurun_out/tests_c.log
timeout -k 10 400 python -u tools/probes/custom_model_c2.py 20 user > gpurun_out/custom20b.log 2>&1 || exit 1
grep model gpurun_out/custom20b.log | cut -c1-600
