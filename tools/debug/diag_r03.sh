set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/diag
timeout -k 10 120 python3 -u tools/debug/gave_up_diag.py > gpurun_out/diag/gave_up.log 2>&1 || { echo diag failed; tail -20 gpurun_out/diag/gave_up.log; exit 1; }
tail -30 gpurun_out/diag/gave_up.log
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fallbacks.py tests/test_gpu_fused.py tests/test_stochastic.py > gpurun_out/diag/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/diag/tests.log; exit 1; }
tail -3 gpurun_out/diag/tests.log
