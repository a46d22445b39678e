set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_multirank.py > gpurun_out/mr.log 2>&1 || { echo "multirank failed"; tail -40 gpurun_out/mr.log; exit 1; }
tail -5 gpurun_out/mr.log
