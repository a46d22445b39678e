timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py -v --timeout 200 --timeout-method thread -m gpu -x > gpurun_out/e2e.log 2>&1; echo e2e_exit=$?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --cpu-baseline-seconds 5 > gpurun_out/bench1.log 2>&1; echo bench_exit=$?
tail -30 gpurun_out/e2e.log; tail -5 gpurun_out/bench1.log
