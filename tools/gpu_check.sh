#!/bin/bash
# One GPU call: smoke, parity tests, bench line, rocprof kernel stats.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke_exit=$?"; tail -3 gpurun_out/smoke.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests_exit=$?"
tail -5 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --cpu-baseline-seconds 8 > gpurun_out/bench.log 2>&1 || { echo bench_fail; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || { echo prof_fail; tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name '*stats*'
