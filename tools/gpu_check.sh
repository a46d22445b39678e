#!/bin/bash
# One GPU call: smoke, parity tests, bench line, rocprof kernel stats.
# Stops at the first step that faults / times out (exit codes other than 0/1).
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 500 python -u -m pytest $TESTS -m gpu -v --timeout 200 --timeout-method thread
step bench 300 python -u bench.py --steps 3 --warmup 2 --cpu-baseline-seconds 8
if [ -n "$PROF" ]; then
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline
fi
