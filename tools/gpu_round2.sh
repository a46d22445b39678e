#!/bin/bash
# One GPU call: smoke, the -m gpu suite, the bench under the driver's command,
# and (PROF=1) the same bench under a rocprofv3 kernel trace.  Stops at the
# first step that faults / times out (exit codes other than 0/1).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step bench 300 python -u bench.py --steps 20 --warmup 5
if [ -n "$PROF" ]; then
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
fi
