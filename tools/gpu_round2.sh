#!/bin/bash
# One GPU call: smoke, the -m gpu suite, the fused-round modes on the c3
# shape, and the bench under the driver's command.  Stops at the first step
# that faults / times out (exit codes other than 0/1).
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step fused_tests 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread
step fused_modes 200 python -u tools/bench_fused.py --rates 3e-1 3e-2 1e-3 1e-4 --modes plain filter --reps 3
step gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step bench 300 python -u bench.py --steps 20 --warmup 5
