#!/bin/bash
# Round check: smoke, the whole -m gpu suite, then the driver's bench command.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 400 python -u bench.py --steps 20 --warmup 5
step custom_model 300 python -u tools/probes/custom_model_c2.py 12
