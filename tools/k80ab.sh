#!/bin/bash
# K80 x3 chain variants: correctness (tools/probes/x3_k80_debug.py against
# the f64 mode) and the c3 x3 launch time, against the KB layout (libx3old).
export PYTHONPATH=$PWD
mkdir -p gpurun_out
for L in "$@"; do
  echo "== $L"
  ABCGPU_LIB=$L timeout -k 5 100 python3 -u tools/probes/x3_k80_debug.py | tail -1 || exit 1
done
for L in ab/libx3old.so "$@"; do
  ABCGPU_LIB=$L timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/ab_x3.log 2>&1 || exit 1
  echo "== $L"; tail -1 gpurun_out/ab_x3.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), 'x3 avg ms', round(d['roofline']['avg_launch_ms'], 3), 'frac', round(d['roofline']['frac'], 4))"
done
