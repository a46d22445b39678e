#!/bin/bash
# Interleaved A/B of the x3 density kernel on one box: bench.py (c3) with
# the in-tree library and the variants given, printing the x3 launch
# average and the throughput of each run.
mkdir -p gpurun_out
for L in "$@"; do
  ABCGPU_LIB=$L timeout -k 10 200 python -u bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline > gpurun_out/ab_x3.log 2>&1 || exit 1
  echo "== $L"; tail -1 gpurun_out/ab_x3.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), 'x3 avg ms', round(d['roofline']['avg_launch_ms'], 3), 'frac', round(d['roofline']['frac'], 4))"
done
