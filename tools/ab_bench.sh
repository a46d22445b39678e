#!/bin/bash
# Interleaved A/B of whole bench lines on one box: bench.py with the given
# libraries (ABCGPU_LIB) and extra bench arguments (BENCH_ARGS), printing
# accepted/s, ms per generation and the bench's stage split for each run.
#   BENCH_ARGS="--pop 100000 --steps 20 --warmup 5" bash tools/ab_bench.sh LIB...
mkdir -p gpurun_out
for L in "$@"; do
  ABCGPU_LIB=$L timeout -k 10 240 python -u bench.py ${BENCH_ARGS:---steps 6 --warmup 2} --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1 || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  echo "== $L"; tail -1 gpurun_out/ab_bench.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); s=d['stages']
print(round(d['value']), 'ms/gen', round(d['ms_per_step'], 3), {k: round(v, 2) for k, v in s.items() if k.endswith('_ms')})"
done
