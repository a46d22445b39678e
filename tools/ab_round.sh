#!/bin/bash
# Interleaved A/B of the fused candidate round: tools/bench_fused.py and the
# c3 bench with the in-tree library and a variant ($1), alternating.
V=${1:-ab/libboxold.so}
mkdir -p gpurun_out
for L in $V pyabc_amd/libabcgpu.so $V pyabc_amd/libabcgpu.so; do
  echo "== $L"
  ABCGPU_LIB=$L timeout -k 10 200 python -u tools/bench_fused.py --wsigma 2.2 --rates 1e-3 1e-4 --modes plain --reps 3 2>&1 | grep cand || exit 1
  ABCGPU_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_round.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_round.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), 'x3 avg ms', round(d['roofline']['avg_launch_ms'], 3), 'cand/s %.3e' % d['candidate_kernel']['candidates_per_s'], {k: round(v) for k, v in d['stages'].items() if k != 'note'})"
done
