mkdir -p gpurun_out
for v in "pyabc_amd/libabcgpu.so 0" "pyabc_amd/libabcgpu.so 0.01" "ab/libguide.so 0.01"; do
  set -- $v
  ABCGPU_LIB=$1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --filter-below $2 > gpurun_out/ab_bench.log 2>&1 || exit 1
  echo "== $1 filter_below=$2"; tail -1 gpurun_out/ab_bench.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), d['generation_ms'][-6:], {k: round(v) for k, v in d['stages'].items() if k != 'note'}, '%.3e' % d['candidate_kernel']['candidates_per_s'])"
done
for L in pyabc_amd/libabcgpu.so ab/libguide.so; do echo "== $L"; ABCGPU_LIB=$L timeout -k 10 200 python -u tools/bench_fused.py --wsigma 2.2 --rates 1e-2 1e-3 1e-4 --modes plain filter --reps 3 2>&1 | grep cand || exit 1; done
