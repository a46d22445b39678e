export TMPDIR=/tmp PYTHONPATH=$PWD
bash tools/ab_local_fit.sh ab/libkbm.so
for L in ab/libknnt0.so ab/libknnt2.so ab/libknnt3.so ab/libknnt4.so; do echo $L; ABCGPU_LIB=$L timeout -k 10 120 python3 tools/probes/knn_timing.py || exit 1; done
for fb in 0 3e-4 1e-3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --filter-below $fb > gpurun_out/bench_fb$fb.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/bench_fb$fb.log'):
    if l.startswith('{'):
        d = json.loads(l); print('filter_below $fb', round(d['value']), 'cand_ms', round(d['stages']['candidate_rounds_ms']), 'last gens', d['generation_ms'][-4:])"
done
