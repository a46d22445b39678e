#!/bin/bash
# Same-box A/B of libabcgpu builds (tools/build_src_variant.sh variants;
# DEFAULT = the in-tree library), interleaved, one line per run.
#   bash tools/ab.sh MODE LIB...        MODE: bench | fused | fit | mad | pdf
#   bench: bench.py (BENCH_ARGS) -> accepted/s, ms/gen, x3 launch avg, stages
#   fused: tools/bench_fused.py (FUSED_ARGS) -> candidates/s
#   fit:   tools/probes/c5_fit_probe.py k = 50 and N/4 -> kernel-trace fit ms
#   mad:   the MAD GPU tests, then tools/bench_components.py --only c4
#   pdf:   tools/probes/local_pdf_probe.py -> LocalTransition density ms
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp PYTHONPATH=$R
mkdir -p $R/gpurun_out
MODE=$1; shift
lib() { [ "$1" = DEFAULT ] && echo $R/pyabc_amd/libabcgpu.so || echo $R/$1; }
for rep in $(seq ${REPS:-1}); do
for L in "$@"; do
  LIB=$(lib $L); n=$(basename $LIB .so)
  case $MODE in
  bench)
    ABCGPU_LIB=$LIB timeout -k 10 300 python3 -u $R/bench.py ${BENCH_ARGS:---steps 6 --warmup 2} --no-cpu-baseline > $R/gpurun_out/ab_bench.log 2>&1 || { tail -5 $R/gpurun_out/ab_bench.log; exit 1; }
    echo "== $L"; tail -1 $R/gpurun_out/ab_bench.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); s=d['stages']; r=d.get('roofline') or {}
print(round(d['value']), 'ms/gen', round(d['ms_per_step'], 3), 'x3', round(r.get('avg_launch_ms', 0), 3),
      {k: round(v, 2) for k, v in s.items() if k.endswith('_ms')})" ;;
  fused)
    echo "== $L"
    ABCGPU_LIB=$LIB timeout -k 10 200 python3 -u $R/tools/bench_fused.py ${FUSED_ARGS:---rates 1e-2 1e-4 --modes plain --reps 3} 2>&1 | grep -E "candidates/s|Error|error" || exit 1 ;;
  fit)
    for k in 50 quarter; do
      rm -rf /tmp/abl
      ABCGPU_LIB=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/abl -o run -- python3 $R/tools/probes/c5_fit_probe.py $k > $R/gpurun_out/abl.log 2>&1 || { echo "failed $L $k"; tail -5 $R/gpurun_out/abl.log; exit 1; }
      python3 -c "
import csv, glob
tot = 0.0; parts = []
for r in csv.DictReader(open(glob.glob('/tmp/abl/**/*kernel_stats.csv', recursive=True)[0])):
    ms = float(r['AverageNs']) / 1e6
    if any(t in r['Name'] for t in ('knn_', 'local_', 'mm_')):
        tot += ms
        if ms > 0.05: parts.append('%s %.3f' % (r['Name'].split('(')[0].split('::')[-1][:26], ms))
print('%-22s k=%-8s fit %.3f ms | %s' % ('$n', '$k', tot, ', '.join(parts)))"
    done ;;
  mad)
    echo "== $L"
    ABCGPU_LIB=$LIB timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $R/tests/test_gpu_kernels.py $R/tests/test_gpu_rows.py -k "mad or MAD or adaptive" 2>&1 | tail -1 || exit 1
    ABCGPU_LIB=$LIB timeout -k 10 120 python3 -u $R/tools/bench_components.py --only c4 2>&1 | grep "MAD" | cut -c1-200 || exit 1 ;;
  pdf)
    echo "== $L"
    ABCGPU_LIB=$LIB timeout -k 10 120 python3 $R/tools/probes/local_pdf_probe.py --reps 10 2>&1 | tail -2 || exit 1 ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
  esac
done
done
