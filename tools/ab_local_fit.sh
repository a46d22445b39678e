#!/bin/bash
# c5 LocalTransition fit kernel averages (rocprofv3) for the in-tree library
# and variants given as arguments (built with tools/build_src_variant.sh).
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out
for L in pyabc_amd/libabcgpu.so "$@"; do
  for k in 50 quarter; do
    rm -rf /tmp/abl
    ABCGPU_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/abl -o run -- python3 tools/probes/c5_fit_probe.py $k > gpurun_out/abl.log 2>&1 || { echo "failed $L $k"; tail -5 gpurun_out/abl.log; exit 1; }
    python3 -c "
import csv, glob
tot = 0.0; parts = []
for r in csv.DictReader(open(glob.glob('/tmp/abl/**/*kernel_stats.csv', recursive=True)[0])):
    ms = float(r['AverageNs']) / 1e6
    if any(t in r['Name'] for t in ('knn_', 'local_', 'mm_')):
        tot += ms
        if ms > 0.05: parts.append('%s %.3f' % (r['Name'].split('(')[0].split('::')[-1][:26], ms))
print('%-22s k=%-8s fit %.3f ms | %s' % ('$L'.split('/')[-1], '$k', tot, ', '.join(parts)))"
  done
done
