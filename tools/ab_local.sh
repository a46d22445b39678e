#!/bin/bash
# Interleaved A/B of the LocalTransition fit at c5's default k (N = 1e5,
# d = 5, k = N/4): kernel averages with the in-tree library and a variant.
V=${1:-ab/libmmold.so}
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in $V pyabc_amd/libabcgpu.so $V pyabc_amd/libabcgpu.so; do
  rm -rf gpurun_out/abl
  ABCGPU_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl -o run -- python3 tools/probes/c5_fit_probe.py quarter > gpurun_out/abl.log 2>&1 || exit 1
  echo "== $L"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/abl/run_kernel_stats.csv')):
    if 'moments' in r['Name'] or 'select' in r['Name']: print('  %-40s %.3f ms' % (r['Name'][:40], float(r['AverageNs'])/1e6))"
done
