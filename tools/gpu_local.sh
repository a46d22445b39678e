#!/bin/bash
# LocalTransition fit on the GPU box: parity tests, then c5 kernel traces
# (k = 50 and k = N/4) of tools/probes/c5_fit_probe.py.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/local
mkdir -p $O
[ "$1" = "notest" ] || timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "local" tests/test_gpu_rows.py::test_c5_local_fit_default_k \
  > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
[ "$1" = "notest" ] || tail -3 $O/tests.log
for k in 50 quarter; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lt_$k -o run -- python3 tools/probes/c5_fit_probe.py $k > $O/trace_$k.log 2>&1 || { echo "trace $k failed"; tail -5 $O/trace_$k.log; exit 1; }
  find /tmp/lt_$k -name "*kernel_stats.csv" -exec cp {} $O/c5_${k}_kernel_stats.csv \;
  echo "== k=$k"
  python3 -c "
import csv
for r in csv.DictReader(open('$O/c5_${k}_kernel_stats.csv')):
    print('  %-60s %4s %9.3f ms' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))"
done
