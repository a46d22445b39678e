#!/bin/bash
# Round-4 job e: HEAD's measurements for DESIGN.md / BASELINE.md -- the bench
# (driver default, the 20-generation c3 command, c2), its rocprofv3 kernel
# trace, the component table.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo "bench default failed"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_c3_20gen.log 2>&1 || { echo "bench 20 failed"; tail -5 $O/bench_c3_20gen.log; exit 1; }
tail -1 $O/bench_c3_20gen.log | cut -c1-300
timeout -k 10 300 python3 -u bench.py --pop 100000 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_20gen.log 2>&1 || { echo "bench c2 failed"; tail -5 $O/bench_c2_20gen.log; exit 1; }
tail -1 $O/bench_c2_20gen.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r04etr -o run -- python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c3_rocprof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/bench_c3_rocprof.log; exit 1; }
find /tmp/r04etr -name "*kernel_stats.csv" -exec cp {} $O/bench_c3_5step_kernel_stats.csv \;
tail -1 $O/bench_c3_rocprof.log | cut -c1-200
timeout -k 10 480 python3 -u tools/bench_components.py --only c4,quantile,c5,sampler,cv,stochastic,history > $O/components.log 2>&1 || { echo "components failed"; tail -5 $O/components.log; exit 1; }
echo components ok
