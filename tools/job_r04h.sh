#!/bin/bash
# Round-4 job h: the final HEAD measurements -- bench (driver default, 20
# generations, c2), its rocprofv3 kernel trace, the x3 traffic passes.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r04h
W=/tmp/r04hw
mkdir -p $O $W
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo "bench default failed"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_c3_20gen.log 2>&1 || { echo "bench 20 failed"; tail -5 $O/bench_c3_20gen.log; exit 1; }
tail -1 $O/bench_c3_20gen.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --pop 100000 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_20gen.log 2>&1 || { echo "bench c2 failed"; exit 1; }
tail -1 $O/bench_c2_20gen.log | cut -c1-200
ARGS="--steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/trace -o run -- python3 -u bench.py $ARGS > $O/bench_c3_rocprof.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $W/trace -name "*kernel_stats.csv" -exec cp {} $O/bench_c3_5step_kernel_stats.csv \;
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $W/x3pmc$i -o run -- python3 bench.py $ARGS > $O/x3pmc$i.log 2>&1 || { echo "x3 pmc $i failed"; tail -3 $O/x3pmc$i.log; exit 1; }
done
python3 tools/traffic_from_pmc.py $W "mvn_x3_kernelILi3ELi10ELb0E" 1000000 10 $O/x3_traffic_c3.json
