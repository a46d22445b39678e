#!/bin/bash
# Round measurements for DESIGN/BASELINE: c3 under the driver's bench command
# with a rocprofv3 kernel trace, the c2 bench line, and the component benches.
export TMPDIR=/tmp
OUT=gpurun_out/meas
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_trace.log 2>&1 || { echo "c3 trace failed"; exit 1; }
echo c3 trace ok
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --pop 100000 --no-cpu-baseline > $OUT/c2_bench.log 2>&1 || { echo "c2 failed"; exit 1; }
echo c2 ok
timeout -k 10 400 python -u tools/bench_components.py --only ${COMPONENTS:-c4,quantile,c5,e2e} > $OUT/components.log 2>&1 || { echo "components failed"; exit 1; }
echo components ok
