#!/bin/bash
# Round measurements for DESIGN/BASELINE: the c3 20-generation bench line,
# the c2 bench line, the component benches and a c2 host-gap trace
# (kernel + HIP runtime trace; tools/host_gaps.py reads it).
export TMPDIR=/tmp
OUT=gpurun_out/meas
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_20gen.log 2>&1 || { echo "c3 failed"; exit 1; }
echo c3 ok
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --pop 100000 --no-cpu-baseline > $OUT/c2_bench.log 2>&1 || { echo "c2 failed"; exit 1; }
echo c2 ok
timeout -k 10 400 python -u tools/bench_components.py --only ${COMPONENTS:-c4,quantile,c5,e2e} > $OUT/components.log 2>&1 || { echo "components failed"; exit 1; }
echo components ok
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $OUT/c2trace -o run -- python3 bench.py --pop 100000 --steps 3 --warmup 2 --no-cpu-baseline > $OUT/c2trace.log 2>&1 || { echo "c2 trace failed"; exit 1; }
echo c2 trace ok
