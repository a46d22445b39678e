#!/bin/bash
# Profiles of the default bench (c3) for profiles/: kernel-trace stats, then
# one rocprofv3 --pmc pass per counter group (FETCH_SIZE, WRITE_SIZE, SQ busy),
# each in its own run (MI355X_MICROARCH.md: PMC slots, no trace domains).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo trace ok
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
  echo "pmc $i ok"
done
