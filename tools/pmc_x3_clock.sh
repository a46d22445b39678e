#!/bin/bash
# PMC passes over the x3 density at the c3 shape (N = M = 1e6, d = 10,
# hinted), for the library named by ABCGPU_LIB (default: in-tree): issue
# and MFMA counters plus GRBM_GUI_ACTIVE, whose quotient by 8 x the kernel's
# duration is the clock the chip held (MI355X_MICROARCH.md, DVFS give-back).
#   ABCGPU_LIB=ab/libx.so bash tools/pmc_x3_clock.sh OUTDIR
OUT=${1:-gpurun_out/x3pmc}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--N 1000000 --M 1000000 --prec x3+hint --reps 2"
i=0
for set in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_COUNT" ; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/bench_mvn.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_clock_summary.py mvn_x3_kernel $OUT > $OUT/summary.txt && cat $OUT/summary.txt
