#!/bin/bash
# PMC passes over the transition-density micro-benchmark (one rocprofv3 run
# per counter group; see MI355X_MICROARCH.md "rocprofv3 PMC slots").
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--prec ${PREC:-x3} --reps 2"
i=0
for set in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE GRBM_COUNT" \
  "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/bench_mvn.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
echo done
