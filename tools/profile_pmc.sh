#!/bin/bash
# Stall / issue / occupancy counters of kernels under a probe command, one
# rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: PMC slots, no
# trace domains), summarised per kernel by tools/pmc_summary.py.
#   bash tools/profile_pmc.sh NAME "KERNEL_SUBSTR ..." python3 tools/probes/x.py [args]
#   -> gpurun_out/pmc_NAME/summary.txt
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
NAME=$1; KERNELS=$2; shift 2
O=gpurun_out/pmc_$NAME
W=/tmp/pmc_$NAME
mkdir -p $O $W
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $W/p$i -o run -- "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
: > $O/summary.txt
for kn in $KERNELS; do python3 tools/pmc_summary.py $kn $(find $W -name "*.db") >> $O/summary.txt 2>&1; done
cat $O/summary.txt
