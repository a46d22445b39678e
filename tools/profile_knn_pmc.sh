#!/bin/bash
# PMC of knn_select_kernel<5> on the c5 fit (k = 50), normalised per 64-row
# tile-wave step (N/16 row tiles x N/16 particle tiles x 2 sweeps).
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/knnpmc
W=/tmp/knnpmc
mkdir -p $O $W
args="tools/probes/c5_fit_probe.py ${1:-50}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $W/p1 -o run -- python3 $args > $O/p1.log 2>&1 || { echo p1 failed; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $W/p2 -o run -- python3 $args > $O/p2.log 2>&1 || { echo p2 failed; tail -5 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_ACTIVE_INST_SCA TCC_HIT_sum TCC_MISS_sum -d $W/p3 -o run -- python3 $args > $O/p3.log 2>&1 || { echo p3 failed; tail -5 $O/p3.log; exit 1; }
for kn in knn_select_kernel knn_dense_kernel; do python3 tools/pmc_summary.py $kn $(find $W -name "*.db") --per 1 >> $O/summary.txt 2>&1; done
cat $O/summary.txt
