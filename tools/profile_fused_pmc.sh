#!/bin/bash
# PMC passes over the fused candidate round (tools/bench_fused.py, plain mode,
# c3 shape at acceptance 1e-4), one rocprofv3 run per counter group.
#   tools/profile_fused_pmc.sh OUTDIR
set -e
out=${1:-gpurun_out/fpmc}
export TMPDIR=/tmp PYTHONPATH=$PWD
args="tools/bench_fused.py ${FUSED_ARGS:---rates 1e-4 --B 67108864 --reps 1 --modes plain}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $out/p1 -o run -- python3 $args > $out.p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d $out/p2 -o run -- python3 $args > $out.p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_EXP SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $out/p3 -o run -- python3 $args > $out.p3.log 2>&1
