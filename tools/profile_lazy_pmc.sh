#!/bin/bash
# PMC passes over the fused round in plain and early-reject (lazy) modes on
# the c3 shape with skewed importance weights (ESS/N ~ 1%, as in c3's last
# generations), acceptance 1e-4: L2 hit / miss counts, VALU instructions,
# waves and wave cycles per kernel.  One rocprofv3 run per counter group.
#   tools/profile_lazy_pmc.sh OUTDIR
set -e
out=${1:-gpurun_out/lpmc}
mkdir -p $out
export TMPDIR=/tmp PYTHONPATH=$PWD
args="tools/bench_fused.py --wsigma 2.2 --rates 1e-4 --B 67108864 --reps 1 --modes plain filter"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD -d $out/p1 -o run -- python3 $args > $out/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $out/p2 -o run -- python3 $args > $out/p2.log 2>&1
