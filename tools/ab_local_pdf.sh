# Same-box A/B of the LocalTransition density (tools/probes/local_pdf_probe.py):
# probe timings and kernel-trace stats per library, then one PMC pass
# (clock / MFMA / VALU) on the first unless NOPMC is set.
#   bash tools/ab_local_pdf.sh DEFAULT ab/libv1.so ...   (-> gpurun_out/ablp_<name>)
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
first=""
for L in "$@"; do
  if [ "$L" = DEFAULT ]; then n=default; lib=$R/pyabc_amd/libabcgpu.so; else n=$(basename $L .so); lib=$R/$L; fi
  [ -z "$first" ] && first=$lib && fn=$n
  ABCGPU_LIB=$lib timeout -k 10 120 python3 $R/tools/probes/local_pdf_probe.py --reps 10 > $R/gpurun_out/ablp_$n.log 2>&1
  ABCGPU_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ablp_$n -o run -- python3 $R/tools/probes/local_pdf_probe.py --reps 5 >> $R/gpurun_out/ablp_$n.log 2>&1
done
[ -n "$NOPMC" ] && exit 0
ABCGPU_LIB=$first timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/ablp_pmc_$fn/p1 -o run -- python3 $R/tools/probes/local_pdf_probe.py --reps 3 > $R/gpurun_out/ablp_pmc_$fn.log 2>&1
python3 $R/tools/pmc_clock_summary.py local_mfma_kernel $R/gpurun_out/ablp_pmc_$fn > $R/gpurun_out/ablp_pmc_$fn/summary.txt
