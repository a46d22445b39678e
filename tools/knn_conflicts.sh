#!/bin/bash
# LDS bank-conflict share and time of knn_select_kernel<5> on the c5 fit
# (N = 1e5, d = 5; k = 50 and k = N/4) for each library given (ABCGPU_LIB):
# one rocprofv3 pass with SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE and the
# kernel trace, summarised by tools/pmc_clock_summary.py.
export TMPDIR=/tmp PYTHONPATH=$PWD
OUT=${OUT:-gpurun_out/knnc}
mkdir -p $OUT
for L in "$@"; do
  for k in 50 quarter; do
    n=$(basename $L .so)_$k
    rm -rf /tmp/knnc_$n
    ABCGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace --output-format csv -d /tmp/knnc_$n -o run -- python3 tools/probes/c5_fit_probe.py $k > $OUT/$n.log 2>&1 || { echo "failed $n"; tail -5 $OUT/$n.log; exit 1; }
    echo "== $n"
    python3 tools/pmc_clock_summary.py knn_select_kernel /tmp/knnc_$n
    python3 tools/pmc_clock_summary.py knn_dense_kernel /tmp/knnc_$n | tail -1
  done
done
