#!/bin/bash
# Round-4 first GPU job: the full -m gpu suite on HEAD (incl. the self-launched
# 2-rank bench), the x3 traffic passes on the main instantiation, the k-NN PMC
# on knn_dense_kernel<5,true> at k = N/4, and the ABC_DEFER_V2 A/B.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r04a
W=/tmp/r04w
mkdir -p $O $W
timeout -k 5 60 ./tools/probes/mfma_mix > $O/mfma_mix.txt 2>&1 || { echo "mfma probe failed"; cat $O/mfma_mix.txt; exit 1; }
cat $O/mfma_mix.txt
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $W/x3pmc$i -o run -- python3 bench.py $ARGS > $O/x3pmc$i.log 2>&1 || { echo "x3 pmc $i failed"; tail -3 $O/x3pmc$i.log; exit 1; }
  echo "x3 pmc $i ok"
done
python3 tools/traffic_from_pmc.py $W "mvn_x3_kernel<3, 8, false>" 1000000 10 $O/x3_traffic_c3.json > $O/traffic.log 2>&1 || { echo traffic failed; cat $O/traffic.log; }
cat $O/traffic.log
K=/tmp/knnpmc
args="tools/probes/c5_fit_probe.py quarter"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $K/p1 -o run -- python3 $args > $O/knn_p1.log 2>&1 || { echo knn p1 failed; tail -5 $O/knn_p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $K/p2 -o run -- python3 $args > $O/knn_p2.log 2>&1 || { echo knn p2 failed; tail -5 $O/knn_p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_ACTIVE_INST_SCA TCC_HIT_sum TCC_MISS_sum -d $K/p3 -o run -- python3 $args > $O/knn_p3.log 2>&1 || { echo knn p3 failed; tail -5 $O/knn_p3.log; exit 1; }
for kn in knn_select_kernel knn_dense_kernel knn_resolve_kernel; do python3 tools/pmc_summary.py $kn $(find $K -name "*.db") --per 1 >> $O/knn_pmc_summary.txt 2>&1; done
echo knn pmc ok
bash tools/ab_defer_v2.sh > $O/defer_v2_ab.log 2>&1 || { echo "defer v2 A/B failed"; tail -20 $O/defer_v2_ab.log; exit 1; }
cat $O/defer_v2_ab.log
