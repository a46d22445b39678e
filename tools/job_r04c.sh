#!/bin/bash
# Round-4 job c: parity of the changed kernels (weighted-quantile select +
# sorted fallback, padded k-NN rows, accept tail, wide LocalTransition,
# large-N statistics), then same-box A/Bs of the c5 fit (unpadded baseline /
# padded / DEFER_V2 / dense-kernel shapes); the k-NN PMC on the padded
# kernel, the c3 trace and x3 traffic passes, the user-model probe, the
# candidate round with weight-sorted records.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r04c
W=/tmp/r04cw
mkdir -p $O $W
# PART=tests: the GPU parity suites; PART=rest: everything after (two gpurun calls)
if [ "${PART:-tests}" = tests ]; then
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_rows.py tests/test_gpu_fused.py tests/test_gpu_fallbacks.py \
  tests/test_gpu_e2e.py::test_large_n_parity_vs_reference > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
exit 0
fi
ABCGPU_LIB=ab/libdeferv2.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "local" tests/test_gpu_rows.py::test_c5_local_fit_default_k > $O/defer_v2_tests.log 2>&1 \
  && echo "v2 tests ok" || { echo "v2 tests failed"; tail -15 $O/defer_v2_tests.log; }
bash tools/ab_local_fit.sh ab/libbase_local.so ab/libdeferv2.so ab/libdm_w8.so ab/libdm_sb1.so > $O/ab_local_fit.log 2>&1 || { echo "ab failed"; cat $O/ab_local_fit.log; exit 1; }
cat $O/ab_local_fit.log
K=/tmp/knnpmc
args="tools/probes/c5_fit_probe.py quarter"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $K/p1 -o run -- python3 $args > $O/knn_p1.log 2>&1 || { echo knn p1 failed; tail -5 $O/knn_p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $K/p2 -o run -- python3 $args > $O/knn_p2.log 2>&1 || { echo knn p2 failed; tail -5 $O/knn_p2.log; exit 1; }
for kn in knn_select_kernel knn_dense_kernel knn_resolve_kernel; do python3 tools/pmc_summary.py $kn $(find $K -name "*.db") --per 1 >> $O/knn_pmc_summary.txt 2>&1; done
echo knn pmc ok
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/trace -o run -- python3 bench.py $ARGS > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $W/trace -name "*kernel_stats.csv" -exec cp {} $O/bench_c3_3step_kernel_stats.csv \;
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $W/x3pmc$i -o run -- python3 bench.py $ARGS > $O/x3pmc$i.log 2>&1 || { echo "x3 pmc $i failed"; tail -3 $O/x3pmc$i.log; exit 1; }
done
python3 tools/traffic_from_pmc.py $W "mvn_x3_kernelILi3ELi8ELb0E" 1000000 10 $O/x3_traffic_c3.json > $O/traffic.log 2>&1 || true
cat $O/traffic.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/cm -o run -- python3 -u tools/probes/custom_model_c2.py 20 > $O/custom20.log 2>&1 || { echo "custom probe failed"; tail -5 $O/custom20.log; exit 1; }
find $W/cm -name "*kernel_stats.csv" -exec cp {} $O/custom_model_kernel_stats.csv \;
grep model $O/custom20.log | cut -c1-700
for ws in 0 2.2; do
  for so in "" "--sort-weights"; do
    timeout -k 10 120 python3 -u tools/bench_fused.py --wsigma $ws --rates 1e-4 --B 134217728 --reps 2 --modes plain $so > $O/fused_w${ws}${so}.log 2>&1 || { echo "bench_fused failed"; tail -5 $O/fused_w${ws}${so}.log; exit 1; }
    echo "wsigma $ws $so: $(grep candidates $O/fused_w${ws}${so}.log)"
  done
done
