#!/bin/bash
# Round-3 baseline evidence on HEAD's kernels:
#  1. c3 population weights of late generations (ancestor-draw access analysis);
#  2. PMC of the fused candidate round on the c3 shape (uniform and skewed
#     weights): VALU instructions, L2 hits / misses per candidate;
#  3. bench.py c3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (x3 traffic).
# Raw rocprofv3 output stays in /tmp on the box; only summaries go to
# gpurun_out (the copy-back limit is 64 MiB).  Every GPU step has its own
# time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/r03base
W=/tmp/r03w
mkdir -p $O $W
timeout -k 10 240 python3 -u tools/dump_c3_population.py --gens 25 --keep 3 --out $O/pop > $O/dump.log 2>&1 || { echo "dump failed"; tail -5 $O/dump.log; exit 1; }
echo dump ok
timeout -k 5 60 ./tools/probes/mfma_f16_groups > $O/mfma_f16_groups.txt 2>&1 || { echo "probe failed"; exit 1; }
echo probe ok
for ws in 0 2.2; do
  args="tools/bench_fused.py --wsigma $ws --rates 1e-4 --B 67108864 --reps 1 --modes plain"
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES -d $W/fpmc_w$ws/p1 -o run -- python3 $args > $O/fpmc_w$ws.p1.log 2>&1 || { echo "fpmc p1 failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $W/fpmc_w$ws/p2 -o run -- python3 $args > $O/fpmc_w$ws.p2.log 2>&1 || { echo "fpmc p2 failed"; exit 1; }
  python3 tools/pmc_summary.py fused_round $(find $W/fpmc_w$ws -name "*.db") --per 67108864 > $O/fpmc_w$ws.summary.txt 2>&1 || true
  echo "fused pmc w$ws ok"
done
ARGS="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/trace -o run -- python3 bench.py $ARGS > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $W/trace -name "*kernel_stats.csv" -exec cp {} $O/trace_kernel_stats.csv \;
echo trace ok
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $W/pmc$i -o run -- python3 bench.py $ARGS > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $O/pmc$i.log; exit 1; }
  echo "pmc $i ok"
done
python3 tools/traffic_from_pmc.py $W mvn_x3_kernel 1000000 10 $O/x3_traffic_c3.json > $O/traffic.log 2>&1 || true
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_stochastic.py tests/test_gpu_fallbacks.py > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
echo tests ok
