# rocprofv3 kernel-trace + FETCH_SIZE + WRITE_SIZE passes of the weighted
# quantile component bench (N = 1e6 and 1e5), one pass each; summarise with
# python tools/pmc_kernels.py gpurun_out/qpmc --match wq_ --fetch-scale 2
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CMD="python3 $R/tools/bench_components.py --only quantile --reps 20"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/qpmc/trace -o run -- $CMD > $R/gpurun_out/qpmc_trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/qpmc/fetch -o run -- $CMD > $R/gpurun_out/qpmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/qpmc/write -o run -- $CMD > $R/gpurun_out/qpmc_write.log 2>&1
cd $R && python3 tools/pmc_kernels.py gpurun_out/qpmc --match wq_ --fetch-scale 2
