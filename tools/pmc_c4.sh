# rocprofv3 kernel-trace + FETCH_SIZE + WRITE_SIZE passes of the c4 component bench
# (pnorm, column std, column MAD), one pass each; summarise with
# python tools/pmc_kernels.py gpurun_out/mad
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CMD="python3 $R/tools/bench_components.py --only c4 --reps 2"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mad/trace -o run -- $CMD > $R/gpurun_out/mad_trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/mad/fetch -o run -- $CMD > $R/gpurun_out/mad_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/mad/write -o run -- $CMD > $R/gpurun_out/mad_write.log 2>&1
