# kernel-trace stats of the c4 component bench for variant libraries
#   bash tools/ab_kernels.sh ab/libsel_v3.so ...   (-> gpurun_out/abk_<name>)
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  ABCGPU_LIB=$R/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abk_$n -o run -- python3 $R/tools/bench_components.py --only c4 --reps 2 > $R/gpurun_out/abk_$n.log 2>&1
done
