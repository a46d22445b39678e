export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cu -o run -- python3 tools/probes/custom_model_c2.py 20 user > gpurun_out/cu_trace.log 2>&1 || { tail -5 gpurun_out/cu_trace.log; exit 1; }
f=$(find /tmp/cu -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/custom_user_kernel_stats_after.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:14]:
    print('%-70s %6s %10.3f ms total %8.1f us avg' % (r['Name'][:70], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e3))"
