#!/bin/bash
# usage: gpuq.sh OUTFILE TIMEOUT CMD...  -- retries only when the pool had no free slot (nothing ran)
out=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" $out && grep -q "nothing was charged" $out; }; then
    echo "[gpuq] slot busy, retry $i" >> $out.retries; sleep 150; continue
  fi
  break
done
echo "[gpuq] rc=$rc" >> $out
