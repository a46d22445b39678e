#!/bin/bash
# A/B timing of several builds of libabcgpu on one box (interleaved) with
# tools/bench_fused.py:  bash tools/ab_fused.sh "ab/lib0.so ab/lib1.so" [args]
LIBS=$1; shift
ARGS=${@:---rates 1e-2 1e-4 --modes plain --reps 3}
for rep in 1 2; do
  for L in $LIBS; do
    echo "== $L"
    ABCGPU_LIB=$L timeout -k 10 200 python -u tools/bench_fused.py $ARGS 2>&1 | grep -E "candidates/s|Error|error" || exit 1
  done
done
