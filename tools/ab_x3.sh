#!/bin/bash
# A/B timing of two builds of libabcgpu on the same box (interleaved):
#   A = ab/libA.so, B = the in-tree pyabc_amd/libabcgpu.so
# usage: bash tools/ab_x3.sh [bench_mvn args]
ARGS=${@:---prec x3+hint}
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then LIBV=ab/libA.so; else LIBV=pyabc_amd/libabcgpu.so; fi
    echo -n "$v: "
    ABCGPU_LIB=$LIBV timeout -k 10 200 python -u tools/bench_mvn.py $ARGS 2>/dev/null | grep kernel
  done
done
