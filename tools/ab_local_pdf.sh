#!/bin/bash
# c5 LocalTransition density (1e5 x 1e5) per library: bench_components c5's pdf line.
export PYTHONPATH=$PWD
for L in "$@"; do
  echo "== $L $(ABCGPU_LIB=$L timeout -k 10 200 python3 -u tools/bench_components.py --only c5 2>&1 | grep 'LocalTransition.pdf' | cut -c1-140)"
done
