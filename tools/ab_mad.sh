#!/bin/bash
# Same-box A/B of column-MAD variants (tools/build_src_variant.sh libraries):
# the MAD/adaptive GPU tests, then the c4 component bench line, per library.
#   bash tools/ab_mad.sh LIB...
export PYTHONPATH=$PWD
for L in "$@"; do
  echo "== $L"
  ABCGPU_LIB=$L timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_rows.py -k "mad or MAD or adaptive" 2>&1 | tail -1 || exit 1
  ABCGPU_LIB=$L timeout -k 10 120 python3 -u tools/bench_components.py --only c4 2>&1 | grep "MAD" | cut -c1-200 || exit 1
done
