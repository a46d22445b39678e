#!/bin/bash
# Build a variant of libabcgpu with one source recompiled under extra flags,
# for on-box A/B timing (tools/ab_fused.sh):
#   bash tools/build_variant.sh ab/libcg2.so abc_fused.hip -DABC_FR_CG=2
set -e
OUT=$1; SRC=$2; shift 2
mkdir -p "$(dirname "$OUT")"
python -m pyabc_amd.build > /dev/null
OBJS=$(ls pyabc_amd/_build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I include -Wno-unused-result "$@" \
  -c pyabc_amd/csrc/$SRC -o "$OUT.$SRC.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS "$OUT.$SRC.o"
rm -f "$OUT.$SRC.o"
echo "built $OUT"
