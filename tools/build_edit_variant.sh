#!/bin/bash
# A/B variant of libabcgpu with one source edited by sed expressions (the
# tree's sources are copied, edited, and SRC recompiled), e.g.
#   bash tools/build_edit_variant.sh ab/libdm_w8.so abc_local.hip abc_local_dense.h \
#        's/constexpr int DM_W = 4;/constexpr int DM_W = 8;/'
set -e
OUT=$1; SRC=$2; EDITED=$3; shift 3
mkdir -p "$(dirname "$OUT")"
python -m pyabc_amd.build > /dev/null
T=$(mktemp -d)
mkdir -p $T/pyabc_amd $T/include
cp -r pyabc_amd/csrc $T/pyabc_amd/
cp include/*.h $T/include/
for e in "$@"; do sed -i "$e" $T/pyabc_amd/csrc/$EDITED; done
if cmp -s pyabc_amd/csrc/$EDITED $T/pyabc_amd/csrc/$EDITED; then echo "edit changed nothing"; exit 1; fi
OBJS=$(ls pyabc_amd/_build/*.o | grep -v "/$SRC.o")
EXTRA=${EXTRA_OVERRIDE-$(python3 -c "import pyabc_amd.build as b; print(' '.join(b.EXTRA.get('$SRC', [])))")}
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I include -Wno-unused-result $EXTRA \
  -c $T/pyabc_amd/csrc/$SRC -o "$OUT.$SRC.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS "$OUT.$SRC.o"
rm -rf "$OUT.$SRC.o" $T
echo "built $OUT"
