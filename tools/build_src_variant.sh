#!/bin/bash
# Build a variant of libabcgpu in which one csrc file is replaced by an
# edited copy (a same-box A/B of a kernel change, no build-time switches in
# the product sources):
#   bash tools/build_src_variant.sh ab/libv.so ab/abc_mvn_x3.v1.hip abc_mvn_x3.hip
# VARIANT_FLAGS in the environment: extra compiler flags for the edited file.
# Further arguments: edited headers, copied next to the source (they shadow
# the csrc headers of the same name).
set -e
OUT=$1; VSRC=$2; SRC=$3; shift 3
mkdir -p "$(dirname "$OUT")"
python -m pyabc_amd.build > /dev/null
OBJS=$(ls pyabc_amd/_build/*.o | grep -v "/$SRC.o")
EXTRA="$(python3 -c "import pyabc_amd.build as b; print(' '.join(b.EXTRA.get('$SRC', [])))") $VARIANT_FLAGS"
T=$(mktemp -d)
cp "$VSRC" $T/$SRC
for h in "$@"; do cp "$h" $T/; done
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I include -I pyabc_amd/csrc \
  -Wno-unused-result $EXTRA -c $T/$SRC -o "$OUT.$SRC.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS "$OUT.$SRC.o"
rm -rf "$OUT.$SRC.o" $T
echo "built $OUT ($SRC from $VSRC)"
