#!/bin/bash
# Build a variant of libabcgpu whose source file SRC (and its headers) come
# from git revision REV, the rest from the working tree: the same-box A/B
# baseline of a kernel change.
#   bash tools/build_baseline.sh ab/libbase.so HEAD abc_local.hip
set -e
OUT=$1; REV=$2; SRC=$3
mkdir -p "$(dirname "$OUT")"
python -m pyabc_amd.build > /dev/null
T=$(mktemp -d)
mkdir -p $T/pyabc_amd/csrc $T/include
for f in $(git ls-tree --name-only $REV pyabc_amd/csrc/) $(git ls-tree --name-only $REV include/); do
  git show $REV:$f > $T/$f
done
OBJS=$(ls pyabc_amd/_build/*.o | grep -v "/$SRC.o")
EXTRA=$(python3 -c "import pyabc_amd.build as b; print(' '.join(b.EXTRA.get('$SRC', [])))")
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -I include -Wno-unused-result $EXTRA \
  -c $T/pyabc_amd/csrc/$SRC -o "$OUT.$SRC.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJS "$OUT.$SRC.o"
rm -rf "$OUT.$SRC.o" $T
echo "built $OUT ($SRC from $REV)"
