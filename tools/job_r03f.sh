#!/bin/bash
# deferred collect v2: LocalTransition tests + c5 traces, A/B against the
# select's own collect sweep (ab/libnodefer.so)
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
bash tools/gpu_local.sh || exit 1
bash tools/ab_local_fit.sh ab/libnodefer.so ab/libnodefer.so pyabc_amd/libabcgpu.so
