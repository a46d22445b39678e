#!/bin/bash
# round 3 final GPU call: LocalTransition tests + c5 traces with the deferred
# collect, its A/B against the select's own collect sweep, then the round
# check (smoke, the whole -m gpu suite, the driver's bench command, the
# custom-model probe)
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
bash tools/gpu_local.sh || exit 1
bash tools/ab_local_fit.sh ab/libnodefer.so || exit 1
bash tools/gpu_round.sh
