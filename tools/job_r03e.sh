#!/bin/bash
# round 3: deferred-collect LocalTransition fit (tests + c5 traces), then the
# k-NN sweep A/B (k-block-major MFMA order) and the filter_below bench sweep
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD
bash tools/gpu_local.sh || exit 1
bash tools/job_r03d.sh
