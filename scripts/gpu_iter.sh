#!/bin/bash
# GPU box, one iteration: -m gpu suite, block timeline (stamps lib), A/B microbench vs a variant
# library, phase clocks, bench line.  Stops at the first failure.
#   bash scripts/gpu_iter.sh TAG [VARIANT]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; VAR=${2:-old}
LIBD=$PWD/shape_based_object_detection_amd/lib
VARD=$PWD/variants
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/tests_$TAG.log 2>&1 && \
SBOD_LIB=$VARD/libsbod_hip_stamps.so timeout -k 10 120 python scripts/timeline.py > gpurun_out/timeline_$TAG.log 2>&1 && \
bash scripts/gpu_ab.sh $TAG $VAR
rc=$?; echo "EXIT $rc"; exit $rc
