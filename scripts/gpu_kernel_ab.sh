#!/bin/bash
# GPU box: kernel_ab.py alternating the variant library and the current one (old, new, old, new).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; VAR=${2:-old}
LIBD=$PWD/shape_based_object_detection_amd/lib
mkdir -p gpurun_out
run() { SBOD_LIB=$1 timeout -k 10 120 python scripts/kernel_ab.py >> gpurun_out/kab_$TAG.json 2>> gpurun_out/kab_$TAG.err; }
run $LIBD/libsbod_hip_$VAR.so && run $LIBD/libsbod_hip.so && run $LIBD/libsbod_hip_$VAR.so && run $LIBD/libsbod_hip.so
rc=$?; echo "EXIT $rc"; exit $rc
