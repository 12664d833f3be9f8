#!/bin/bash
# GPU box: phase clocks (printf from a few workgroups) and the per-workgroup timeline of the hot
# kernels, from the diagnostic libraries (build_phase_lib.sh / build_stamps_lib.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
LIBD=$PWD/shape_based_object_detection_amd/lib
VARD=$PWD/variants
mkdir -p gpurun_out
SBOD_LIB=$VARD/libsbod_hip_phase.so timeout -k 10 200 python scripts/phase_detect.py > gpurun_out/phase_$TAG.log 2>&1 && \
SBOD_LIB=$VARD/libsbod_hip_stamps.so timeout -k 10 120 python scripts/timeline.py > gpurun_out/timeline_$TAG.log 2>&1
rc=$?; echo "EXIT $rc"; exit $rc
