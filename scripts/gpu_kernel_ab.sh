#!/bin/bash
# GPU box: kernel_ab.py over variant libraries and the current one, two rounds in turn.
#   bash scripts/gpu_kernel_ab.sh TAG VARIANT [VARIANT...]   (lib/libsbod_hip_<VARIANT>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
LIBD=$PWD/shape_based_object_detection_amd/lib
VARD=$PWD/variants
mkdir -p gpurun_out
run() { SBOD_LIB=$1 timeout -k 10 120 python scripts/kernel_ab.py >> gpurun_out/kab_$TAG.json 2>> gpurun_out/kab_$TAG.err; }
rc=0
for round in 1 2; do
  for v in "$@"; do run $VARD/libsbod_hip_$v.so || { rc=$?; break 2; }; done
  run $LIBD/libsbod_hip.so || { rc=$?; break; }
done
echo "EXIT $rc"; exit $rc
