#!/bin/bash
# GPU box: scripts/gpu_r3.sh (suite, smoke, bench line, rocprofv3 stats), then the DCN C4 64x64
# figure of the `head` variant vs the current library, two rounds in turn.
#   bash scripts/gpu_full_dcnab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
bash scripts/gpu_r3.sh $TAG && \
for v in $PWD/variants/libsbod_hip_head.so $PWD/shape_based_object_detection_amd/lib/libsbod_hip.so \
         $PWD/variants/libsbod_hip_head.so $PWD/shape_based_object_detection_amd/lib/libsbod_hip.so; do
  echo "$v" >> gpurun_out/dcnab_$TAG.json
  SBOD_LIB=$v timeout -k 10 150 python scripts/dcn_bench.py --sizes 64 >> gpurun_out/dcnab_$TAG.json 2>> gpurun_out/dcnab_$TAG.err || exit 1
done
rc=$?
echo "EXIT $rc"
exit $rc
