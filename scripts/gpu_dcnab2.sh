#!/bin/bash
# GPU box: DCN parity tests, then the C4 64x64 figure of the `head` variant vs the current
# library, two rounds in turn.   bash scripts/gpu_dcnab2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/dcntests_$TAG.log 2>&1 && \
for v in $PWD/variants/libsbod_hip_head.so $PWD/shape_based_object_detection_amd/lib/libsbod_hip.so \
         $PWD/variants/libsbod_hip_head.so $PWD/shape_based_object_detection_amd/lib/libsbod_hip.so; do
  echo "$v" >> gpurun_out/dcnab_$TAG.json
  SBOD_LIB=$v timeout -k 10 150 python scripts/dcn_bench.py --sizes 64 >> gpurun_out/dcnab_$TAG.json 2>> gpurun_out/dcnab_$TAG.err || exit 1
done
rc=$?
echo "EXIT $rc"
exit $rc
