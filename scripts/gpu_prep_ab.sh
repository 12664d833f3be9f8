#!/bin/bash
# GPU box, round 4: DCN parity, then a same-box A/B of the DCN maps: x transpose and weight layouts
# as two launches (variant preold) vs one (k_dcn_prep), in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/prep_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/prep_ab_$TAG.jsonl
: > $out
for r in 1 2 3; do
  SBOD_LIB=$V/libsbod_hip_preold.so timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out \
      2>> gpurun_out/prep_ab_$TAG.err || exit 1
  timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out 2>> gpurun_out/prep_ab_$TAG.err || exit 1
done
echo done
