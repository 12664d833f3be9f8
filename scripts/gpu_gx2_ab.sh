#!/bin/bash
# GPU box, round 4: DCN parity, then a same-box A/B of the dx gather's LDS staging (variant gxold:
# scalar writes, stride 64*VEC+1) vs the default (float4 writes, stride 64*VEC+8), in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gx2_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/gx2_ab_$TAG.jsonl
: > $out
for r in 1 2 3; do
  SBOD_LIB=$V/libsbod_hip_gxold.so timeout -k 10 200 python -u scripts/gx_ab.py gxold >> $out 2>> gpurun_out/gx2_ab_$TAG.err || exit 1
  timeout -k 10 200 python -u scripts/gx_ab.py default >> $out 2>> gpurun_out/gx2_ab_$TAG.err || exit 1
done
echo done
