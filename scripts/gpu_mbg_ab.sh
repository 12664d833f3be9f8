#!/bin/bash
# GPU box, round 4: criterion parity, then a same-box A/B of the focal gradient loop without the
# per-slot one-hot selects (default) vs with them (variant mbold): criterion kernels alone
# (scripts/mb_ab.py) and the bench step, three rounds in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_criteria.py tests/test_gpu_criterion_fused.py tests/test_gpu_bf16.py \
    tests/test_gpu_multibox_tiles.py tests/test_gpu_c1.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/mbg_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/mbg_ab_$TAG.jsonl
: > $out
for r in 1 2 3; do
  SBOD_LIB=$V/libsbod_hip_mbold.so timeout -k 10 200 python -u scripts/mb_ab.py mbold >> $out 2>> gpurun_out/mbg_ab_$TAG.err || exit 1
  timeout -k 10 200 python -u scripts/mb_ab.py default >> $out 2>> gpurun_out/mbg_ab_$TAG.err || exit 1
done
echo done
