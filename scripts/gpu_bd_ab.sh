#!/bin/bash
# GPU box, round 4: DCN parity (small maps take 32-pixel k_dcn_bwd_data blocks), then a same-box
# A/B of the DCN maps: 64-pixel blocks everywhere (variant bd64) vs the default, in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/bd_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/bd_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  SBOD_LIB=$V/libsbod_hip_bd64.so timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 --maps 16,8 >> $out \
      2>> gpurun_out/bd_ab_$TAG.err || exit 1
  timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 --maps 16,8 >> $out 2>> gpurun_out/bd_ab_$TAG.err || exit 1
  SBOD_LIB=$V/libsbod_hip_bd64.so timeout -k 10 200 python -u scripts/gx_ab.py bd64 >> $out 2>> gpurun_out/bd_ab_$TAG.err || exit 1
  timeout -k 10 200 python -u scripts/gx_ab.py default >> $out 2>> gpurun_out/bd_ab_$TAG.err || exit 1
done
echo done
