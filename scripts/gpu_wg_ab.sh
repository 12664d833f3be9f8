#!/bin/bash
# GPU box, round 4: same-box A/B of k_dcn_bwd_weight's target workgroup count (512 default, 768,
# 1024) over the DCN maps (scripts/dcn_maps.py), two rounds in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
out=gpurun_out/wg_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out 2>> gpurun_out/wg_ab_$TAG.err || exit 1
  for v in ${VARIANTS:-wg768 wg1024}; do
    SBOD_LIB=$V/libsbod_hip_$v.so timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out \
        2>> gpurun_out/wg_ab_$TAG.err || exit 1
  done
done
echo done
