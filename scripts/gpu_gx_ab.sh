#!/bin/bash
# GPU box, round 4: DCN parity on the gather variants' default, then a same-box A/B of the dx
# gather's block / rows-in-flight knobs (scripts/gx_ab.py), two rounds in turn.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
out=gpurun_out/gx_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  timeout -k 10 200 python -u scripts/gx_ab.py default >> $out 2>> gpurun_out/gx_ab_$TAG.err || exit 1
  for v in p8 r16 p8r16 p4r16; do
    SBOD_LIB=$V/libsbod_hip_gx_$v.so timeout -k 10 200 python -u scripts/gx_ab.py $v >> $out \
        2>> gpurun_out/gx_ab_$TAG.err || exit 1
  done
done
echo done
