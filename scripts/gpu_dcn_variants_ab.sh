#!/bin/bash
# GPU box, round 4: DeformConv2d fwd+bwd at C4's 64x64 map over A/B variant libraries
# (lib/variants/libsbod_hip_<V>.so) and the tree's library, two rounds in turn, plus one kernel
# trace per library.   Usage: bash scripts/gpu_dcn_variants_ab.sh TAG V [V...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
LIBD=$PWD/shape_based_object_detection_amd/lib
mkdir -p gpurun_out
out=gpurun_out/dcnvar_$TAG.jsonl
: > $out
run() { echo "{\"lib\": \"$1\"}" >> $out; SBOD_LIB=$1 timeout -k 10 120 python scripts/dcn_bench.py --sizes 64 \
    >> $out 2>> gpurun_out/dcnvar_$TAG.err; }
for round in 1 2; do
  for v in "$@"; do run $LIBD/variants/libsbod_hip_$v.so || exit 1; done
  run $LIBD/libsbod_hip.so || exit 1
done
for v in "$@"; do
  SBOD_LIB=$LIBD/variants/libsbod_hip_$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/dvt_${TAG}_$v \
      -o run --output-format csv -- python3 scripts/dcn_variants.py all > gpurun_out/dvt_${TAG}_$v.log 2>&1 || exit 1
done
echo done
