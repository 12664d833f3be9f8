#!/bin/bash
# GPU box, round 4: DCN parity (incl. the fork-join capture test), then a same-box A/B of the DCN
# maps: the serial library (variant "serial") vs the default (side-stream fork/join), in turn.
#   Usage: bash scripts/gpu_dcn_fork_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/dcnfork_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/dcnfork_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  SBOD_LIB=$V/libsbod_hip_serial.so timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out \
      2>> gpurun_out/dcnfork_ab_$TAG.err || exit 1
  timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out 2>> gpurun_out/dcnfork_ab_$TAG.err || exit 1
done
echo done
