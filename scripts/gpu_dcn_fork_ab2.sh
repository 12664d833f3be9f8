#!/bin/bash
# GPU box, round 4: same-box A/B of the DCN maps (serial library vs side-stream fork/join, eager
# figures), then the fork-join capture test on the serial library (does the capture crash
# without the fork too?).   Usage: bash scripts/gpu_dcn_fork_ab2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
out=gpurun_out/dcnfork_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  SBOD_LIB=$V/libsbod_hip_serial.so timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out \
      2>> gpurun_out/dcnfork_ab_$TAG.err || exit 1
  timeout -k 10 240 python -u scripts/dcn_maps.py --iters 10 >> $out 2>> gpurun_out/dcnfork_ab_$TAG.err || exit 1
done
SBOD_LIB=$V/libsbod_hip_serial.so timeout -k 10 200 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -v \
    -k fork_join --timeout 120 --timeout-method thread > gpurun_out/dcnfork_serialtest_$TAG.log 2>&1
echo "serial test rc $?"
