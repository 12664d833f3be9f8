#!/bin/bash
# GPU box, round 4: bf16 parity tests on the default library, then a same-box A/B of the criterion
# kernels (scripts/mb_ab.py) over library variants in turn, then the phase-clock build's per-tile
# phase stamps.   Usage: bash scripts/gpu_mb_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
V=$PWD/shape_based_object_detection_amd/lib/variants
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_criterion_fused.py tests/test_gpu_gt_fold.py \
    -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/mb_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/mb_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for lib in base default w0; do
    if [ $lib = default ]; then
      timeout -k 10 200 python -u scripts/mb_ab.py default >> $out 2>> gpurun_out/mb_ab_$TAG.err || exit 1
    else
      SBOD_LIB=$V/libsbod_hip_$lib.so timeout -k 10 200 python -u scripts/mb_ab.py $lib >> $out \
          2>> gpurun_out/mb_ab_$TAG.err || exit 1
    fi
  done
done
SBOD_LIB=$V/libsbod_hip_phase.so timeout -k 10 200 python -u scripts/mb_ab.py phase > gpurun_out/mb_phase_$TAG.log 2>&1 || exit 1
echo done
