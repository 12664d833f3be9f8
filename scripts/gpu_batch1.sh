#!/bin/bash
# GPU box, one call: -m gpu suite + smoke; per-kernel A/B (step kernels) and DCN A/B of the
# `head` variant vs the current library; the submit-order x priority bench lines and timelines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1 && \
bash scripts/gpu_kernel_ab.sh $TAG head && \
for v in $PWD/variants/libsbod_hip_head.so $PWD/shape_based_object_detection_amd/lib/libsbod_hip.so \
         $PWD/variants/libsbod_hip_head.so $PWD/shape_based_object_detection_amd/lib/libsbod_hip.so; do
  echo "$v" >> gpurun_out/dcnab_$TAG.json
  SBOD_LIB=$v timeout -k 10 150 python scripts/dcn_bench.py --sizes 64 >> gpurun_out/dcnab_$TAG.json 2>> gpurun_out/dcnab_$TAG.err || exit 1
done && \
bash scripts/gpu_order.sh $TAG
rc=$?
echo "EXIT $rc"
exit $rc
