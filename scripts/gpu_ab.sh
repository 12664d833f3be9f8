#!/bin/bash
# GPU box: the -m gpu tests selected by K (pytest -k; "" = all), then per-kernel A/B of
# variant libraries vs the current one (scripts/kernel_ab.py, two rounds in turn).
#   bash scripts/gpu_ab.sh TAG "K" VARIANT [VARIANT...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} \
    > gpurun_out/tests_$TAG.log 2>&1 && \
bash scripts/gpu_kernel_ab.sh $TAG "$@"
rc=$?
echo "EXIT $rc"
exit $rc
