#!/bin/bash
# GPU box: selected -m gpu tests, then kernel_ab.py over variant libraries vs the current one.
#   bash scripts/gpu_iter2.sh TAG "TEST_SELECTOR" VARIANT [VARIANT...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
SEL=${1:-tests}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 && bash scripts/gpu_kernel_ab.sh $TAG "$@"
rc=$?; echo "EXIT $rc"; exit $rc
