#!/bin/bash
# GPU box: -m gpu suite, then A/B microbench vs a variant library, phase clocks, bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
VAR=${1:-old}; shift
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu -x > gpurun_out/tests_$TAG.log 2>&1 && \
bash scripts/gpu_ab.sh $TAG $VAR "$@"
rc=$?; echo "EXIT $rc"; exit $rc
