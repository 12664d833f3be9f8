#!/bin/bash
# GPU box: a subset (or all) of the -m gpu tests, then the bench line (+ optional extra bench args).
# Usage: bash scripts/gpu_r2.sh TAG "TEST_SELECTOR" [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
SEL=${1:-tests}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "EXIT $rc"
exit $rc
