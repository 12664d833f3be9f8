#!/bin/bash
# GPU box: criterion/detect GPU tests, host-time breakdown, bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_criteria.py tests/test_gpu_operators.py -q -x > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 240 python scripts/host_breakdown.py > gpurun_out/hostbd_$TAG.json 2> gpurun_out/hostbd_$TAG.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "EXIT $rc"; exit $rc
