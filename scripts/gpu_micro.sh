#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 300 python scripts/microbench.py "$@" > gpurun_out/micro_$TAG.json 2> gpurun_out/micro_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof_$TAG -o run --output-format csv -- \
    python scripts/microbench.py "$@" > gpurun_out/mprof_$TAG.log 2>&1
rc=$?; echo "EXIT $rc"; exit $rc
