#!/bin/bash
# GPU box: the bench line and a rocprofv3 kernel-stats run of the same bench command.
#   bash scripts/gpu_bench.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
