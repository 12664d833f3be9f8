#!/bin/bash
# GPU box: rocprofv3 kernel trace + stats of one bench run (extra bench args passed through).
# Usage: bash scripts/gpu_prof.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-dcn "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
