#!/bin/bash
# GPU box: the -m gpu suite, then the bench line + rocprofv3 kernel stats (stops at the first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu -x > gpurun_out/tests_$TAG.log 2>&1 && \
bash scripts/gpu_bench_profile.sh "$TAG" "$@"
rc=$?
echo "EXIT $rc"
exit $rc
