#!/bin/bash
# GPU box: cProfile of the bench step's host side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python scripts/host_profile.py > gpurun_out/hostprof_$TAG.txt 2>&1
rc=$?; echo "EXIT $rc"; exit $rc
