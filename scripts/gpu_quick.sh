#!/bin/bash
# GPU box: full -m gpu suite, the phase-clock detect run, then a short bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu -x > gpurun_out/tests_$TAG.log 2>&1 && \
SBOD_LIB=$PWD/variants/libsbod_hip_phase.so timeout -k 10 200 \
    python scripts/phase_detect.py > gpurun_out/phase_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "EXIT $rc"; exit $rc
