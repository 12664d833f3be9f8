#!/bin/bash
# GPU box: A/B microbench of variant libraries on the same box (old, new, old again), then the
# phase-clock detect run and a bench line with the current library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
VAR=${1:-old}; shift
LIBD=$PWD/shape_based_object_detection_amd/lib
VARD=$PWD/variants
mkdir -p gpurun_out
run_mb() { SBOD_LIB=$1 timeout -k 10 200 python scripts/microbench.py --iters 200 >> gpurun_out/ab_$TAG.json 2>> gpurun_out/ab_$TAG.err; }
run_mb $VARD/libsbod_hip_$VAR.so && run_mb $LIBD/libsbod_hip.so && run_mb $VARD/libsbod_hip_$VAR.so && \
run_mb $LIBD/libsbod_hip.so && \
SBOD_LIB=$VARD/libsbod_hip_phase.so timeout -k 10 200 python scripts/phase_detect.py > gpurun_out/phase_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "EXIT $rc"; exit $rc
