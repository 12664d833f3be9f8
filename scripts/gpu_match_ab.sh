#!/bin/bash
# GPU box: matcher-related -m gpu tests, per-kernel A/B of variant libraries (kernel_ab.py:
# default, each variant, default again), then a bench line.
#   bash scripts/gpu_match_ab.sh TAG "TEST FILES" VAR1 [VAR2 ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
SEL=$1; shift
LIBD=$PWD/shape_based_object_detection_amd/lib
VARD=$PWD/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { echo "TESTS FAILED"; exit 1; }
ab() { SBOD_LIB=$1 timeout -k 10 120 python scripts/kernel_ab.py >> gpurun_out/kab_$TAG.json 2>> gpurun_out/kab_$TAG.err; }
ab $LIBD/libsbod_hip.so || exit 1
for v in "$@"; do ab $VARD/libsbod_hip_$v.so || exit 1; done
ab $LIBD/libsbod_hip.so || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-dcn > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "EXIT $rc"; exit $rc
