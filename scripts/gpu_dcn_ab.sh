#!/bin/bash
# GPU box: DCN parity tests (current library), then dcn_bench at H=64 over variant libraries
# and the current one (two rounds in turn), then rocprofv3 kernel stats of the current one.
#   bash scripts/gpu_dcn_ab.sh TAG VARIANT [VARIANT...]   (lib/libsbod_hip_<VARIANT>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
LIBD=$PWD/shape_based_object_detection_amd/lib
VARD=$PWD/variants
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/dcntests_$TAG.log 2>&1 || { echo "EXIT tests"; exit 1; }
run() { echo "$1" >> gpurun_out/dcnab_$TAG.json; SBOD_LIB=$1 timeout -k 10 120 python scripts/dcn_bench.py --sizes 64 \
    >> gpurun_out/dcnab_$TAG.json 2>> gpurun_out/dcnab_$TAG.err; }
for round in 1 2; do
  for v in "$@"; do run $VARD/libsbod_hip_$v.so || { echo "EXIT ab"; exit 1; }; done
  run $LIBD/libsbod_hip.so || { echo "EXIT ab"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_$TAG -o run --output-format csv -- \
    python scripts/dcn_bench.py --sizes 64 --iters 3 --warmup 1 > gpurun_out/dprof_$TAG.log 2>&1
rc=$?; echo "EXIT $rc"; exit $rc
