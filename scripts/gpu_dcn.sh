#!/bin/bash
# GPU box: DCN parity tests, DCN timing, then rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -q -x --timeout 120 --timeout-method thread > gpurun_out/dcntests_$TAG.log 2>&1 && \
timeout -k 10 300 python scripts/dcn_bench.py "$@" > gpurun_out/dcn_$TAG.json 2> gpurun_out/dcn_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_$TAG -o run --output-format csv -- \
    python scripts/dcn_bench.py --iters 3 --warmup 1 > gpurun_out/dprof_$TAG.log 2>&1
rc=$?; echo "EXIT $rc"; exit $rc
