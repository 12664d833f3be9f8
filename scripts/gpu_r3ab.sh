#!/bin/bash
# GPU box, round 3: -m gpu suite, smoke, per-kernel A/B of variant libraries vs the current one
# (scripts/kernel_ab.py, two rounds), the bench line, and its rocprofv3 kernel-stats run.
#   bash scripts/gpu_r3ab.sh TAG VARIANT [VARIANT...] -- [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out
SBOD_TOL_PROBE=$PWD/gpurun_out/tol_$TAG.jsonl timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1 && \
bash scripts/gpu_kernel_ab.sh $TAG "${VARS[@]}" && \
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "EXIT $rc"
exit $rc
