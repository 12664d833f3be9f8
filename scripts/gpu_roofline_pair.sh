#!/bin/bash
# GPU box, round 4: the headline roofline's two measurements from the same idle state — the bench
# line (HIP events) and the rocprofv3 trace of the same command — each after a 20 s pause (the
# profiled run otherwise follows a full bench run and the test suite), then the line's window
# check; a second unprofiled line closes the sequence.   Usage: bash scripts/gpu_roofline_pair.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
sleep 20 && \
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/pair_bench_$TAG.json 2> gpurun_out/pair_bench_$TAG.err && \
sleep 20 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pair_prof_$TAG -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline "$@" > gpurun_out/pair_prof_$TAG.log 2>&1 && \
python3 scripts/roofline_check.py gpurun_out/pair_bench_$TAG.json gpurun_out/pair_prof_$TAG/run_kernel_trace.csv \
    gpurun_out/pair_roofline_check_$TAG.json gpurun_out/pair_prof_$TAG.log > /dev/null && \
sleep 20 && \
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/pair_bench2_$TAG.json 2> gpurun_out/pair_bench2_$TAG.err
echo "EXIT $?"
