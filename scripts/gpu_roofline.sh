#!/bin/bash
# GPU box: bench line, kernel-trace stats of the same command, the two PMC passes (FETCH_SIZE and
# WRITE_SIZE separately), and one pass of clock/occupancy counters (--kernel-trace/--stats only,
# no other trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python bench.py "$@" --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pmcf_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pmcw_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmcc_$TAG -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pmcc_$TAG.log 2>&1 && \
python scripts/pmc_traffic.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG --out gpurun_out/pmc_traffic_$TAG.json > /dev/null
rc=$?; echo "EXIT $rc"; exit $rc
