#!/bin/bash
# GPU box, round 4: the -m gpu suite (the given test files first), smoke(), the bench line and a
# rocprofv3 kernel-stats run of the same bench command.  Every GPU step has its own time limit;
# the chain stops at the first failure.
#   Usage: FIRST="tests/test_x.py ..." bash scripts/gpu_r4.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
ok=0
if [ -n "$FIRST" ]; then
  timeout -k 10 300 python -u -m pytest $FIRST -m gpu -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/tests_first_$TAG.log 2>&1 || ok=1
fi
[ $ok -eq 0 ] && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 && \
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 && \
    python3 scripts/roofline_check.py gpurun_out/bench_$TAG.json gpurun_out/prof_$TAG/run_kernel_trace.csv \
        gpurun_out/roofline_check_$TAG.json gpurun_out/prof_$TAG.log > /dev/null
rc=$?
[ $ok -ne 0 ] && rc=1
# SUBMIT=1: the host cost of each piece of the step's submit / collect (scripts/submit_probe.py)
if [ $rc -eq 0 ] && [ -n "$SUBMIT" ]; then
  timeout -k 10 180 python -u scripts/submit_probe.py --out gpurun_out/submit_probe_$TAG.json \
      > gpurun_out/submit_probe_$TAG.log 2>&1
  rc=$?
fi
# OVH=1: the profiler's per-dispatch cost (scripts/rocprof_overhead.py), plain then profiled
if [ $rc -eq 0 ] && [ -n "$OVH" ]; then
  timeout -k 10 180 python -u scripts/rocprof_overhead.py --out gpurun_out/ovh_plain_$TAG.json \
      > gpurun_out/ovh_$TAG.log 2>&1 && \
  timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/ovh_$TAG -o run --output-format csv -- \
      python3 scripts/rocprof_overhead.py --out gpurun_out/ovh_prof_$TAG.json >> gpurun_out/ovh_$TAG.log 2>&1 && \
  python3 scripts/rocprof_overhead.py --combine gpurun_out/ovh_plain_$TAG.json gpurun_out/ovh_prof_$TAG.json \
      gpurun_out/ovh_$TAG/run_kernel_trace.csv gpurun_out/rocprof_overhead_$TAG.json >> gpurun_out/ovh_$TAG.log 2>&1
  rc=$?
fi
echo "EXIT $rc"
exit $rc
