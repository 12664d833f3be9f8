#!/bin/bash
# GPU box, round 4: the pipelined-step tests, then a same-box A/B (two rounds in turn) of the
# step's submit path and stream / hardware-queue count.   Usage: bash scripts/gpu_prog_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/prog_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/prog_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for f in "--submit graph" "--submit direct" "--crit-streams 3 --det-streams 3 --hw-queues 8" \
           "--crit-streams 4 --det-streams 4 --hw-queues 8 --depth 6"; do
    timeout -k 10 300 python -u bench.py --steps 400 --no-dcn --no-cpu-baseline $f \
        > gpurun_out/prog_bench.tmp 2>> gpurun_out/prog_ab_$TAG.err || exit 1
    tail -1 gpurun_out/prog_bench.tmp >> $out
  done
done
echo done
