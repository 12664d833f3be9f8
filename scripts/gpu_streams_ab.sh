#!/bin/bash
# GPU box, round 4: tests touching the bench step and DCN, then a same-box A/B of one vs two
# criterion streams in the bench step (two rounds in turn), then the DCN per-map kernel trace.
#   Usage: bash scripts/gpu_streams_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dcn.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/streams_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/streams_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for n in 1 2; do
    timeout -k 10 240 python -u bench.py --steps 300 --no-dcn --no-cpu-baseline --no-c2 --crit-streams $n \
        > gpurun_out/streams_bench.tmp 2>> gpurun_out/streams_ab_$TAG.err || exit 1
    tail -1 gpurun_out/streams_bench.tmp >> $out
  done
done
bash scripts/gpu_dcn_r4.sh $TAG nopmc
