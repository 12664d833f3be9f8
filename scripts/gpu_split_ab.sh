#!/bin/bash
# GPU box, round 4: the pipelined-step tests, then a same-box A/B of the criterion's matcher on a
# high-priority match stream (--crit-split 1) vs one criterion stream per step (0), 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/split_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/split_ab_$TAG.jsonl
: > $out
for r in 1 2 3; do
  for sp in 0 1; do
    for k in 300 20; do
      timeout -k 10 300 python3 bench.py --steps $k --warmup 5 --crit-split $sp --no-dcn --no-cpu-baseline --no-c2 \
          > gpurun_out/split.tmp 2>> gpurun_out/split_ab_$TAG.err || exit 1
      tail -1 gpurun_out/split.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); \
print(json.dumps({'split': $sp, 'steps': $k, 'ms': d['ms_per_step'], 'host': d['host_us_per_step']}))" >> $out || exit 1
    done
  done
done
echo done
