#!/bin/bash
# GPU box, round 4: the pipelined-step tests, then a same-box A/B of the submit path (direct
# recorded calls / one forked graph per step / two graphs per step), at 300 and at 20 steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/forkab_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/fork_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for sub in direct fork graph; do
    for k in 300 20; do
      timeout -k 10 300 python -u bench.py --steps $k --warmup 5 --no-dcn --no-cpu-baseline --submit $sub \
          > gpurun_out/forkab.tmp 2>> gpurun_out/fork_ab_$TAG.err || exit 1
      tail -1 gpurun_out/forkab.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); \
print(json.dumps({'submit': '$sub', 'steps': $k, 'ms_per_step': d['ms_per_step'], 'host': d.get('host_us_per_step'), \
'c2': d.get('c2_bf16', {}).get('ms_per_step')}))" >> $out || exit 1
    done
  done
done
echo done
