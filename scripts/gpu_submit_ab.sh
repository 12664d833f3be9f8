#!/bin/bash
# GPU box, round 4: the pipelined-step tests (graph and direct submit), then a same-box A/B of
# graph replay vs direct (recorded-call) submit at pipeline depth 3 and 4 (two rounds in turn),
# then the DCN tests and maps.   Usage: bash scripts/gpu_submit_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dcn.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/submit_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/submit_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for f in "4 graph" "4 direct" "3 direct"; do
    set -- $f
    timeout -k 10 240 python -u bench.py --steps 400 --no-dcn --no-cpu-baseline --no-c2 --depth $1 --submit $2 \
        > gpurun_out/submit_bench.tmp 2>> gpurun_out/submit_ab_$TAG.err || exit 1
    tail -1 gpurun_out/submit_bench.tmp >> $out
  done
done
bash scripts/gpu_dcn_r4.sh $TAG nopmc
