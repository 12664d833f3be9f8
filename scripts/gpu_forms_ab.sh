#!/bin/bash
# GPU box, round 4: same-box A/B of the criterion / detect forms inside the bench step (two rounds
# in turn), after the tests that cover both forms.   Usage: bash scripts/gpu_forms_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect_fused.py tests/test_gpu_criterion_fused.py \
    tests/test_gpu_graph.py tests/test_gpu_loss_finish.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/forms_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/forms_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for f in "two two" "one two" "two one"; do
    set -- $f
    timeout -k 10 240 python -u bench.py --steps 200 --no-dcn --no-cpu-baseline --no-c2 --crit-form $1 --det-form $2 \
        > gpurun_out/forms_bench.tmp 2>> gpurun_out/forms_ab_$TAG.err || exit 1
    tail -1 gpurun_out/forms_bench.tmp >> $out
  done
done
echo done
