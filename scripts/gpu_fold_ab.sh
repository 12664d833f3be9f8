#!/bin/bash
# GPU box, round 4: the GT-fold parity tests and the pipelined-step tests, then a same-box A/B (three
# rounds in turn) of the direct submit with the GT packing folded into the matcher (--gt-fold 1)
# and as its own launch (--gt-fold 0), plus a kernel trace of each form.
#   Usage: bash scripts/gpu_fold_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gt_fold.py tests/test_gpu_graph.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/fold_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/fold_ab_$TAG.jsonl
: > $out
for r in 1 2 3; do
  for f in 1 0; do
    timeout -k 10 300 python -u bench.py --steps 400 --no-dcn --no-cpu-baseline --gt-fold $f \
        > gpurun_out/fold_bench.tmp 2>> gpurun_out/fold_ab_$TAG.err || exit 1
    tail -1 gpurun_out/fold_bench.tmp >> $out
  done
done
for f in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fold_prof_${TAG}_$f -o run --output-format csv \
      -- python3 bench.py --steps 200 --no-dcn --no-cpu-baseline --gt-fold $f > gpurun_out/fold_prof_$f.log 2>&1 || exit 1
done
echo done
