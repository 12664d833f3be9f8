#!/bin/bash
# GPU box, round 4: the pipelined-step tests, then a same-box A/B of the bench step's pipeline
# depth and criterion streams (two rounds in turn), and the submit-cost probe.
#   Usage: bash scripts/gpu_depth_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/depth_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/depth_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for f in "2 1 -" "2 2 -" "3 2 -" "4 2 -" "4 4 --one-stream"; do
    set -- $f
    o=$3; [ "$o" = "-" ] && o=
    timeout -k 10 240 python -u bench.py --steps 400 --no-dcn --no-cpu-baseline --no-c2 --depth $1 --crit-streams $2 $o \
        > gpurun_out/depth_bench.tmp 2>> gpurun_out/depth_ab_$TAG.err || exit 1
    tail -1 gpurun_out/depth_bench.tmp >> $out
  done
done
timeout -k 10 180 python -u scripts/submit_probe.py --out gpurun_out/submit_probe_$TAG.json > gpurun_out/submit_probe_$TAG.log 2>&1
# DCN: the tests, then the backward split by requested gradients (one kernel trace per subset)
[ -n "$DCN" ] || { echo done; exit 0; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/dcn_tests_$TAG.log 2>&1 || exit 1
for v in all weight x om; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/dv_${TAG}_$v -o run --output-format csv -- \
      python3 scripts/dcn_variants.py $v > gpurun_out/dv_${TAG}_$v.log 2>&1 || exit 1
done
bash scripts/gpu_dcn_r4.sh $TAG nopmc
