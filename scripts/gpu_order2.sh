#!/bin/bash
# GPU box: bench lines (no DCN / CPU baseline, 300 steps) for criterion_first vs detect_early,
# three rounds in turn, then the step timeline of detect_early.   bash scripts/gpu_order2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
for round in 1 2 3; do
  for o in criterion_first detect_early; do
    timeout -k 10 150 python -u bench.py --steps 300 --no-dcn --no-cpu-baseline --order $o \
        >> gpurun_out/o2_$TAG.jsonl 2>> gpurun_out/o2_$TAG.err || exit 1
  done
done
SBOD_LIB=$PWD/variants/libsbod_hip_stamps.so timeout -k 10 120 python -u scripts/step_timeline.py --order detect_early \
    >> gpurun_out/o2tl_$TAG.jsonl 2>> gpurun_out/o2tl_$TAG.err
echo "EXIT $?"
