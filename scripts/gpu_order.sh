#!/bin/bash
# GPU box: bench lines (no DCN, no CPU baseline, 300 steps) for each submit order x stream
# priority, two rounds, and the step timeline of each order.   bash scripts/gpu_order.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
for round in 1 2; do
  for o in criterion_first detect_first; do
    for p in detect criterion; do
      timeout -k 10 150 python -u bench.py --steps 300 --no-dcn --no-cpu-baseline --order $o --priority $p \
          >> gpurun_out/order_$TAG.jsonl 2>> gpurun_out/order_$TAG.err || exit 1
    done
  done
done
for o in criterion_first detect_first; do
  SBOD_LIB=$PWD/variants/libsbod_hip_stamps.so timeout -k 10 120 python -u scripts/step_timeline.py --order $o \
      >> gpurun_out/otl_$TAG.jsonl 2>> gpurun_out/otl_$TAG.err || exit 1
done
echo done
