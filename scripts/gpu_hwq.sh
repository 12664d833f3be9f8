#!/bin/bash
# GPU box: bench lines (no DCN / CPU baseline, 300 steps) with 4 (the box default) and 8 hardware
# queues per process, two rounds in turn.   bash scripts/gpu_hwq.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
for round in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python -u bench.py --steps 300 --no-dcn --no-cpu-baseline \
        | sed "s/^{/{\"hw_queues\": $q, /" >> gpurun_out/hwq_$TAG.jsonl 2>> gpurun_out/hwq_$TAG.err || exit 1
  done
done
echo "EXIT 0"
