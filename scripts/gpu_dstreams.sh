#!/bin/bash
# GPU box: bench lines (no DCN / CPU baseline, 300 steps) with 1 and 2 detect streams x priority,
# two rounds, then the step timeline with 2 detect streams.   bash scripts/gpu_dstreams.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
for round in 1 2; do
  for n in 1 2; do
    for p in detect criterion; do
      timeout -k 10 150 python -u bench.py --steps 300 --no-dcn --no-cpu-baseline --det-streams $n --priority $p \
          >> gpurun_out/ds_$TAG.jsonl 2>> gpurun_out/ds_$TAG.err || exit 1
    done
  done
done
SBOD_LIB=$PWD/variants/libsbod_hip_stamps.so timeout -k 10 120 python -u scripts/step_timeline.py --det-streams 2 \
    >> gpurun_out/dstl_$TAG.jsonl 2>> gpurun_out/dstl_$TAG.err
echo "EXIT $?"
