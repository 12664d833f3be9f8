#!/bin/bash
# GPU box: the step's concurrent per-kernel timeline (stamps build), in the three modes.
#   bash scripts/gpu_timeline.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
for m in pipelined crit det; do
  SBOD_LIB=$PWD/variants/libsbod_hip_stamps.so timeout -k 10 120 python -u scripts/step_timeline.py --mode $m \
      >> gpurun_out/tl_$TAG.jsonl 2>> gpurun_out/tl_$TAG.err || exit 1
done
echo done
