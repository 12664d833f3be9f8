#!/bin/bash
# GPU box: the bench step under each stream priority x graph submit order, two rounds in turn
# (hot-path value only: no CPU baseline, DCN or C2 figures).   bash scripts/gpu_order_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
rc=0
for round in 1 2; do
  for pr in criterion detect none; do
    for od in criterion_first detect_first; do
      timeout -k 10 120 python bench.py --no-cpu-baseline --no-dcn --no-c2 --steps 300 --priority $pr --order $od \
        >> gpurun_out/order_$TAG.jsonl 2>> gpurun_out/order_$TAG.err || { rc=$?; break 3; }
    done
  done
done
echo "EXIT $rc"; exit $rc
