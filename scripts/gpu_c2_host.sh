#!/bin/bash
# GPU box, round 4: why the C2 step's host submit is slower than the headline's — batch size,
# resident-batch count, dtype and Python's GC in turn (scripts/c2_probe.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/c2_probe.py --steps 400 --rounds 2 --out gpurun_out/c2_host_$TAG.jsonl --variants \
  '[{"B":32,"dtype":"f32","n_batches":6,"gt_fold":false},{"B":16,"dtype":"f32","n_batches":6,"gt_fold":false},
    {"B":16,"dtype":"f32","n_batches":12,"gt_fold":false},{"B":16,"dtype":"bf16","n_batches":12},
    {"B":16,"dtype":"bf16","n_batches":12,"nogc":true},{"B":16,"dtype":"bf16","n_batches":6}]' \
  > gpurun_out/c2_host_$TAG.log 2>&1 || exit 1
echo done
