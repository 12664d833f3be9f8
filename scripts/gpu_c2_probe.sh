#!/bin/bash
# GPU box, round 4: the C2 step's structure probe and the criterion's per-workgroup stamps.
#   Usage: bash scripts/gpu_c2_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/c2_probe.py --steps 400 --out gpurun_out/c2_probe_$TAG.jsonl \
    > gpurun_out/c2_probe_$TAG.log 2>&1 || exit 1
SBOD_LIB=$PWD/shape_based_object_detection_amd/lib/variants/libsbod_hip_stamps.so timeout -k 10 200 \
    python -u scripts/c2_stamps.py --out gpurun_out/c2_stamps_$TAG.json > gpurun_out/c2_stamps_$TAG.log 2>&1 || exit 1
echo done
