#!/bin/bash
# GPU box: DCN C4 fwd+bwd at 32/16/8 (scripts/dcn_maps.py) over split-K caps of the forward and
# slice caps of the weight gradient (tuning probe).   bash scripts/gpu_dcn_split.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
for fs in 64 16 8 4; do
  for ws in 64 8 4 2; do
    echo "{\"fwd_split_max\": $fs, \"wgrad_slices_max\": $ws}" >> gpurun_out/dsplit_$TAG.jsonl
    SBOD_DCN_FWD_SPLIT_MAX=$fs SBOD_DCN_WGRAD_SLICES_MAX=$ws timeout -k 10 120 python -u scripts/dcn_maps.py --maps 32,16,8 --iters 10 \
        >> gpurun_out/dsplit_$TAG.jsonl 2>> gpurun_out/dsplit_$TAG.err || exit 1
  done
done
echo "EXIT 0"
