#!/bin/bash
# GPU box, round 4: DeformConv2d per map size under a rocprofv3 kernel trace (per-kernel split,
# grid sizes tell the maps apart), then the PMC passes at H=64 (MFMA busy, waits, FETCH, WRITE).
#   Usage: bash scripts/gpu_dcn_r4.sh TAG [nopmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dtr_$TAG -o run --output-format csv -- \
    python3 scripts/dcn_maps.py --iters 10 > gpurun_out/dcn_maps_$TAG.jsonl 2> gpurun_out/dcn_maps_$TAG.err || exit 1
[ "$2" = "nopmc" ] && { echo done; exit 0; }
bash scripts/gpu_dcn_pmc.sh $TAG || exit 1
echo done
