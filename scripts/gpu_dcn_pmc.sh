#!/bin/bash
# GPU box: PMC passes (one rocprofv3 run per counter group) over the DCN forward+backward at
# H=64; optional probe-variant timings first.  Usage: gpu_dcn_pmc.sh TAG [variant ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
for v in "$@"; do
  SBOD_LIB=$PWD/shape_based_object_detection_amd/lib/libsbod_hip_$v.so timeout -k 10 120 \
    python scripts/dcn_bench.py --sizes 64 --iters 5 > gpurun_out/dcn_$v.json 2>&1 || exit 1
done
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/dpmc_${TAG}_$i -o run --output-format csv -- \
    python scripts/dcn_bench.py --sizes 64 --iters 1 --warmup 1 > gpurun_out/dpmc_${TAG}_$i.log 2>&1 || exit 1
done
echo done
