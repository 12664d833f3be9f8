#!/bin/bash
# GPU box: SQ/LDS counter passes (one rocprofv3 run per group) over a short bench step run.
# Usage: gpu_step_pmc.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_BUSY_CU_CYCLES"
i=0
if [ -n "$ONLY_ACTIVE" ]; then LIST=("$P3"); else LIST=("$P1" "$P2" "$P3"); fi
for P in "${LIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/spmc_${TAG}_$i -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 3 --no-dcn --no-cpu-baseline > gpurun_out/spmc_${TAG}_$i.log 2>&1 || exit 1
done
echo done
