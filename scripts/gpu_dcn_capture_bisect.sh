#!/bin/bash
# GPU box, round 4: which earlier DCN tests make the captured-DCN test crash in capture_end
# (a fresh process captures fine: scripts/dcn_capture_probe.py).  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
log=gpurun_out/dcn_capture_bisect_${1:-run}.log
: > $log
for k in "captured" "partial or state_backward or captured" "module_surface or captured" \
         "golden or against_oracle or captured" "c4 or captured"; do
  echo "=== -k $k" >> $log
  timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -m gpu -x -v -k "$k" --timeout 120 \
      --timeout-method thread >> $log 2>&1 || { echo "FAIL rc $? : $k" >> $log; exit 1; }
done
echo done
