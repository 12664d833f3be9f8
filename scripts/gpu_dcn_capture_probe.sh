#!/bin/bash
# GPU box, round 4: which DCN shapes / warm-up histories capture (scripts/dcn_capture_probe.py),
# least to most suspect; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
log=gpurun_out/dcn_capture_probe_${1:-run}.log
: > $log
for cfg in ${CFGS:-"16 256 256 8 2 0"}; do
  timeout -k 10 120 python -u scripts/dcn_capture_probe.py $cfg >> $log 2>&1 || { echo "FAIL $cfg rc $?" >> $log; exit 1; }
done
echo done
