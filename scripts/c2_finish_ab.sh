#!/bin/bash
# C2 (B=16 bf16, host-bound) with the loss finish fused into the loss pass (one launch fewer per
# step) vs the separate finish launch; REPS rounds alternating on one box.
#   bash scripts/c2_finish_ab.sh TAG [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
TAG=$1; REPS=${2:-3}
for i in $(seq 1 $REPS); do
  for f in separate fused; do
    out=$O/c2f_${TAG}_${f}_$i
    timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dcn --c2-finish $f > $out.json 2> $out.err || { tail -20 $out.err; exit 1; }
    python -c "
import json; d=json.loads(open('$out.json').read().strip().splitlines()[-1]); c=d['c2_bf16']
print('$f', $i, 'c2', c['ms_per_step'], c['runs_ms_per_step'], c['roofline']['avg_us'], 'head', d['ms_per_step'])"
  done
done
echo EXIT 0
