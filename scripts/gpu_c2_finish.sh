#!/bin/bash
# GPU box: config C2 (B=16 bf16) with the loss finish fused into the loss pass vs the separate
# one-block k_loss_final, rounds alternating (bench.py's c2_bf16 figure).
#   bash scripts/gpu_c2_finish.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-3}
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $R); do
  for f in fused separate; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 50 --warmup 10 --no-dcn --no-cpu-baseline --c2-finish $f \
        > $O/c2f_${TAG}_${f}_$r.json 2>> $O/c2f_$TAG.err || { echo "bench $f failed"; tail -5 $O/c2f_$TAG.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c2f_${TAG}_${f}_$r.json').read().strip().splitlines()[-1]); c=d['c2_bf16']
print('$f r$r', c['ms_per_step'], c['runs_ms_per_step'], c['roofline']['avg_us'], c['roofline']['frac'])"
  done
done
echo EXIT 0
