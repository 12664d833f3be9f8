#!/bin/bash
# GPU box: the driver's 20-step command under the step's launch forms, rounds alternating:
# default (8 launches), GT packing folded into the matcher (--gt-fold 1), the loss finish fused
# into the loss pass (--finish fused), both.
#   bash scripts/gpu_forms20.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-3}
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $R); do
  for f in "default:" "fold:--gt-fold 1" "fused:--finish fused" "fold_fused:--gt-fold 1 --finish fused"; do
    n=${f%%:*}; args=${f#*:}
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 $args \
        > $O/f20_${TAG}_${n}_$r.json 2>> $O/f20_${TAG}.err || { echo "bench $n failed"; tail -5 $O/f20_${TAG}.err; exit 1; }
    echo "$n r$r $(python scripts/bench_summary.py $O/f20_${TAG}_${n}_$r.json | cut -c1-120)"
  done
done
echo EXIT 0
