#!/bin/bash
# Launches per step vs the host-bound pipelined step: the default (8 launches + event), the loss
# finish in the loss pass (fused, -1), + the GT packing folded into the matcher (-1), + NMS and
# merge in one launch (-1); the driver's 20 timed steps and 300, REPS rounds on one box.
#   bash scripts/launch_count_ab.sh TAG [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
TAG=$1; REPS=${2:-2}
declare -A CFG=([base]="--finish separate --gt-fold 0 --det-form two" [fin]="--finish fused --gt-fold 0 --det-form two"
                [finfold]="--finish fused --gt-fold 1 --det-form two" [all]="--finish fused --gt-fold 1 --det-form one")
for i in $(seq 1 $REPS); do
  for c in base fin finfold all; do
    for s in 20 300; do
      f=$O/lc_${TAG}_${c}_${s}_$i
      timeout -k 10 300 python -u bench.py --steps $s --warmup 5 --no-cpu-baseline --no-dcn --no-c2 ${CFG[$c]} > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); r=d['timed_run_detail']
print('$c', $s, $i, d['ms_per_step'], 'submit', d['host_us_per_step'], 'native', r.get('native_submit_us_per_step',{}).get('total_us'), 'k', d['kernel_us_per_step'].get('k_multibox'), d['kernel_us_per_step'].get('k_match_tile'))"
    done
  done
done
echo EXIT 0
