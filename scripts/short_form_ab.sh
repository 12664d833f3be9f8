#!/bin/bash
# The driver's command (20 timed steps, 5 warm-up) for the launch-count forms, REPS rounds
# alternating on one box: which default serves the short figure best.
#   bash scripts/short_form_ab.sh TAG [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
TAG=$1; REPS=${2:-5}
declare -A CFG=([base]="--finish separate --gt-fold 0 --det-form two" [fin]="--finish fused --gt-fold 0 --det-form two"
                [all]="--finish fused --gt-fold 1 --det-form one")
for i in $(seq 1 $REPS); do
  for c in base fin all; do
    f=$O/sf_${TAG}_${c}_$i
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dcn --no-c2 ${CFG[$c]} > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); r=d['timed_run_detail']
print('$c', $i, d['ms_per_step'], 'submit', d['host_us_per_step']['submit'], 'span', r['steps_span_us'], 'tail', r['last_submit_to_end_us'])"
  done
done
echo EXIT 0
