#!/bin/bash
# GPU-side step interval (scripts/gpu_interval.py) for the detect form (two launches / one) and
# the loss finish (separate k_loss_final / fused into k_multibox), alternated over two rounds.
set -o pipefail
O=gpurun_out/interval_forms_${1:-a}.jsonl
: > $O
run() {   # det_form finish
  timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 --det-form $1 --finish $2 \
      2>>gpurun_out/interval_forms.err | tail -1 >> $O || exit 1
}
for r in 1 2; do
  run two separate && run one separate && run two fused && run one fused || exit 1
done
cat $O
