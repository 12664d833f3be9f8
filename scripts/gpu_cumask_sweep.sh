#!/bin/bash
# GPU-side step interval (scripts/gpu_interval.py) with the criterion streams CU-masked to leave
# K CUs to the detect chain (spread: every (256/K)-th CU id; block: the top K ids), two rounds.
set -o pipefail
O=gpurun_out/cumask_sweep_${1:-a}.jsonl
: > $O
run() {   # reserve mask
  timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 --crit-cu-reserve $1 --mask $2 \
      2>>gpurun_out/cumask_sweep.err | tail -1 >> $O || exit 1
}
for r in 1 2; do
  run 0 spread && run 16 spread && run 32 spread && run 64 spread && run 32 block && run 64 block || exit 1
done
cat $O
