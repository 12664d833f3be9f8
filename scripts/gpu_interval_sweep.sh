#!/bin/bash
# GPU-side step interval (scripts/gpu_interval.py) over stream counts and hardware queues.
# One process per configuration; stops at the first failure.
set -o pipefail
O=gpurun_out/interval_sweep_${1:-a}.jsonl
: > $O
run() {   # hw_queues crit_streams det_streams batches
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 --crit-streams $2 \
      --det-streams $3 --batches $4 2>>gpurun_out/interval_sweep.err | tail -1 >> $O || exit 1
}
run 4 2 2 6 && run 4 2 3 6 && run 4 3 3 6 && run 8 2 2 6 && run 8 2 3 6 && run 8 3 3 6 && \
run 8 2 4 8 && run 8 4 4 8 && run 16 3 3 6 && run 16 4 4 8 && run 16 3 6 6
cat $O
