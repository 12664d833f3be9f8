#!/bin/bash
# GPU-side step interval: each step's criterion and detect on one stream (--shared-streams), steps
# spread over 2 / 4 streams, against the default layout (2 criterion + 2 detect streams).
set -o pipefail
O=gpurun_out/shared_streams_${1:-a}.jsonl
: > $O
run() {   # hw_queues args...
  q=$1; shift
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 "$@" \
      2>>gpurun_out/shared_streams.err | tail -1 >> $O || exit 1
}
for r in 1 2; do
  run 4 && run 4 --shared-streams --crit-streams 4 --batches 8 && run 8 --shared-streams --crit-streams 4 --batches 8 \
    && run 4 --shared-streams --crit-streams 3 --batches 6 && run 4 --shared-streams --crit-streams 2 --batches 6 || exit 1
done
cat $O
