#!/bin/bash
# GPU-side step interval with each step's detect on the criterion's batch (offset 0, the bench) or
# on another resident batch (offset 3): whether the two reads of one batch's scores share the
# Infinity Cache.  Three alternating rounds.
set -o pipefail
O=gpurun_out/detect_offset_${1:-a}.jsonl
: > $O
for r in 1 2 3; do
  for k in 0 3; do
    timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 --detect-offset $k 2>>gpurun_out/detect_offset.err \
        | tail -1 >> $O || exit 1
  done
done
cat $O
