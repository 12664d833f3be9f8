#!/bin/bash
# Dispatch-floor probe on the GPU-side step interval: N empty kernels (1 or 2,048 workgroups) added
# to each step's criterion and detect streams.  Two rounds.
set -o pipefail
O=gpurun_out/null_probe_${1:-a}.jsonl
: > $O
run() {
  timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 "$@" 2>>gpurun_out/null_probe.err | tail -1 >> $O || exit 1
}
for r in 1 2; do
  run && run --null-kernels 1 --null-blocks 1 && run --null-kernels 2 --null-blocks 1 && \
    run --null-kernels 1 --null-blocks 2048 || exit 1
done
cat $O
