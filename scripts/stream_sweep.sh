#!/bin/bash
# Streams / depth / hardware queues sweep of the headline step (300 timed steps, REPS rounds).
#   bash scripts/stream_sweep.sh TAG [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
TAG=$1; REPS=${2:-2}
declare -A CFG=([s224]="--crit-streams 2 --det-streams 2 --depth 4" [s226]="--crit-streams 2 --det-streams 2 --depth 6"
                [s336]="--crit-streams 3 --det-streams 3 --depth 6 --hw-queues 8" [s448]="--crit-streams 4 --det-streams 4 --depth 8 --hw-queues 16"
                [s223]="--crit-streams 2 --det-streams 2 --depth 3")
for i in $(seq 1 $REPS); do
  for c in s224 s226 s336 s448 s223; do
    f=$O/ss_${TAG}_${c}_$i
    timeout -k 10 300 python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-dcn --no-c2 ${CFG[$c]} > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
    python -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1])
print('$c', $i, d['ms_per_step'], d['host_us_per_step'], d['kernel_us_per_step'].get('k_multibox'))"
  done
done
echo EXIT 0
