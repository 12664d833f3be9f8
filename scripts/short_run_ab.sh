#!/bin/bash
# The driver's short bench command (20 timed steps, 5 warm-up) against the default and a long
# run on one box: how much of the short figure is pipeline fill / drain.
#   bash scripts/short_run_ab.sh TAG [extra bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
TAG=$1; shift
for i in 1 2 3; do
  for cfg in "20 5" "50 10" "300 10"; do
    set -- $cfg "$@"
    s=$1; w=$2; shift 2
    timeout -k 10 300 python -u bench.py --steps $s --warmup $w --no-cpu-baseline --no-dcn --no-c2 "$@" > $O/short_${TAG}_${s}_$i.json 2> $O/short_${TAG}_${s}_$i.err || { tail -20 $O/short_${TAG}_${s}_$i.err; exit 1; }
    python -c "
import json,sys
d=json.loads(open('$O/short_${TAG}_${s}_$i.json').read().strip().splitlines()[-1])
print('steps', $s, 'run', $i, 'ms', d['ms_per_step'], 'host', d.get('host_us_per_step'), 'detail', d.get('timed_run_detail'))"
  done
done
echo EXIT 0
