#!/bin/bash
# Host wait mode (hipSetDeviceFlags schedule: runtime default vs spin vs yield) at the driver's 20
# timed steps and at 300, REPS rounds alternating on one box.   bash scripts/sync_ab.sh TAG [REPS]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out; mkdir -p $O
TAG=$1; REPS=${2:-4}
for i in $(seq 1 $REPS); do
  for m in auto spin yield; do
    for s in 20 300; do
      f=$O/sy_${TAG}_${m}_${s}_$i
      timeout -k 10 300 python -u bench.py --steps $s --warmup 5 --no-cpu-baseline --no-dcn --no-c2 --sync $m > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); r=d['timed_run_detail']
print('$m', $s, $i, d['ms_per_step'], 'submit', d['host_us_per_step'], 'first', r['submit_us_first4'], 'tail', r['last_submit_to_end_us'], 'api', d.get('api_ms_per_step'))"
    done
  done
done
echo EXIT 0
