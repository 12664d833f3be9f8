#!/bin/bash
# GPU box: the driver's 20-step command, default vs the GT packing folded into the matcher
# (--gt-fold 1), rounds alternating; then one 300-step run of each.
#   bash scripts/gpu_fold20.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-6}
O=gpurun_out; mkdir -p $O
run() {  # name steps args...
  local n=$1 k=$2; shift 2
  timeout -k 10 300 python -u bench.py --gpus 1 --steps $k --warmup 5 --no-dcn --no-cpu-baseline --no-c2 "$@" \
      > $O/fo_${TAG}_${n}_${k}_$r.json 2>> $O/fo_${TAG}.err || { echo "bench $n failed"; tail -5 $O/fo_${TAG}.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/fo_${TAG}_${n}_${k}_$r.json').read().strip().splitlines()[-1]); t=d['timed_run_detail']
print('$n $k r$r', d['ms_per_step'], t['submit_us_median'], t['last_submit_to_end_us'], d['kernel_us_per_step'].get('k_match_tile'))"
}
for r in $(seq 1 $R); do
  run default 20 || exit 1
  run fold 20 --gt-fold 1 || exit 1
done
r=0
run default 300 || exit 1
run fold 300 --gt-fold 1 || exit 1
echo EXIT 0
