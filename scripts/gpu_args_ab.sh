#!/bin/bash
# GPU box: the -m gpu suite, then ab_base vs this tree (both with the GT fold), rounds alternating:
# 300-step runs (native submit phases) and the driver's 20-step command.
#   bash scripts/gpu_args_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-3}
O=$PWD/gpurun_out; mkdir -p $O
ROOT=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/atests_$TAG.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/atests_$TAG.log; exit 1; }
tail -1 $O/atests_$TAG.log
for r in $(seq 1 $R); do
  for t in ab_base .; do
    n=$( [ "$t" = "." ] && echo new || echo base )
    for k in 300 20; do
      ( cd $ROOT/$t && timeout -k 10 300 python -u bench.py --gpus 1 --steps $k --warmup 5 --no-dcn --no-cpu-baseline --no-c2 \
          --gt-fold 1 > $O/aa_${TAG}_${n}_${k}_$r.json 2>> $O/aa_$TAG.err ) || { echo "bench $n failed"; tail -5 $O/aa_$TAG.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/aa_${TAG}_${n}_${k}_$r.json').read().strip().splitlines()[-1]); t=d['timed_run_detail']
print('$n $k r$r', d['ms_per_step'], t['submit_us_median'], t.get('native_submit_us_per_step'))"
    done
  done
done
echo EXIT 0
