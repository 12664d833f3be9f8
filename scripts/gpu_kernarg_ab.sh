#!/bin/bash
# GPU box: the driver's 20-step command with the HIP runtime's kernel arguments in device memory
# (this runtime's default) vs host memory (HIP_FORCE_DEV_KERNARG=0), rounds alternating; then one
# 300-step run of each.
#   bash scripts/gpu_kernarg_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-5}
O=gpurun_out; mkdir -p $O
run() {  # name value steps
  local n=$1 v=$2 k=$3
  ( if [ -n "$v" ]; then export HIP_FORCE_DEV_KERNARG=$v; fi
    timeout -k 10 300 python -u bench.py --gpus 1 --steps $k --warmup 5 --no-dcn --no-cpu-baseline --no-c2 \
      > $O/ka_${TAG}_${n}_${k}_$r.json 2>> $O/ka_${TAG}.err ) || { echo "bench $n failed"; tail -5 $O/ka_${TAG}.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/ka_${TAG}_${n}_${k}_$r.json').read().strip().splitlines()[-1]); t=d['timed_run_detail']
print('$n $k r$r', d['ms_per_step'], t['submit_us_median'], t['submit_us_first4'], t['last_submit_to_end_us'], round(sum(d['kernel_us_per_step'].values()),1))"
}
for r in $(seq 1 $R); do
  run dev "" 20 || exit 1
  run host 0 20 || exit 1
done
r=0
run dev "" 300 || exit 1
run host 0 300 || exit 1
echo EXIT 0
