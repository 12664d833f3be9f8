#!/bin/bash
# GPU box: whole-tree A/B of the step — ab_base/ (a worktree of an earlier commit, built in place)
# against this tree, alternating: step_modes2.py (steady-state intervals) and the driver's
# 20-step bench command.
#   bash scripts/gpu_tree_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-2}
O=$PWD/gpurun_out; mkdir -p $O
ROOT=$PWD
for r in $(seq 1 $R); do
  for t in ab_base .; do
    n=$( [ "$t" = "." ] && echo new || echo base )
    ( cd $ROOT/$t && timeout -k 10 300 python -u scripts/step_modes2.py --steps 300 >> $O/tmodes_${TAG}_$n.json 2>> $O/tmodes_${TAG}.err ) || { echo "modes $n failed"; tail -5 $O/tmodes_${TAG}.err; exit 1; }
    ( cd $ROOT/$t && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 \
        > $O/tb20_${TAG}_${n}_$r.json 2>> $O/tb20_${TAG}.err ) || { echo "bench $n failed"; tail -5 $O/tb20_${TAG}.err; exit 1; }
    echo "$n r$r modes $(tail -1 $O/tmodes_${TAG}_$n.json | python -c 'import json,sys; d=json.load(sys.stdin); print({k:v for k,v in d["rep1"].items()})')"
    echo "$n r$r bench20 $(python $ROOT/scripts/bench_summary.py $O/tb20_${TAG}_${n}_$r.json | cut -c1-200)"
  done
done
echo EXIT 0
