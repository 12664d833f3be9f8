#!/bin/bash
# GPU box: the driver's 20-step command under several bench flag sets, alternating round by round.
#   bash scripts/gpu_flag_ab.sh TAG ROUNDS "FLAGS A" "FLAGS B" ...   ("-" = no flags)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=$2; shift 2
O=gpurun_out; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for f in "$@"; do
    i=$((i+1)); fl="$f"; [ "$fl" = "-" ] && fl=""
    timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 $fl \
        > $O/fab_${TAG}_${i}_$r.json 2>> $O/fab_${TAG}.err || { echo "bench [$f] failed"; tail -5 $O/fab_${TAG}.err; exit 1; }
    echo "[$f] r$r $(python scripts/bench_summary.py $O/fab_${TAG}_${i}_$r.json | cut -c1-120)"
  done
done
echo EXIT 0
