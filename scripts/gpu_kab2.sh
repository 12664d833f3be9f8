#!/bin/bash
# GPU box: per-kernel event times (scripts/kernel_ab.py) of ab_base and this tree, alternating.
#   bash scripts/gpu_kab2.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-2}
O=$PWD/gpurun_out; mkdir -p $O
for r in $(seq 1 $R); do
  for t in ab_base .; do
    ( cd $t && timeout -k 10 150 python scripts/kernel_ab.py ) >> $O/kab2_$TAG.json 2>> $O/kab2_$TAG.err || { echo "kab failed"; tail -5 $O/kab2_$TAG.err; exit 1; }
  done
done
cat $O/kab2_$TAG.json
