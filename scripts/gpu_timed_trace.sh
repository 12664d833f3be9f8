#!/bin/bash
# GPU box: rocprofv3 kernel traces of the bench's timed region at 20 and 300 steps, summarised by
# scripts/timed_trace.py (dispatches inside the line's timed_window_ns).
#   bash scripts/gpu_timed_trace.sh TAG [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out; mkdir -p $O
for n in 20 300; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tt_${TAG}_$n -o run --output-format csv -- \
      python bench.py --steps $n --warmup 5 --no-dcn --no-c2 --no-cpu-baseline "$@" > $O/tt_${TAG}_$n.log 2>&1 \
      || { echo "trace $n failed"; tail -20 $O/tt_${TAG}_$n.log; exit 1; }
  python scripts/timed_trace.py $O/tt_${TAG}_$n.log $O/tt_${TAG}_$n/run_kernel_trace.csv --list > $O/tt_${TAG}_$n.txt || exit 1
  head -60 $O/tt_${TAG}_$n.txt
done
echo EXIT 0
