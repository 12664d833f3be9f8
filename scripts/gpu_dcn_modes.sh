#!/bin/bash
# GPU box (diagnostic): DCN 64x64 fwd+bwd eager vs hipGraph replay, each alone and under a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for m in eager graph eager graph; do timeout -k 10 120 python scripts/dcn_eager_graph.py --mode $m || exit 1; done
for m in eager graph; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/dmode_$m -o run --output-format csv -- \
    python scripts/dcn_eager_graph.py --mode $m > $O/dmode_$m.log 2>&1 || { tail -5 $O/dmode_$m.log; exit 1; }
  tail -1 $O/dmode_$m.log
done
echo EXIT 0
