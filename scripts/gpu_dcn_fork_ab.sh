#!/bin/bash
# GPU box: DCN tests, then the C4 maps (bench.dcn_figure: hipGraph replay + eager) in ab_base and
# this tree, rounds alternating.
#   bash scripts/gpu_dcn_fork_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-2}
O=$PWD/gpurun_out; mkdir -p $O
ROOT=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_dcn.py -q -x --timeout 300 --timeout-method thread \
   > $O/dtests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/dtests_$TAG.log; exit 1; }
tail -1 $O/dtests_$TAG.log
for r in $(seq 1 $R); do
  for t in ab_base .; do
    n=$( [ "$t" = "." ] && echo new || echo base )
    ( cd $ROOT/$t && timeout -k 10 300 python -u scripts/dcn_maps.py --iters 10 > $O/dmaps_${TAG}_${n}_$r.jsonl 2>> $O/dmaps_$TAG.err ) \
      || { echo "maps $n failed"; tail -5 $O/dmaps_$TAG.err; exit 1; }
    python -c "
import json
rows=[json.loads(l) for l in open('$O/dmaps_${TAG}_${n}_$r.jsonl')]
print('$n r$r', [(r['config'].split()[-3], r['ms'], r['mfma_frac'], r['eager_ms']) for r in rows])"
  done
done
echo EXIT 0
