#!/bin/bash
# GPU box: criterion-side parity tests, then the whole-tree A/B against ab_base (kernel_ab.py in
# both trees, step_modes2.py and the 20-step bench alternating).
#   bash scripts/gpu_crit_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-2}
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_criteria.py tests/test_gpu_match.py tests/test_gpu_bf16.py tests/test_gpu_operators.py \
   tests/test_gpu_loss_finish.py tests/test_gpu_c1.py tests/test_gpu_c5.py tests/test_gpu_api_fast.py tests/test_gpu_gt_fold.py tests/test_gpu_stress.py tests/test_gpu_graph.py -q -x \
   --timeout 200 --timeout-method thread > $O/ctests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/ctests_$TAG.log; exit 1; }
tail -1 $O/ctests_$TAG.log
for t in ab_base .; do
  n=$( [ "$t" = "." ] && echo new || echo base )
  ( cd $t && timeout -k 10 150 python scripts/kernel_ab.py ) >> $O/ckab_$TAG.json 2>> $O/ckab_$TAG.err || { echo "kab failed"; tail -5 $O/ckab_$TAG.err; exit 1; }
done
cat $O/ckab_$TAG.json
bash scripts/gpu_tree_ab.sh $TAG $R
