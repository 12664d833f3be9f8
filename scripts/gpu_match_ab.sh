#!/bin/bash
# GPU box: matcher / criterion parity tests, per-kernel times of ab_base and this tree
# (kernel_ab.py), k_match_tile stamps (stamps build), then the whole-tree A/B (gpu_tree_ab.sh).
#   bash scripts/gpu_match_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-1}
O=$PWD/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_stress.py tests/test_gpu_criteria.py \
   tests/test_gpu_gt_fold.py tests/test_gpu_graph.py tests/test_gpu_bf16.py tests/test_gpu_c1.py tests/test_gpu_operators.py \
   tests/test_gpu_loss_finish.py tests/test_gpu_api_fast.py -q -x --timeout 200 --timeout-method thread \
   > $O/mtests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/mtests_$TAG.log; exit 1; }
tail -1 $O/mtests_$TAG.log
for t in ab_base . ab_base .; do
  ( cd $t && timeout -k 10 150 python scripts/kernel_ab.py ) >> $O/mkab_$TAG.json 2>> $O/mkab_$TAG.err || { echo "kab failed"; tail -5 $O/mkab_$TAG.err; exit 1; }
done
cat $O/mkab_$TAG.json
SBOD_LIB=$PWD/shape_based_object_detection_amd/lib/variants/libsbod_hip_stamps.so timeout -k 10 120 python scripts/match_stamps.py --reps 3 \
   > $O/mstamps_$TAG.json 2> $O/mstamps_$TAG.err || { echo "stamps failed"; tail -5 $O/mstamps_$TAG.err; exit 1; }
tail -2 $O/mstamps_$TAG.json
bash scripts/gpu_tree_ab.sh $TAG $R
