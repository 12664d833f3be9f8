#!/bin/bash
# GPU box: detect / graph / bf16 parity tests, then the kernel A/B against a variant, then the
# step modes probe (steady-state intervals).
#   bash scripts/gpu_detect_ab.sh TAG V
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; V=$2
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_detect.py tests/test_gpu_detect_fused.py tests/test_gpu_graph.py \
   tests/test_gpu_bf16.py tests/test_gpu_map.py tests/test_gpu_c1.py -q -x --timeout 200 --timeout-method thread \
   > $O/dtests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/dtests_$TAG.log; exit 1; }
tail -1 $O/dtests_$TAG.log
bash scripts/gpu_ab_pmc.sh $TAG $V nopmc || exit 1
timeout -k 10 300 python -u scripts/step_modes2.py > $O/modes_$TAG.json 2> $O/modes_$TAG.err || { tail -20 $O/modes_$TAG.err; exit 1; }
cat $O/modes_$TAG.json
echo EXIT 0
