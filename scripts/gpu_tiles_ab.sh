#!/bin/bash
# GPU box, round 4: parity of the multi-tile focal pass, then a same-box A/B of tiles per workgroup
# (SBOD_MB_TILES 1 = k_multibox, 2, 3): the criterion kernels alone (scripts/mb_ab.py) and the
# bench step, in turn.   Usage: bash scripts/gpu_tiles_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multibox_tiles.py tests/test_gpu_criterion_fused.py \
    tests/test_gpu_loss_finish.py tests/test_gpu_graph.py tests/test_gpu_bf16.py -m gpu -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/tiles_tests_$TAG.log 2>&1 || exit 1
out=gpurun_out/tiles_ab_$TAG.jsonl
: > $out
for r in 1 2; do
  for t in ${TILES:-1 2 3}; do
    SBOD_MB_TILES=$t timeout -k 10 200 python -u scripts/mb_ab.py tiles$t >> $out 2>> gpurun_out/tiles_ab_$TAG.err || exit 1
    SBOD_MB_TILES=$t timeout -k 10 300 python -u bench.py --steps 400 --no-dcn --no-cpu-baseline \
        > gpurun_out/tiles_bench.tmp 2>> gpurun_out/tiles_ab_$TAG.err || exit 1
    tail -1 gpurun_out/tiles_bench.tmp | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); \
print(json.dumps({'tiles': $t, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'roofline': d['roofline'], \
'c2': d.get('c2_bf16', {}).get('ms_per_step'), 'c2_mb_us': d.get('c2_bf16', {}).get('roofline', {}).get('avg_us'), \
'kernel_us_per_step': d.get('kernel_us_per_step'), 'host': d.get('host_us_per_step')}))" >> $out || exit 1
  done
done
echo done
