#!/bin/bash
# A/B: pass-1 segment workgroups of 4 waves (product) vs 8 waves (-DSBOD_SEG_W=8 variant):
# the detect tests on the variant, then alternating rounds of the GPU-side step interval
# (scripts/gpu_interval.py) and the default bench line's kernel times.
set -o pipefail
T=${1:-a}
O=gpurun_out/segw_ab_$T.jsonl
: > $O
V=$PWD/shape_based_object_detection_amd/lib/variants/segw8/libsbod_hip.so
SBOD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/segw_tests_$T.log 2>&1 || { tail -5 gpurun_out/segw_tests_$T.log; exit 1; }
tail -1 gpurun_out/segw_tests_$T.log
for r in 1 2; do
  for L in product segw8; do
    E=""
    [ $L = segw8 ] && E="SBOD_LIB=$V"
    env $E timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 2>>gpurun_out/segw_ab.err | tail -1 \
        | sed "s/^{/{\"lib\": \"$L\", /" >> $O || exit 1
    env $E timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 --no-dcn --no-c2 --no-cpu-baseline \
        2>>gpurun_out/segw_ab.err | tail -1 > gpurun_out/segw_bench_$T.json || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/segw_bench_$T.json').read()); print(json.dumps({'lib': '$L', 'round': $r, 'ms_per_step': d['ms_per_step'], 'kernel_us_per_step': d['kernel_us_per_step']}))" >> $O || exit 1
  done
done
cat $O
