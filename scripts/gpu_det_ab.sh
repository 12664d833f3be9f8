#!/bin/bash
# A/B of the detect chain: base (lib/variants/base: the tree before the change), the product
# library, and lib/variants/segw8 (the product with 8-wave pass-1 segments).  The detect tests
# on the product and on segw8 first; then alternating rounds of the GPU-side step interval
# (scripts/gpu_interval.py) and the default bench line's kernel times and step time.
set -o pipefail
T=${1:-a}
O=gpurun_out/det_ab_$T.jsonl
: > $O
VD=$PWD/shape_based_object_detection_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py tests/test_gpu_detect_fused.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/det_tests_$T.log 2>&1 || { tail -5 gpurun_out/det_tests_$T.log; exit 1; }
tail -1 gpurun_out/det_tests_$T.log
SBOD_LIB=$VD/segw8/libsbod_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py \
    tests/test_gpu_detect_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/det_tests_w8_$T.log 2>&1 \
    || { tail -5 gpurun_out/det_tests_w8_$T.log; exit 1; }
tail -1 gpurun_out/det_tests_w8_$T.log
for r in 1 2; do
  for L in base product segw8; do
    E=""
    [ $L != product ] && E="SBOD_LIB=$VD/$L/libsbod_hip.so"
    env $E timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 2>>gpurun_out/det_ab.err | tail -1 \
        | sed "s/^{/{\"lib\": \"$L\", /" >> $O || exit 1
    env $E timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 --no-dcn --no-c2 --no-cpu-baseline \
        2>>gpurun_out/det_ab.err | tail -1 > gpurun_out/det_bench_$T.json || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/det_bench_$T.json').read()); print(json.dumps({'lib': '$L', 'round': $r, 'ms_per_step': d['ms_per_step'], 'kernel_us_per_step': d['kernel_us_per_step']}))" >> $O || exit 1
  done
done
cat $O
