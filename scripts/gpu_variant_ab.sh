#!/bin/bash
# A/B of variant libraries (lib/variants/<name>/) against the product library on the GPU-side step
# interval (scripts/gpu_interval.py) and the default bench line's kernel times:
#   bash scripts/gpu_variant_ab.sh TAG "tests ..." NAME [NAME ...]
# the given test files run on every variant first (parity); then two alternating rounds.
set -o pipefail
T=$1; TESTS=$2; shift 2
O=gpurun_out/variant_ab_$T.jsonl
: > $O
VD=$PWD/shape_based_object_detection_amd/lib/variants
for V in "$@"; do
  SBOD_LIB=$VD/$V/libsbod_hip.so timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 \
      --timeout-method thread > gpurun_out/variant_ab_tests_${T}_$V.log 2>&1 \
      || { tail -5 gpurun_out/variant_ab_tests_${T}_$V.log; exit 1; }
  echo "$V: $(tail -1 gpurun_out/variant_ab_tests_${T}_$V.log)"
done
for r in 1 2; do
  for L in product "$@"; do
    E=""
    [ $L != product ] && E="SBOD_LIB=$VD/$L/libsbod_hip.so"
    env $E timeout -k 10 120 python -u scripts/gpu_interval.py --reps 2 2>>gpurun_out/variant_ab.err | tail -1 \
        | sed "s/^{/{\"lib\": \"$L\", /" >> $O || exit 1
    env $E timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 --no-dcn --no-c2 --no-cpu-baseline \
        2>>gpurun_out/variant_ab.err | tail -1 > gpurun_out/variant_ab_bench_$T.json || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/variant_ab_bench_$T.json').read()); print(json.dumps({'lib': '$L', 'round': $r, 'ms_per_step': d['ms_per_step'], 'roofline_other': d.get('roofline_other'), 'kernel_us_per_step': d['kernel_us_per_step']}))" >> $O || exit 1
  done
done
cat $O
