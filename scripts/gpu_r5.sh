#!/bin/bash
# Round-5 GPU pass (one gpurun call): the -m gpu suite with the DCN tolerance report, the
# one-launch variant's tests against the variant library, the k_multibox per-workgroup stamps,
# and a 300-step bench line.  Every GPU step has its own time limit; the first failure ends it.
#   bash scripts/gpu_r5.sh TAG [--no-tests] [--no-stamps] [--no-variant] [--bench-args "..."]
set -o pipefail
TAG=$1; shift
TESTS=1; STAMPS=1; VARIANT=1; BARGS="--steps 300 --warmup 10 --no-cpu-baseline --no-dcn"
while [ $# -gt 0 ]; do
  case $1 in
    --no-tests) TESTS=0;;
    --no-stamps) STAMPS=0;;
    --no-variant) VARIANT=0;;
    --bench-args) BARGS=$2; shift;;
  esac
  shift
done
O=gpurun_out
mkdir -p $O
LIBV=$PWD/shape_based_object_detection_amd/lib/variants
if [ $TESTS = 1 ]; then
  rm -f $O/dcn_tol_$TAG.jsonl
  SBOD_DCN_TOL_REPORT=$O/dcn_tol_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_$TAG.log; exit 1; }
  tail -3 $O/tests_$TAG.log
fi
if [ $VARIANT = 1 ] && [ -f $LIBV/libsbod_hip_onelaunch.so ]; then
  SBOD_LIB=$LIBV/libsbod_hip_onelaunch.so timeout -k 10 300 python -u -m pytest tests/test_gpu_criterion_fused.py -x -q \
    --timeout 120 --timeout-method thread > $O/variant_tests_$TAG.log 2>&1 || { echo "variant tests failed"; tail -30 $O/variant_tests_$TAG.log; exit 1; }
  tail -2 $O/variant_tests_$TAG.log
fi
if [ $STAMPS = 1 ] && [ -f $LIBV/libsbod_hip_stamps.so ]; then
  SBOD_LIB=$LIBV/libsbod_hip_stamps.so timeout -k 10 300 python -u scripts/mb_imbalance.py --out $O/mb_imb_$TAG.json \
    > $O/mb_imb_$TAG.log 2>&1 || { echo "stamps failed"; tail -20 $O/mb_imb_$TAG.log; exit 1; }
  grep -v amdgpu.ids $O/mb_imb_$TAG.log | cut -c1-400
fi
timeout -k 10 600 python -u bench.py $BARGS > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -20 $O/bench_$TAG.err; exit 1; }
python - "$O/bench_$TAG.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']
print('bench', d['ms_per_step'], 'ms', d['value'], 'img/s', 'roofline', r['kernel'], r['avg_us'], 'us frac', r['frac'],
      'kernels', d.get('kernel_us_per_step'), 'host', d.get('host_us_per_step'))
for k, v in (d.get('roofline_other') or {}).items():
    print('other', k, v['avg_us'], 'us frac', v['frac'], 'in-step', v['in_step_avg_us'])
print('api', d.get('api_ms_per_step'))
if 'c2_bf16' in d:
    c = d['c2_bf16']
    print('c2', c['ms_per_step'], 'ms', c['roofline']['avg_us'], 'us frac', c['roofline']['frac'])
EOF
