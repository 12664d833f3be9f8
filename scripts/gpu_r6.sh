#!/bin/bash
# Round-6 pass (one gpurun call): the -m gpu suite, the variant library's tests, smoke(), the
# default bench line, and the driver's own command (--steps 20 --warmup 5) three times.
#   bash scripts/gpu_r6.sh TAG [quick]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
O=gpurun_out; mkdir -p $O
LIBV=$PWD/shape_based_object_detection_amd/lib/variants
rm -f $O/dcn_tol_$TAG.jsonl
SBOD_DCN_TOL_REPORT=$O/dcn_tol_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q -x \
  --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
SBOD_LIB=$LIBV/libsbod_hip_onelaunch.so timeout -k 10 300 python -u -m pytest tests/test_gpu_criterion_fused.py -q \
  --timeout 120 --timeout-method thread > $O/variant_tests_$TAG.log 2>&1 || { echo "variant tests failed"; tail -30 $O/variant_tests_$TAG.log; exit 1; }
tail -1 $O/variant_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -20 $O/bench_$TAG.err; exit 1; }
python scripts/bench_summary.py $O/bench_$TAG.json
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 \
      > $O/bench20_${TAG}_$i.json 2> $O/bench20_${TAG}_$i.err || { echo "bench20 failed"; tail -20 $O/bench20_${TAG}_$i.err; exit 1; }
  python scripts/bench_summary.py $O/bench20_${TAG}_$i.json
done
# the data-parallel step rehearsed on this one GPU (two ranks on cuda:0 over gloo: RCCL refuses
# two ranks on one device): DPGraph with the next step's matcher + all-reduce issued ahead
SBOD_BENCH_SAME_DEVICE=1 SBOD_BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 \
    --no-dcn --no-cpu-baseline --no-c2 > $O/dp2_$TAG.json 2> $O/dp2_$TAG.err || { echo "dp2 failed"; tail -20 $O/dp2_$TAG.err; exit 1; }
python scripts/bench_summary.py $O/dp2_$TAG.json
echo EXIT 0
