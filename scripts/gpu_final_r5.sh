#!/bin/bash
# Round-5 final-tree pass (one gpurun call): the -m gpu suite (DCN tolerance report), the variant
# library's tests, smoke(), the default bench line, a rocprofv3 kernel trace of the bench with the
# roofline cross-check, and the two PMC traffic passes (FETCH_SIZE, WRITE_SIZE) -> pmc summary.
#   bash scripts/gpu_final_r5.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
O=gpurun_out; mkdir -p $O
LIBV=$PWD/shape_based_object_detection_amd/lib/variants
rm -f $O/dcn_tol_$TAG.jsonl
SBOD_DCN_TOL_REPORT=$O/dcn_tol_$TAG.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread > $O/tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/tests_$TAG.log; exit 1; }
tail -1 $O/tests_$TAG.log
SBOD_LIB=$LIBV/libsbod_hip_onelaunch.so timeout -k 10 300 python -u -m pytest tests/test_gpu_criterion_fused.py -q \
  --timeout 120 --timeout-method thread > $O/variant_tests_$TAG.log 2>&1 || { echo "variant tests failed"; tail -30 $O/variant_tests_$TAG.log; exit 1; }
tail -1 $O/variant_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -20 $O/bench_$TAG.err; exit 1; }
python - $O/bench_$TAG.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']
print('bench', d['ms_per_step'], d['value'], r['kernel'], r['avg_us'], r['frac'], 'other',
      {k: (v['avg_us'], v['frac']) for k, v in (d.get('roofline_other') or {}).items()}, 'api', d.get('api_ms_per_step'))
print('c2', d['c2_bf16']['ms_per_step'], d['c2_bf16']['roofline']['avg_us'], 'dcn', {k: (v['ms'], v['mfma_frac']) for k, v in d['dcn']['maps'].items()},
      'cpu', d['cpu_baseline']['value'])
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-dcn > $O/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_$TAG.log; exit 1; }
python scripts/roofline_check.py $O/bench_$TAG.json $O/prof_$TAG/run_kernel_trace.csv $O/roofline_check_$TAG.json $O/prof_$TAG.log > /dev/null
python -c "
import json; h=json.load(open('$O/roofline_check_$TAG.json'))['headline']; print('check', json.dumps(h))"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 > $O/pmcf_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -5 $O/pmcf_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 > $O/pmcw_$TAG.log 2>&1 || { echo "pmc write failed"; tail -5 $O/pmcw_$TAG.log; exit 1; }
python scripts/pmc_traffic.py $O/pmcf_$TAG $O/pmcw_$TAG --out $O/pmc_traffic_$TAG.json | tail -12
bash scripts/gpu_dcn_pmc.sh $TAG > $O/dcn_pmc_$TAG.log 2>&1 || { echo "dcn pmc failed"; tail -5 $O/dcn_pmc_$TAG.log; exit 1; }
echo EXIT 0
