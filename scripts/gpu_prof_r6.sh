#!/bin/bash
# Round-6 profiling pass (one gpurun call, after scripts/gpu_r6.sh TAG has written bench_TAG.json):
# a rocprofv3 kernel trace of the bench with the roofline cross-check, the two PMC traffic passes
# (FETCH_SIZE, WRITE_SIZE) -> pmc summary, and the DCN PMC passes.
#   bash scripts/gpu_prof_r6.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u bench.py --no-dcn > $O/pbench_$TAG.json 2> $O/pbench_$TAG.err || { echo "bench failed"; tail -20 $O/pbench_$TAG.err; exit 1; }
python scripts/bench_summary.py $O/pbench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o run --output-format csv -- \
    python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-dcn > $O/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_$TAG.log; exit 1; }
python scripts/roofline_check.py $O/pbench_$TAG.json $O/prof_$TAG/run_kernel_trace.csv $O/roofline_check_$TAG.json $O/prof_$TAG.log > /dev/null
python -c "
import json; h=json.load(open('$O/roofline_check_$TAG.json'))['headline']; print('check', json.dumps(h))"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 > $O/pmcf_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -5 $O/pmcf_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 > $O/pmcw_$TAG.log 2>&1 || { echo "pmc write failed"; tail -5 $O/pmcw_$TAG.log; exit 1; }
python scripts/pmc_traffic.py $O/pmcf_$TAG $O/pmcw_$TAG --out $O/pmc_traffic_$TAG.json | tail -12
bash scripts/gpu_dcn_pmc.sh $TAG > $O/dcn_pmc_$TAG.log 2>&1 || { echo "dcn pmc failed"; tail -5 $O/dcn_pmc_$TAG.log; exit 1; }
tail -3 $O/dcn_pmc_$TAG.log
echo EXIT 0
