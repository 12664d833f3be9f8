#!/bin/bash
# GPU box: criterion parity tests, then config C2 (bf16 B=16) against ab_base, alternating.
#   bash scripts/gpu_c2_ab.sh TAG [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; R=${2:-3}
O=$PWD/gpurun_out; mkdir -p $O
ROOT=$PWD
timeout -k 10 500 python -u -m pytest tests/test_gpu_criteria.py tests/test_gpu_bf16.py tests/test_gpu_loss_finish.py \
   tests/test_gpu_c1.py tests/test_gpu_api_fast.py tests/test_gpu_operators.py -q -x \
   --timeout 200 --timeout-method thread > $O/c2tests_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/c2tests_$TAG.log; exit 1; }
tail -1 $O/c2tests_$TAG.log
for r in $(seq 1 $R); do
  for t in ab_base .; do
    n=$( [ "$t" = "." ] && echo new || echo base )
    ( cd $ROOT/$t && timeout -k 10 300 python -u bench.py --gpus 1 --steps 50 --warmup 10 --no-dcn --no-cpu-baseline \
        > $O/c2b_${TAG}_${n}_$r.json 2>> $O/c2b_${TAG}.err ) || { echo "bench $n failed"; tail -5 $O/c2b_${TAG}.err; exit 1; }
    echo "$n r$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d["c2_bf16"]; print(d["ms_per_step"], c["ms_per_step"], c["roofline"]["avg_us"], c["roofline"]["frac"])' $O/c2b_${TAG}_${n}_$r.json)"
  done
done
echo EXIT 0
