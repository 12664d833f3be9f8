#!/bin/bash
# GPU box: variant-library A/B of the step (lib/variants/<V>/libsbod_hip.so, a full variant
# directory with the extensions) against the product library, alternating: step_modes2.py
# (steady state) and the driver's 20-step bench command; kernel_ab per-kernel times once each.
#   bash scripts/gpu_var_ab.sh TAG V [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; V=$2; R=${3:-2}
O=gpurun_out; mkdir -p $O
LIBD=$PWD/shape_based_object_detection_amd/lib
for r in $(seq 1 $R); do
  for n in $V prod; do
    L=$LIBD/libsbod_hip.so; [ "$n" = "prod" ] || L=$LIBD/variants/$V/libsbod_hip.so
    SBOD_LIB=$L timeout -k 10 300 python -u scripts/step_modes2.py --steps 300 >> $O/vmodes_${TAG}_$n.json 2>> $O/vmodes_${TAG}.err || { echo "modes $n failed"; tail -5 $O/vmodes_${TAG}.err; exit 1; }
    SBOD_LIB=$L timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 \
        > $O/vb20_${TAG}_${n}_$r.json 2>> $O/vb20_${TAG}.err || { echo "bench $n failed"; tail -5 $O/vb20_${TAG}.err; exit 1; }
    echo "$n r$r modes $(tail -1 $O/vmodes_${TAG}_$n.json | python -c 'import json,sys; d=json.load(sys.stdin); print({k:v for k,v in d["rep1"].items()})')"
    echo "$n r$r bench20 $(python scripts/bench_summary.py $O/vb20_${TAG}_${n}_$r.json | cut -c1-330)"
  done
done
echo EXIT 0
