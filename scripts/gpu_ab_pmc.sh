#!/bin/bash
# GPU box: per-kernel A/B (kernel_ab.py) of lib/variants/libsbod_hip_<V>.so against the product
# library, two rounds in turn, then the product library's FETCH_SIZE / WRITE_SIZE passes.
#   bash scripts/gpu_ab_pmc.sh TAG V [nopmc]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; V=$2
O=gpurun_out; mkdir -p $O
LIBD=$PWD/shape_based_object_detection_amd/lib
run() { SBOD_LIB=$1 timeout -k 10 150 python scripts/kernel_ab.py >> $O/kab_$TAG.json 2>> $O/kab_$TAG.err; }
for round in 1 2; do
  run $LIBD/variants/libsbod_hip_$V.so || { echo "kab $V failed"; tail -5 $O/kab_$TAG.err; exit 1; }
  run $LIBD/libsbod_hip.so || { echo "kab product failed"; tail -5 $O/kab_$TAG.err; exit 1; }
done
cat $O/kab_$TAG.json
if [ "$3" != "nopmc" ]; then
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 > $O/pmcf_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -5 $O/pmcf_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$TAG -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --no-dcn --no-cpu-baseline --no-c2 > $O/pmcw_$TAG.log 2>&1 || { echo "pmc write failed"; tail -5 $O/pmcw_$TAG.log; exit 1; }
python scripts/pmc_traffic.py $O/pmcf_$TAG $O/pmcw_$TAG --out $O/pmc_traffic_$TAG.json | tail -12
fi
echo EXIT 0
