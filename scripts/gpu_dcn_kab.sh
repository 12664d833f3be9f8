#!/bin/bash
# DCN per-kernel A/B: rocprofv3 kernel trace of the 64x64 (and 8x8) maps for the product library
# and each named variant library, one profiled run per map; prints the median duration of every
# DCN kernel per library and map.
#   bash scripts/gpu_dcn_kab.sh TAG variant1 [variant2 ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out; mkdir -p $O
LIBV=$PWD/shape_based_object_detection_amd/lib/variants
run() {   # name lib
  local name=$1 lib=$2
  if [ -n "$lib" ]; then export SBOD_LIB=$lib; else unset SBOD_LIB; fi
  # one profiled run per map: two maps can launch a kernel with the same grid (the weight
  # gradient's 64x64 and 32x32 grids coincide), and a per-grid median would mix them
  : > $O/kab_${TAG}_$name.log
  for H in $(echo ${MAPS:-64,8} | tr ',' ' '); do
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kab_${TAG}_${name}_m$H -o run --output-format csv -- \
        python scripts/dcn_maps.py --maps $H --iters 5 >> $O/kab_${TAG}_$name.log 2>&1 || { echo "$name failed"; tail -20 $O/kab_${TAG}_$name.log; exit 1; }
  done
  python - $O/kab_${TAG}_${name} $name <<'PY'
import csv, glob, sys, statistics
d = {}
for f in sorted(glob.glob(sys.argv[1] + '_m*/run_kernel_trace.csv')):
    m = f.split('_m')[-1].split('/')[0]
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('sbod::', '')[:34]
        key = '%s %sx%sx%s @%s' % (n, r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'], m)
        d.setdefault(key, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = {}
for k, v in d.items():
    if 'rocprim' in k:
        continue
    print('%-10s %-62s n %3d median %8.2f' % (sys.argv[2], k, len(v), statistics.median(v)))
PY
  grep '"ms"' $O/kab_${TAG}_$name.log | python -c "
import json,sys
for ln in sys.stdin:
    r=json.loads(ln); print('$name', r['config'][-22:], 'ms', r['ms'], 'eager', r.get('eager_ms'))"
}
run product ''
for v in "$@"; do
  if [ -n "$TESTS" ]; then   # the variant's DCN parity tests first
    SBOD_LIB=$LIBV/$v/libsbod_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -q -x --timeout 120 \
      --timeout-method thread > $O/kab_${TAG}_${v}_tests.log 2>&1 || { echo "$v tests failed"; tail -30 $O/kab_${TAG}_${v}_tests.log; exit 1; }
    tail -1 $O/kab_${TAG}_${v}_tests.log
  fi
  run $v $LIBV/$v/libsbod_hip.so
done
echo EXIT 0
