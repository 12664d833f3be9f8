#!/bin/bash
# Round-5 DCN pass (one gpurun call): the DCN parity tests with the tolerance report, the map
# timings of the product library and (if built) of the split-bf16 A/B library, and a rocprofv3
# kernel trace of the product library's maps.
#   bash scripts/gpu_dcn_r5.sh TAG [--no-ab] [--no-prof]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
AB=1; PROF=1
for a in "$@"; do case $a in --no-ab) AB=0;; --no-prof) PROF=0;; esac; done
O=gpurun_out; mkdir -p $O
LIBV=$PWD/shape_based_object_detection_amd/lib/variants
rm -f $O/dcn_tol_$TAG.jsonl
SBOD_DCN_TOL_REPORT=$O/dcn_tol_$TAG.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_dcn.py -q -x --timeout 120 \
  --timeout-method thread > $O/dcntests_$TAG.log 2>&1 || { echo "dcn tests failed"; tail -40 $O/dcntests_$TAG.log; exit 1; }
tail -2 $O/dcntests_$TAG.log
python - $O/dcn_tol_$TAG.jsonl <<'PY'
import json, sys
worst = {}
for ln in open(sys.argv[1]):
    r = json.loads(ln)
    k = r['what'].split('@')[0]
    w = worst.get(k)
    if w is None or r['max_err_over_tol'] > w['max_err_over_tol']:
        worst[k] = r
for k, r in sorted(worst.items()):
    print('tol %-28s err/tol %.3f max_rel_above_floor %.2e above %d/%d' % (k[:28], r['max_err_over_tol'],
          r['max_rel_above_floor'], r['entries_above_floor'], r['n']))
PY
timeout -k 10 300 python -u scripts/dcn_maps.py > $O/dcn_maps_$TAG.jsonl 2> $O/dcn_maps_$TAG.err || { echo "maps failed"; tail -20 $O/dcn_maps_$TAG.err; exit 1; }
python -c "
import json,sys
for ln in open(sys.argv[1]):
    r=json.loads(ln); print('maps', r['config'][-30:], r['ms'], 'frac', r['mfma_frac'], 'eager', r.get('eager_ms'))
" $O/dcn_maps_$TAG.jsonl
if [ $AB = 1 ] && [ -f $LIBV/libsbod_hip_dcnsplit.so ]; then
  SBOD_LIB=$LIBV/libsbod_hip_dcnsplit.so timeout -k 10 300 python -u scripts/dcn_maps.py > $O/dcn_maps_split_$TAG.jsonl 2> $O/dcn_maps_split_$TAG.err || { echo "split maps failed"; tail -20 $O/dcn_maps_split_$TAG.err; exit 1; }
  python -c "
import json,sys
for ln in open(sys.argv[1]):
    r=json.loads(ln); print('split maps', r['config'][-30:], r['ms'], 'frac', r['mfma_frac'], 'eager', r.get('eager_ms'))
" $O/dcn_maps_split_$TAG.jsonl
fi
if [ $PROF = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dprof_$TAG -o run --output-format csv -- \
      python scripts/dcn_maps.py --iters 5 > $O/dprof_$TAG.log 2>&1 || { echo "prof failed"; tail -20 $O/dprof_$TAG.log; exit 1; }
  python - $O/dprof_$TAG/run_kernel_trace.csv <<'PY'
import csv, sys, statistics
d = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name'].split('(')[0][:40]
    key = '%s grid %sx%sx%s' % (n, r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
    d.setdefault(key, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in d.items():
    if 'dcn' in k or 'wb_split' in k or 'transpose' in k or 'weight_layouts' in k:
        print('%-70s n %4d median %8.2f us' % (k, len(v), statistics.median(v)))
PY
fi
echo EXIT 0
