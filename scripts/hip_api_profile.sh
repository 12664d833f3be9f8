#!/bin/bash
# HIP runtime API trace of the pipelined bench (no counters): which API calls the per-step host
# submit spends its time in.   bash scripts/hip_api_profile.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
TAG=$1
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/hipapi_$TAG -o run --output-format csv -- \
    python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-dcn --no-c2 > $O/hipapi_$TAG.log 2>&1 || { tail -20 $O/hipapi_$TAG.log; exit 1; }
python - $O/hipapi_$TAG <<'PY'
import csv, glob, sys, collections, statistics
d = sys.argv[1]
f = glob.glob(d + '/**/*hip_api_trace.csv', recursive=True)
if not f:
    print('no hip api trace', glob.glob(d + '/**/*', recursive=True)); sys.exit(1)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    agg[r['Function']].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
tot = sum(sum(v) for v in agg.values())
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:25]:
    print('%-40s n %7d  total %9.1f us  mean %6.2f  median %6.2f' % (k, len(v), sum(v), sum(v) / len(v), statistics.median(v)))
PY
echo EXIT 0
