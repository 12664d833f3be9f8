#!/bin/bash
# Same-box A/B of library builds on the bench: ROUNDS rounds, each running bench.py once per
# library in turn (product = the default libsbod_hip.so, else lib/variants/libsbod_hip_NAME.so).
# One summary line per run: step, both halves' main kernels alone, C2 step and its k_multibox.
#   bash scripts/gpu_lib_ab.sh TAG ROUNDS product NAME [NAME ...] [-- bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; ROUNDS=$2; shift 2
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
BARGS=${*:-"--steps 300 --warmup 10 --no-cpu-baseline --no-dcn"}
O=gpurun_out; mkdir -p $O
LIBV=$PWD/shape_based_object_detection_amd/lib/variants
for r in $(seq 1 $ROUNDS); do
  for name in "${LIBS[@]}"; do
    if [ "$name" = product ]; then unset SBOD_LIB; else export SBOD_LIB=$LIBV/$name/libsbod_hip.so; fi
    f=$O/ab_${TAG}_${name}_$r.json
    timeout -k 10 400 python -u bench.py $BARGS > $f 2> $f.err || { echo "$name failed"; tail -20 $f.err; exit 1; }
    python - $f $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']; c = d.get('c2_bf16') or {}
al = {r['kernel']: r['avg_us']}
al.update({k: v['avg_us'] for k, v in (d.get('roofline_other') or {}).items()})
print('%-8s step %.4f alone %s c2 %s c2_mb %s api %s' % (sys.argv[2], d['ms_per_step'], al, c.get('ms_per_step'),
      (c.get('roofline') or {}).get('avg_us'), d.get('api_ms_per_step')))
PY
  done
done
echo EXIT 0
