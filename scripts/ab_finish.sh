#!/bin/bash
# Loss-finish A/B on one box: the focal loss summed in k_multibox's last workgroup (fused) or by
# a separate one-block launch (separate), alternated REPS times; one summary line per bench run.
#   bash scripts/ab_finish.sh [REPS] [extra bench args...]
set -o pipefail
O=gpurun_out
REPS=${1:-3}; shift
for i in $(seq 1 $REPS); do
for f in fused separate; do
timeout -k 10 400 python -u bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-dcn --finish $f "$@" > $O/ab_$f$i.json 2> $O/ab_$f$i.err || { tail -20 $O/ab_$f$i.err; exit 1; }
python - $O/ab_$f$i.json $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']; c = d.get('c2_bf16', {})
k = d.get('kernel_us_per_step') or {}
print(sys.argv[2], 'step', d['ms_per_step'], 'mb', r['avg_us'], r['frac'], 'c2', c.get('ms_per_step'),
      c.get('roofline', {}).get('avg_us'), 'k_multibox', k.get('k_multibox'), 'k_loss_final', k.get('k_loss_final'),
      'api', d.get('api_ms_per_step'))
PY
done
done
