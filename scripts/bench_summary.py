#!/usr/bin/env python3
"""One-line summary of a bench.py JSON line (diagnostic): step, roofline kernel, other kernels."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']
out = {'ms': d['ms_per_step'], 'frac_step': d.get('step_hbm_frac'), 'roof': (r['kernel'], r['avg_us'], r['frac']),
       'other': {k: (v['avg_us'], v['frac']) for k, v in (d.get('roofline_other') or {}).items()},
       'kus': d.get('kernel_us_per_step'), 'api': d.get('api_ms_per_step'),
       'run': {k: v for k, v in (d.get('timed_run_detail') or {}).items() if k != 'native_submit_us_per_step'}}
if 'c2_bf16' in d:
    out['c2'] = (d['c2_bf16']['ms_per_step'], d['c2_bf16']['roofline']['avg_us'], d['c2_bf16']['roofline']['frac'])
if 'dcn' in d:
    out['dcn'] = {k: (v['ms'], v['mfma_frac']) for k, v in d['dcn']['maps'].items()}
if 'cpu_baseline' in d:
    out['cpu'] = d['cpu_baseline']['value']
print(json.dumps(out))
