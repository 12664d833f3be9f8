"""Per-launch HBM traffic of each sbod kernel from two rocprofv3 PMC passes.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/pmc_traffic.json]

Each directory holds a `--pmc FETCH_SIZE` resp. `--pmc WRITE_SIZE` counter-collection CSV of the
same command (the two counters do not fit one pass on gfx950).  Corrections per
MI355X_MICROARCH.md (HBM section): both counters are in KB; FETCH_SIZE reports half of the
bytes of wide coalesced reads on gfx950, so it is doubled.  Output: mean bytes per launch."""
import argparse
import collections
import csv
import glob
import json
import os
import re


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not files:
        raise SystemExit('no counter_collection.csv under %s' % d)
    acc = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get('Counter_Name') != counter:
                continue
            m = re.search(r'sbod::(k_\w+)', r['Kernel_Name'])
            if m:
                acc[m.group(1)].append(float(r['Counter_Value']))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_dir')
    ap.add_argument('write_dir')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    fe = per_kernel(a.fetch_dir, 'FETCH_SIZE')
    wr = per_kernel(a.write_dir, 'WRITE_SIZE')
    out = {'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of '
                     'bench.py; FETCH_SIZE x2 (gfx950 half-count), KB x1024',
           'kernels': {}}
    for k in sorted(set(fe) & set(wr)):
        f = 2.0 * 1024.0 * sum(fe[k]) / len(fe[k])
        w = 1024.0 * sum(wr[k]) / len(wr[k])
        out['kernels'][k] = {'launches_fetch': len(fe[k]), 'launches_write': len(wr[k]),
                             'fetch_bytes_per_launch': round(f), 'write_bytes_per_launch': round(w),
                             'traffic_bytes_per_launch': round(f + w)}
    s = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, 'w') as fh:
            fh.write(s + '\n')
    print(s)


if __name__ == '__main__':
    main()
