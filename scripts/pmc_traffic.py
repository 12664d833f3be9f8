"""Per-launch HBM traffic of each sbod kernel from two rocprofv3 PMC passes.

    python scripts/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/pmc_traffic.json]

Each directory holds a `--pmc FETCH_SIZE` resp. `--pmc WRITE_SIZE` counter-collection CSV of the
same command (the two counters do not fit one pass on gfx950), grouped by (kernel, grid size).  Corrections per
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
                acc[(m.group(1), int(r.get('Grid_Size') or 0))].append(float(r['Counter_Value']))
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
    # one entry per (kernel, grid size): a kernel launched at several shapes in the same run (the
    # bench's B=32 fp32 step, its C2 B=16 bf16 figure, DCN maps) is not averaged across them.
    # `kernels[k]` is the largest grid's entry (the bench workload), `by_grid[k]` all of them.
    out['by_grid'] = {}
    for key in sorted(set(fe) & set(wr)):
        k, grid = key
        f = 2.0 * 1024.0 * sum(fe[key]) / len(fe[key])
        w = 1024.0 * sum(wr[key]) / len(wr[key])
        e = {'grid_size': grid, 'launches_fetch': len(fe[key]), 'launches_write': len(wr[key]),
             'fetch_bytes_per_launch': round(f), 'write_bytes_per_launch': round(w),
             'traffic_bytes_per_launch': round(f + w)}
        out['by_grid'].setdefault(k, []).append(e)
        if k not in out['kernels'] or grid > out['kernels'][k]['grid_size']:
            out['kernels'][k] = e
    s = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, 'w') as fh:
            fh.write(s + '\n')
    print(s)


if __name__ == '__main__':
    main()
