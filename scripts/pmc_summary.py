#!/usr/bin/env python3
"""Per-kernel means of rocprofv3 --pmc counter CSVs (several passes merged):
    python scripts/pmc_summary.py DIR [DIR ...] [--match SUBSTR]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    match = None
    if '--match' in sys.argv:
        match = sys.argv[sys.argv.index('--match') + 1]
        args = [a for a in args if a != match]
    out = collections.defaultdict(dict)
    for d in args:
        for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
            agg = collections.defaultdict(lambda: collections.defaultdict(float))
            disp = collections.defaultdict(set)
            for r in csv.DictReader(open(f)):
                k = r['Kernel_Name'].split('(')[0].replace('void ', '')
                if match and match not in k:
                    continue
                agg[k][r['Counter_Name']] += float(r['Counter_Value'])
                disp[k].add(r['Dispatch_Id'])
            for k, cs in agg.items():
                for c, v in cs.items():
                    out[k][c] = v / len(disp[k])
                out[k]['dispatches'] = len(disp[k])
    for k in sorted(out):
        print(k, json.dumps({c: float('%.4g' % v) for c, v in sorted(out[k].items())}))


if __name__ == '__main__':
    main()
