"""Per-kernel, per-grid average durations from a rocprofv3 kernel trace CSV."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ''
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if pat in n:
        key = (n.split('(')[0][:60], r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
        d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print('%-60s grid=%s,%s,%s n=%d avg=%.1fus' % (k[0], k[1], k[2], k[3], len(v), sum(v) / len(v)))
