#!/usr/bin/env python3
"""The GPU side of the bench's TIMED region from a rocprofv3 kernel trace of the same run
(diagnostic):

    python scripts/timed_trace.py gpurun_out/prof_TAG.log gpurun_out/prof_TAG/run_kernel_trace.csv

The profiled run's bench line carries `timed_run_detail.timed_window_ns` (host CLOCK_MONOTONIC,
rocprofv3's clock).  Printed: the dispatches inside the window per kernel (count, mean duration),
the window, the first dispatch start / last dispatch end relative to it, the GPU-busy union of
all dispatch intervals, and the idle gaps (no kernel running) longer than 2 us."""
import collections
import csv
import json
import sys


def main(log, trace):
    line = None
    for ln in open(log):
        if ln.startswith('{') and '"timed_run_detail"' in ln:
            line = json.loads(ln)
    w0, w1 = line['timed_run_detail']['timed_window_ns']
    rows = [r for r in csv.DictReader(open(trace))]
    ks = []
    for r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if s >= w0 and e <= w1:
            ks.append((s, e, r['Kernel_Name'].split('(')[0].replace('void ', '')[:48], r.get('Queue_Id', r.get('Stream_Id', ''))))
    ks.sort()
    per = collections.defaultdict(list)
    for s, e, n, q in ks:
        per[n].append((e - s) / 1e3)
    out = {'steps': line['steps'], 'ms_per_step': line['ms_per_step'], 'window_us': (w1 - w0) / 1e3,
           'first_start_us': (ks[0][0] - w0) / 1e3 if ks else None,
           'last_end_us': (max(e for _, e, _, _ in ks) - w0) / 1e3 if ks else None,
           'kernels': {n: {'n': len(v), 'avg_us': round(sum(v) / len(v), 2)} for n, v in per.items()}}
    # busy union and gaps
    busy, gaps, cur_s, cur_e = 0, [], None, None
    for s, e, _, _ in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                if s - cur_e > 2000:
                    gaps.append((round((cur_e - w0) / 1e3, 1), round((s - cur_e) / 1e3, 1)))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    out['gpu_busy_us'] = round(busy / 1e3, 1)
    out['idle_gaps_us'] = gaps[:40]
    # concurrency profile: time with k kernels running
    ev = sorted([(s, 1) for s, _, _, _ in ks] + [(e, -1) for _, e, _, _ in ks])
    conc = collections.Counter()
    k, t0 = 0, None
    for t, d in ev:
        if t0 is not None:
            conc[k] += t - t0
        k += d
        t0 = t
    out['concurrency_us'] = {str(c): round(v / 1e3, 1) for c, v in sorted(conc.items())}
    print(json.dumps(out, indent=1))
    if '--list' in sys.argv:
        for s, e, n, q in ks:
            print('%9.1f %9.1f %6.1f q%s %s' % ((s - w0) / 1e3, (e - w0) / 1e3, (e - s) / 1e3, q, n))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
