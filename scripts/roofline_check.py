#!/usr/bin/env python3
"""Cross-check a bench line's roofline against the rocprofv3 kernel trace of the same command.

    python scripts/roofline_check.py gpurun_out/bench_TAG.json gpurun_out/prof_TAG/run_kernel_trace.csv \
        [profiles/r3_roofline_check_TAG.json] [gpurun_out/prof_TAG.log]

For every HBM-bound kernel of the bench's ALGO_BYTES table, the dispatches of the bench
workload (grid = B x ceil(P/256) workgroups of 256 threads, so the C2 bf16 step and other
shapes in the same run are excluded) are averaged from the trace (End - Start, ns: the
dispatch-level time rocprofv3 reports).  Written: per kernel, the rocprof average, the bench's
event-timed average (kernel_us_per_step), algorithmic bytes per launch, the HBM fraction from
each, and their relative difference; plus the headline kernel's line frac vs the rocprof frac.

With the profiled run's own bench line (its stdout, 4th argument), the headline kernel's
dispatches are also taken from the window of the line's dominant-kernel timing pass only
(`roofline.trace_window_ns`, host CLOCK_MONOTONIC, the clock of rocprofv3's timestamps): the
same eager launches the line's `avg_us` averages, without the warm-up, capture and graph
phases the whole-trace average mixes in.
"""
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main(bench_json, trace_csv, out=None, prof_log=None):
    import bench as BM
    line = json.loads(open(bench_json).read().strip().splitlines()[-1])
    cfg = line['config']
    B, P, C = cfg.get('global_batch', 32) // line['n_gpus'], cfg['n_priors'], cfg['n_classes']
    rl = line['roofline']
    algo = {k: f({'B': B, 'P': P, 'C': C, 'n_cand': 0}) for k, f in BM.ALGO_BYTES.items()}
    # k_det_prepare's candidate-key bytes depend on the workload's count: take them from the line
    if rl['kernel'] == 'k_det_prepare':
        algo['k_det_prepare'] = rl['algorithmic_bytes_per_launch']
    else:
        algo['k_det_prepare'] = line['step_algorithmic_bytes'] - BM.criterion_bytes(B, P, C)
    # the bench workload's dispatches are the ones with Grid_Size_Y == B; tile heights differ per
    # kernel (k_multibox's are sized per CU count, balanced_rows), so each kernel keeps its most
    # frequent grid rather than an assumed 256-row one
    durs = {k: {} for k in algo}
    win, wdurs = None, []
    if prof_log:
        for ln in open(prof_log):
            if ln.startswith('{') and '"roofline"' in ln:
                pl = json.loads(ln)
                # the timing pass of the headline kernel in the profiled run: its own roofline when
                # the profiled run picked the same kernel, else its roofline_other entry
                if pl['roofline'].get('kernel') == rl['kernel']:
                    win = pl['roofline'].get('trace_window_ns')
                else:
                    win = (pl.get('roofline_other') or {}).get(rl['kernel'], {}).get('trace_window_ns')
    def keys_of(name):
        # k_multibox<..., true> is the one-launch criterion (its KernelTimer name: k_criterion)
        if 'k_multibox<' in name:
            return ['k_criterion' if 'true>' in name else 'k_multibox']
        return [k for k in algo if (k + '<') in name or (k + '(') in name]
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            name = r['Kernel_Name']
            for k in keys_of(name):
                if k in algo:
                    if 'unsigned short' in name:      # the bf16 (C2) instantiation
                        continue
                    if int(r['Grid_Size_Y']) == B:
                        t0, t1 = int(r['Start_Timestamp']), int(r['End_Timestamp'])
                        durs[k].setdefault(int(r['Grid_Size_X']), []).append((t0, t1))
    for k, byg in list(durs.items()):
        d = max(byg.values(), key=len) if byg else []
        durs[k] = [t1 - t0 for t0, t1 in d]
        if k == rl['kernel'] and win:
            wdurs = [t1 - t0 for t0, t1 in d if win[0] <= t0 and t1 <= win[1]]
    res = {'bench': os.path.basename(bench_json), 'trace': os.path.basename(trace_csv),
           'workload': {'B': B, 'P': P, 'C': C}, 'peak_GBps': BM.HBM_PEAK_GBS, 'kernels': {}}
    for k, d in durs.items():
        if not d:
            continue
        us = sum(d) / len(d) / 1e3
        bus = line.get('kernel_us_per_step', {}).get(k)
        e = {'dispatches': len(d), 'rocprof_avg_us': round(us, 3), 'bench_event_avg_us': bus,
             'algorithmic_bytes': algo[k], 'frac_rocprof': round(algo[k] / (us * 1e-6) / 1e9 / BM.HBM_PEAK_GBS, 4)}
        if bus:
            e['frac_bench'] = round(algo[k] / (bus * 1e-6) / 1e9 / BM.HBM_PEAK_GBS, 4)
            e['rel_diff'] = round(bus / us - 1.0, 4)
        res['kernels'][k] = e
    hk = rl['kernel']
    if hk in res['kernels']:
        fr = res['kernels'][hk]['frac_rocprof']
        res['headline'] = {'kernel': hk, 'line_frac': rl['frac'], 'line_avg_us': rl['avg_us'],
                           'rocprof_frac': fr, 'rel_diff': round(rl['frac'] / fr - 1.0, 4),
                           'within_5pct': abs(rl['frac'] / fr - 1.0) <= 0.05}
        if wdurs:
            us = sum(wdurs) / len(wdurs) / 1e3
            fw = round(algo[hk] / (us * 1e-6) / 1e9 / BM.HBM_PEAK_GBS, 4)
            res['headline'].update({
                'window_dispatches': len(wdurs), 'window_rocprof_avg_us': round(us, 3),
                'window_rocprof_frac': fw, 'window_rel_diff': round(rl['frac'] / fw - 1.0, 4),
                'window_within_5pct': abs(rl['frac'] / fw - 1.0) <= 0.05})
        elif win:
            res['headline']['window_dispatches'] = 0   # clocks did not line up: whole-trace only
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        with open(out, 'w') as f:
            f.write(txt + '\n')


if __name__ == '__main__':
    main(*sys.argv[1:5])
