#!/usr/bin/env python3
"""What rocprofv3 --kernel-trace adds to each dispatch ("do this" 1).

The bench line times its roofline kernel with HIP start/stop events attached to each dispatch;
the committed rocprofv3 traces report longer dispatches for the same kernel.  This probe runs the
SAME measurements once plainly and once under the profiler, in one process layout:

  * eager: an empty kernel (k_null, one workgroup) and the criterion half of the bench step
    (GT packing + matcher + the fused loss pass k_multibox), each dispatch carrying attached HIP
    events;
  * graph: one hipGraph per resident batch holding [k_null, criterion forward + backward],
    replayed back to back; the wall time per replay from HIP events around the whole run.

    python scripts/rocprof_overhead.py --out gpurun_out/ovh_plain.json
    rocprofv3 --kernel-trace -d gpurun_out/ovh -o run --output-format csv -- \\
        python3 scripts/rocprof_overhead.py --out gpurun_out/ovh_prof.json
    python scripts/rocprof_overhead.py --combine gpurun_out/ovh_plain.json gpurun_out/ovh_prof.json \\
        gpurun_out/ovh/run_kernel_trace.csv profiles/r4_rocprof_overhead_TAG.json

The combined record gives, per kernel: the event-timed average without and with the profiler, the
trace's average, and the graph replay's per-dispatch cost without and with the profiler; the
profiler's added cost per dispatch is (replay_prof - replay_plain) / dispatches per replay.
"""
import argparse
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def measure(out, reps=60, replays=300):
    import torch
    import bench as BM
    from shape_based_object_detection_amd import _lib as L
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    L.lib()
    st = BM.Step(dev, 32, 0, 1, graph=False, n_batches=6, submit='graph', depth=2)
    for _ in range(4):
        st.eager_half('criterion')
    torch.cuda.synchronize()
    res = {'workload': 'SSD512 B=32 criterion half (GT packing + matcher + fused loss pass fwd+bwd)'}
    # eager, attached events
    s = st.cap_stream.cuda_stream
    L.timing_enable('k_null')
    for _ in range(reps):
        L.call('sbod_null_kernel', 1, s)
    torch.cuda.synchronize()
    n, ms = L.timing_query('k_null')
    res['event_us'] = {'k_null': ms * 1e3 / n}
    L.timing_enable('k_multibox')
    for _ in range(reps):
        st.eager_half('criterion')
    torch.cuda.synchronize()
    n, ms = L.timing_query('k_multibox')
    res['event_us']['k_multibox'] = ms * 1e3 / n
    L.timing_enable(None)
    # graph: [k_null, criterion] per resident batch, replayed back to back
    graphs = []
    gt = st.batches[0].stage.stage(st.batches[0].boxes, st.batches[0].labels)
    for bt in st.batches:
        bt.locs.grad = None
        bt.scores.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st.cap_stream):
            L.call('sbod_null_kernel', 1, st.cap_stream.cuda_stream)
            loss = st.crit(bt.locs, bt.scores, gt, None)
            loss.backward(st.one)
        graphs.append(g)
    torch.cuda.synchronize()
    with torch.cuda.stream(st.cap_stream):
        for g in graphs:
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(replays):
            graphs[i % len(graphs)].replay()
        e1.record()
    torch.cuda.synchronize()
    res['graph'] = {'replays': replays, 'dispatches_per_replay': 4,
                    'us_per_replay': e0.elapsed_time(e1) * 1e3 / replays}
    with open(out, 'w') as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def combine(plain, prof, trace, out):
    a, b = json.load(open(plain)), json.load(open(prof))
    durs = {'k_null': [], 'k_multibox': []}
    for r in csv.DictReader(open(trace)):
        name = r['Kernel_Name']
        key = ('k_null' if 'k_null' in name else
               ('k_multibox' if ('k_multibox<float' in name and 'false>' in name) else None))
        if key and int(r['Grid_Size_Y']) in (1, 32):
            durs[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    res = {'workload': a['workload'], 'kernels': {}}
    for k, d in durs.items():
        res['kernels'][k] = {'event_us_plain': round(a['event_us'][k], 3), 'event_us_profiled': round(b['event_us'][k], 3),
                             'trace_us': round(sum(d) / len(d), 3) if d else None, 'trace_dispatches': len(d)}
    ga, gb = a['graph'], b['graph']
    per = ga['dispatches_per_replay']
    res['graph'] = {'us_per_replay_plain': round(ga['us_per_replay'], 3),
                    'us_per_replay_profiled': round(gb['us_per_replay'], 3),
                    'added_us_per_dispatch': round((gb['us_per_replay'] - ga['us_per_replay']) / per, 3)}
    kc = res['kernels']['k_multibox']
    if kc['trace_us']:
        kc['trace_over_event_plain'] = round(kc['trace_us'] / kc['event_us_plain'] - 1.0, 4)
    txt = json.dumps(res, indent=1)
    print(txt)
    with open(out, 'w') as f:
        f.write(txt + '\n')


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--out')
    ap.add_argument('--combine', nargs=4, metavar=('PLAIN', 'PROF', 'TRACE', 'OUT'))
    a = ap.parse_args()
    if a.combine:
        combine(*a.combine)
    else:
        measure(a.out)
