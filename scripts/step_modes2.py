#!/usr/bin/env python3
"""Where the bench step's GPU interval goes (diagnostic, round 6; the direct-submit step).

Steady-state wall time per step (N back-to-back submits over the resident batches, one final
synchronize) of the step's recorded entry-point calls: criterion alone, detect alone, both (the
step's streams: 2 criterion + 2 detect, alternating), and each half on ONE stream (its per-step
chain latency, no overlap between steps); plus the host cost of one submit of each half with the
GPU idle.  The GT packing is not re-issued (each batch's staging buffers already hold its GT).

    python scripts/step_modes2.py [--steps N]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402

N = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 300
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
L.lib()
st = bench.Step(dev, 32, 0, 1, graph=True, two_streams=True, priority='detect', submit='direct', gt_fold=False)
for _ in range(3):
    st.eager_split()
torch.cuda.synchronize()
st.capture()
for _ in range(len(st.slots) + 1):
    st.replay()
torch.cuda.synchronize()
R = len(st.slots)
crit = [s[0] for s in st.slots]
det = [s[1] for s in st.slots]


def on_stream(calls, raw):
    return [(n, tuple(a[:-1]) + (raw,)) for n, a in calls]


one_c = [on_stream(c, st.cap_streams[0].cuda_stream) for c in crit]
one_d = [on_stream(c, st.det_streams[0].cuda_stream) for c in det]


def wall(fn, n=N):
    for i in range(12):
        fn(i % R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i % R)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


def host(fn):
    tt = []
    for i in range(40):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(i % R)
        tt.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    tt.sort()
    return round(tt[len(tt) // 2] * 1e6, 2)


out = {'steps': N, 'resident_batches': R}
for rep in range(2):
    r = {}
    r['criterion_only'] = wall(lambda i: L.replay_calls(crit[i]))
    r['detect_only'] = wall(lambda i: L.replay_calls(det[i]))
    r['both'] = wall(lambda i: (L.replay_calls(crit[i]), L.replay_calls(det[i])))
    r['criterion_one_stream'] = wall(lambda i: L.replay_calls(one_c[i]))
    r['detect_one_stream'] = wall(lambda i: L.replay_calls(one_d[i]))
    r['both_one_stream_each'] = wall(lambda i: (L.replay_calls(one_c[i]), L.replay_calls(one_d[i])))
    r['host_criterion_us'] = host(lambda i: L.replay_calls(crit[i]))
    r['host_detect_us'] = host(lambda i: L.replay_calls(det[i]))
    out['rep%d' % rep] = r
print(json.dumps(out), flush=True)
