#!/usr/bin/env python3
"""Where the graph-mode bench step's time goes (diagnostic): wall time per step of N back-to-back
submits of (a) the criterion graph alone, (b) the detect graph alone, (c) both (one C++ submit,
no host wait), (d) the bench's pipelined step (submit + collect of the previous detections), and
the host cost of one C++ submit.  GPU-bound modes show the device time of their graphs; (c) vs
max(a, b) shows how well the two streams overlap."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402

N = 200
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
L.lib()
C2 = '--c2' in sys.argv      # config C2: SSD512 B=16 bf16, 12 resident batches (bench c2_figure)
st = (bench.Step(dev, 16, 0, 1, graph=True, n_batches=12, dtype=torch.bfloat16) if C2 else
      bench.Step(dev, 32, 0, 1, graph=True, two_streams=True))
for _ in range(3):
    st.eager_split()
torch.cuda.synchronize()
st.capture()
for _ in range(len(st.slots) + 1):
    st()
torch.cuda.synchronize()


def wall(fn, n=N):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


R = len(st.slots)   # resident batches: every mode rotates through them (HBM-resident inputs)
k = [0]


def rot(fn):
    def f():
        i = k[0] % R
        k[0] += 1
        fn(i)
    return f


out = {'config': 'C2 bf16 B=16' if C2 else 'SSD512 fp32 B=32', 'resident_batches': R}
with torch.cuda.stream(st.cap_stream):
    out['criterion_graph_only'] = wall(rot(lambda i: st.slots[i][0].replay()))
with torch.cuda.stream(st.det_stream):
    out['detect_graph_only'] = wall(rot(lambda i: st.slots[i][1].replay()))


def both(i):
    bt = st.batches[i]
    launches, ev, ev_stream = st.fast[i]
    st.batches[0].stage.stage_and_replay(bt.boxes, bt.labels, launches, ev, ev_stream)


out['both_one_submit_no_wait'] = wall(rot(both))
launches, ev, ev_stream = st.fast[0]
ga, gb = st.slots[0][0], st.slots[0][1]
out['pipelined_step'] = wall(st.pipelined)
st.drain()
torch.cuda.synchronize()
# host cost of one submit while the GPU is idle
tt = []
for _ in range(50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.batches[0].stage.stage_and_replay(st.batches[0].boxes, st.batches[0].labels, launches, ev, ev_stream)
    tt.append(time.perf_counter() - t0)
tt.sort()
out['submit_host_us_median'] = round(tt[len(tt) // 2] * 1e6, 2)
for name, g, s in (('criterion', ga, st.cap_stream), ('detect', gb, st.det_stream)):
    tt = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.call('sbod_graph_launch', g.raw_cuda_graph_exec(), s.cuda_stream)
        tt.append(time.perf_counter() - t0)
    tt.sort()
    out['graph_launch_host_us_%s' % name] = round(tt[len(tt) // 2] * 1e6, 2)
torch.cuda.synchronize()
print(json.dumps(out), flush=True)
