"""Host cost of the pieces of one graph-mode bench step (diagnostic): GT staging, each graph
replay, stream switches, event records, the detect collection.  Wall time of the Python calls
only (the GPU work they enqueue is not waited for except where stated)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402
from shape_based_object_detection_amd import core  # noqa: E402

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
L.lib()
st = bench.Step(dev, 32, 0, 1, graph=True, two_streams=True)
with torch.cuda.stream(st.cap_stream):
    for _ in range(3):
        st.eager_split()
torch.cuda.synchronize()
st.capture()
for _ in range(5):
    st()
torch.cuda.synchronize()
N = 200


def t(fn, n=N, sync_every=8):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    for i in range(n):
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
        if i % sync_every == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return round(tot / n * 1e6, 2)


ga, gb, loss, h = st.slots[0]
out = {}
out['stage_device_lists'] = t(lambda: st.batches[0].stage.stage(st.boxes, st.labels))
out['as_rows'] = t(lambda: core._as_rows(st.boxes, st.labels))
bx, lb, _ = core._as_rows(st.boxes, st.labels)
counts = [b.shape[0] for b in st.boxes]
out['launch_pack_only'] = t(lambda: core._launch_pack(bx, lb, counts, st.batches[0].stage.boxes.shape[0], st.batches[0].stage.boxes,
                                                      st.batches[0].stage.labels, st.batches[0].stage.offsets))
out['graph_replay_criterion'] = t(ga.replay)
out['graph_replay_detect'] = t(gb.replay)


def ctx():
    with torch.cuda.stream(st.cap_stream):
        pass


out['stream_context'] = t(ctx)
ev = torch.cuda.Event()
out['event_record'] = t(lambda: ev.record(st.det_stream))
out['launch_replay_total'] = t(st.launch_replay)


def collect():
    _, hh = st.launch_replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hh.wait()
    return time.perf_counter() - t0


vals = [collect() for _ in range(50)]
out['wait_after_sync'] = round(sum(vals) / len(vals) * 1e6, 2)
print(json.dumps(out), flush=True)
