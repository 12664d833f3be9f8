#!/usr/bin/env python3
"""Host cost of each piece of the bench's per-step submit and collect (graph mode, SSD512 B=32),
GPU idle before every measured call (a synchronize after each), median of N calls, microseconds:

  submit_total      Step.launch_replay(): GT packing + both graph launches + the detect event
  pack_only         _sbodhost.pack_device_lists (list checks + one sbod_gt_pack launch)
  graph_criterion   sbod_graph_launch of one criterion graph
  graph_detect      sbod_graph_launch of one detect graph
  event_record      sbod_event_record
  null_launch       sbod_null_kernel (one hipLaunchKernel of an empty kernel)
  collect_ready     DetectHandle.wait() once the GPU has finished (pinned counts -> lists)
  step_pipelined    the bench's pipelined step, back to back (the wall time per step)

    python scripts/submit_probe.py [--out gpurun_out/submit_probe.json]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402
from shape_based_object_detection_amd import core  # noqa: E402


def med(xs):
    xs = sorted(xs)
    return round(xs[len(xs) // 2] * 1e6, 2)


def timed_idle(fn, n):
    out = []
    for i in range(n + 5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        dt = time.perf_counter() - t
        if i >= 5:
            out.append(dt)
    torch.cuda.synchronize()
    return med(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out')
    ap.add_argument('--n', type=int, default=200)
    ap.add_argument('--B', type=int, default=32)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    st = BM.Step(dev, a.B, 0, 1, graph=True, n_batches=6, submit='graph', depth=2)
    for _ in range(3):
        st.eager_split()
    torch.cuda.synchronize()
    st.capture()
    for _ in range(len(st.slots) + 1):
        st.replay()
    torch.cuda.synchronize()
    res = {'B': a.B, 'n': a.n}
    with torch.cuda.stream(st.cap_stream):
        res['submit_total'] = timed_idle(lambda: st.launch_replay()[1].wait(), a.n)   # incl. collect
        hs = []

        def sub():
            hs.append(st.launch_replay()[1])
        res['submit_only'] = timed_idle(sub, a.n)
        for h in hs:
            h.wait()
        hs.clear()
        ext = L.host_ext
        bt = st.batches[0]
        stg = bt.stage
        res['pack_only'] = timed_idle(lambda: ext.pack_device_lists(
            bt.boxes, bt.labels, stg.boxes.shape[0], stg.capacity, 0, stg.boxes.data_ptr(), stg.labels.data_ptr(),
            stg.offsets.data_ptr(), st.cap_stream.cuda_stream, False), a.n)
        launches, ev, ev_stream, _ = st.fast[0]
        res['graph_criterion'] = timed_idle(lambda: L.call('sbod_graph_launch', launches[0][0], launches[0][1]), a.n)
        res['graph_detect'] = timed_idle(lambda: L.call('sbod_graph_launch', launches[1][0], launches[1][1]), a.n)
        res['event_record'] = timed_idle(lambda: L.call('sbod_event_record', ev, ev_stream), a.n)
        res['null_launch'] = timed_idle(lambda: L.call('sbod_null_kernel', 1, st.cap_stream.cuda_stream), a.n)
        # collect once the GPU is done
        coll = []
        for i in range(a.n + 5):
            h = st.launch_replay()[1]
            torch.cuda.synchronize()
            t = time.perf_counter()
            h.wait()
            if i >= 5:
                coll.append(time.perf_counter() - t)
        res['collect_ready'] = med(coll)
        # the pipelined step back to back
        st.pending.clear()
        for _ in range(20):
            st.pipelined()
        st.drain()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.n):
            st.pipelined()
        st.drain()
        torch.cuda.synchronize()
        res['step_pipelined'] = round((time.perf_counter() - t) / a.n * 1e6, 2)
    print(json.dumps(res), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
