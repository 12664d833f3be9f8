#!/usr/bin/env python3
"""Host cost of the drop-in API path: the calls train_anchor.py:271-284 and
:342-363 make — ``criterion(locs, scores, boxes, labels)`` of the reference-named class,
``loss.backward()``, ``models.utils.detect(...)`` — on SSD512 B=32, 6 resident batches.
Per call host time, the synchronous step, the pipelined step (detect collected 3 steps later,
``async_=True``), and a cProfile of the pipelined loop (top functions by own time).

    python scripts/api_profile.py [--out gpurun_out/api_profile.json] [--steps 200]
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402
from shape_based_object_detection_amd.models import utils as MU  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402


def main():
    steps = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 200
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    B = 32
    st = BM.Step(dev, B, 0, 1, graph=False, n_batches=6)
    crit = CR.MultiBoxLoss512(priors_cxcy=st.priors, config=st.cfg)
    pri = st.priors
    cfg = st.cfg

    def step(k, async_):
        bt = st.batches[k % len(st.batches)]
        bt.locs.grad = None
        bt.scores.grad = None
        t0 = time.perf_counter()
        loss = crit(bt.locs, bt.scores, bt.boxes, bt.labels)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        h = MU.detect(bt.locs.detach(), bt.det_scores, 0.01, 0.45, 200, pri, cfg, async_=async_)
        t3 = time.perf_counter()
        return loss, h, (t1 - t0, t2 - t1, t3 - t2)

    for k in range(10):
        step(k, False)
    torch.cuda.synchronize()
    # synchronous API step (lists returned by detect each step)
    t0 = time.perf_counter()
    parts = [0.0, 0.0, 0.0]
    for k in range(steps):
        _, _, p = step(k, False)
        parts = [a + b for a, b in zip(parts, p)]
    torch.cuda.synchronize()
    sync_ms = (time.perf_counter() - t0) / steps * 1e3
    # pipelined: step k issued before step k-3's lists are collected
    depth = 4

    def pipelined(n):
        pend = []
        sub = [0.0, 0.0, 0.0]
        coll = 0.0
        for k in range(n):
            loss, h, p = step(k, True)
            sub = [a + b for a, b in zip(sub, p)]
            pend.append((loss, h))
            if len(pend) >= depth:
                t = time.perf_counter()
                pend.pop(0)[1].wait()
                coll += time.perf_counter() - t
        for _, h in pend:
            h.wait()
        return sub, coll

    pipelined(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sub, coll = pipelined(steps)
    torch.cuda.synchronize()
    pipe_ms = (time.perf_counter() - t0) / steps * 1e3
    pr = cProfile.Profile()
    pr.enable()
    pipelined(100)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(45)
    res = {'B': B, 'steps': steps, 'api_sync_ms_per_step': round(sync_ms, 4),
           'api_pipelined_ms_per_step': round(pipe_ms, 4), 'pipeline_depth': depth,
           'host_us_per_call_sync': {'criterion': round(parts[0] / steps * 1e6, 1),
                                     'backward': round(parts[1] / steps * 1e6, 1),
                                     'detect': round(parts[2] / steps * 1e6, 1)},
           'host_us_per_call_pipelined': {'criterion': round(sub[0] / steps * 1e6, 1),
                                          'backward': round(sub[1] / steps * 1e6, 1),
                                          'detect_launch': round(sub[2] / steps * 1e6, 1),
                                          'collect_incl_wait': round(coll / steps * 1e6, 1)}}
    print(json.dumps(res), flush=True)
    print(s.getvalue()[:6000], flush=True)
    if '--out' in sys.argv:
        res['cprofile_top'] = s.getvalue()[:20000]
        with open(sys.argv[sys.argv.index('--out') + 1], 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
