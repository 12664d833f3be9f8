#!/usr/bin/env python3
"""Config C2 (SSD512 B=16 bf16) step under several step structures, one box, in turn: wall time
per pipelined step and the host's share of it (submit = time inside launch_replay, collect = the
oldest step's wait + list building), so the line says whether the C2 step is host- or GPU-bound.

    python scripts/c2_probe.py [--steps 400] [--out gpurun_out/c2_probe.jsonl]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402

VARIANTS = [
    dict(depth=4), dict(depth=4, gt_fold=False), dict(depth=6), dict(depth=8),
    dict(depth=6, crit_streams=3, det_streams=3), dict(depth=4, dtype='f32'),
]


def run(dev, steps, depth=4, gt_fold=True, crit_streams=2, det_streams=2, dtype='bf16', B=16, n_batches=12,
        nogc=False, det_form='two'):
    import gc
    if nogc:
        gc.collect()
        gc.disable()
    st = BM.Step(dev, B, 0, 1, graph=True, n_batches=n_batches,
                 dtype=torch.bfloat16 if dtype == 'bf16' else torch.float32, priority='detect', depth=depth,
                 crit_streams=crit_streams, det_streams=det_streams, gt_fold=gt_fold, det_form=det_form)
    for _ in range(3):
        st.eager_split()
    torch.cuda.synchronize()
    st.capture()
    for _ in range(len(st.slots) + 1):
        st.replay()
    torch.cuda.synchronize()
    res = []
    with torch.cuda.stream(st.cap_stream):
        for _ in range(3):
            for _ in range(20):
                st.pipelined()
            st.drain()
            torch.cuda.synchronize()
            st.host_submit = st.host_collect = 0.0
            t = time.perf_counter()
            for _ in range(steps):
                st.pipelined()
            st.drain()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            res.append((dt / steps * 1e3, st.host_submit / steps * 1e6, st.host_collect / steps * 1e6))
    res.sort()
    ms, sub, col = res[1]
    if nogc:
        gc.enable()
    del st
    torch.cuda.synchronize()
    return {'ms_per_step': round(ms, 4), 'submit_us': round(sub, 1), 'collect_us': round(col, 1),
            'runs_ms': [round(r[0], 4) for r in res]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=400)
    ap.add_argument('--out')
    ap.add_argument('--variants', help='JSON list of variant dicts (default: the built-in list)')
    ap.add_argument('--rounds', type=int, default=2)
    a = ap.parse_args()
    variants = json.loads(a.variants) if a.variants else VARIANTS
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    out = open(a.out, 'w') if a.out else None
    for rnd in range(a.rounds):
        for v in variants:
            r = dict(v, round=rnd, **run(dev, a.steps, **v))
            print(json.dumps(r), flush=True)
            if out:
                out.write(json.dumps(r) + '\n')
                out.flush()


if __name__ == '__main__':
    main()
