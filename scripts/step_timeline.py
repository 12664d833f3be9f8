#!/usr/bin/env python3
"""Concurrent timeline of the bench's captured step (diagnostic; stamps build:
SBOD_LIB=$PWD/variants/libsbod_hip_stamps.so, scripts/build_stamps_lib.sh).  Every kernel of the
step records per-workgroup wall-clock start / end (s_memrealtime, one clock for both streams);
after N pipelined steps the last launch of each kernel is printed on one time axis — where the
criterion graph (cap_stream) and the detect graph (det_stream) overlap, and what each kernel
costs inside the real step (not alone, not under a profiler).

    SBOD_LIB=... python scripts/step_timeline.py [--steps N] [--mode pipelined|crit|det]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402

REG = 4096   # SBOD_STAMP_REGION
KERNELS = [('gtpack', 8, 'k_gt_pack'), ('match', 5, 'k_match_tile'), ('match', 7, 'k_match_final'),
           ('loss', 4, 'k_multibox'), ('loss', 6, 'k_loss_final'), ('nms', 1, 'k_det_prepare'),
           ('nms', 2, 'k_det_segment_w4'), ('nms', 3, 'k_det_merge')]


def main():
    steps = int(sys.argv[sys.argv.index('--steps') + 1]) if '--steps' in sys.argv else 20
    mode = sys.argv[sys.argv.index('--mode') + 1] if '--mode' in sys.argv else 'pipelined'
    order = sys.argv[sys.argv.index('--order') + 1] if '--order' in sys.argv else 'criterion_first'
    prio = sys.argv[sys.argv.index('--priority') + 1] if '--priority' in sys.argv else 'detect'
    nds = int(sys.argv[sys.argv.index('--det-streams') + 1]) if '--det-streams' in sys.argv else 2
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    lib = L.lib()
    fns = {}
    for tu in ('gtpack', 'match', 'loss', 'nms'):
        f = getattr(lib, 'sbod_debug_stamps_' + tu)
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        fns[tu] = f
    st = bench.Step(dev, 32, 0, 1, graph=True, two_streams=True, priority=prio, order=order, det_streams=nds)
    for _ in range(3):
        st.eager_split()
    torch.cuda.synchronize()
    st.capture()
    for _ in range(len(st.slots) + 1):
        st()
    torch.cuda.synchronize()
    arm = 0
    for _, kid, _ in KERNELS:
        arm |= 1 << kid
    for f in fns.values():
        f(arm, None, 0)

    def crit_only():
        i = st.k % len(st.slots)
        st._next_batch()
        with torch.cuda.stream(st.cap_stream):
            st.slots[i][0].replay()

    def det_only():
        i = st.k % len(st.slots)
        st._next_batch()
        with torch.cuda.stream(st.det_streams[i % len(st.det_streams)]):
            st.slots[i][1].replay()

    fn = {'pipelined': st.pipelined, 'crit': crit_only, 'det': det_only}[mode]
    ctx = torch.cuda.stream(st.cap_stream)   # as bench.py's timed loop
    ctx.__enter__()
    reps = []
    for rep in range(3):
        for _ in range(steps):
            fn()
        if mode == 'pipelined':
            st.drain()
        torch.cuda.synchronize()
        rows = []
        bufs = {}
        for tu in fns:   # one read per translation unit: each read clears that unit's buffer
            bufs[tu] = np.zeros(2 * 16 * REG, dtype=np.uint64)
            fns[tu](arm, bufs[tu].ctypes.data, 16 * REG)   # read, clear, stay armed
        for tu, kid, name in KERNELS:
            b = bufs[tu][2 * kid * REG: 2 * (kid + 1) * REG]
            s = (b[0::2] & np.uint64(0xffffffffffff)).astype(np.int64)
            e = (b[1::2] & np.uint64(0xffffffffffff)).astype(np.int64)
            ok = s > 0
            if ok.any():
                rows.append((name, s[ok], e[ok]))
        t0 = min(r[1].min() for r in rows)
        out = {}
        for name, s, e in rows:
            d = (e - s) / 100.0
            out[name] = {'blocks': int(len(s)), 'first_start': round((s.min() - t0) / 100.0, 2),
                         'median_start': round((np.median(s) - t0) / 100.0, 2),
                         'last_end': round((e.max() - t0) / 100.0, 2),
                         'span': round((e.max() - s.min()) / 100.0, 2),
                         'block_us_median': round(float(np.median(d)), 2),
                         'block_us_max': round(float(d.max()), 2)}
        reps.append(out)
        print(json.dumps({'mode': mode, 'order': order, 'priority': prio, 'det_streams': nds, 'rep': rep,
                          'kernels': out}), flush=True)


if __name__ == '__main__':
    main()
