#!/usr/bin/env python3
"""Per-workgroup wall-clock stamps of the criterion's kernels (diagnostic; stamps build:
EXTRA=-DSBOD_BLOCK_STAMPS bash scripts/build_lib_variant.sh stamps, then
SBOD_LIB=$PWD/shape_based_object_detection_amd/lib/variants/libsbod_hip_stamps.so).  One eager
criterion half (matcher + loss pass, fwd+bwd) alone on the GPU, for C2 (B=16 bf16) and the
headline (B=32 f32): per kernel the launch ramp (first -> last workgroup start), the workgroup
durations, and the tail (last end after the second-to-last end: the finish's last arriver).
Times in microseconds from the matcher's first start (s_memrealtime, 100 MHz).

    SBOD_LIB=... python scripts/c2_stamps.py [--out gpurun_out/c2_stamps.json]
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402

REG = 4096
KERNELS = [('match', 5, 'k_match_tile'), ('match', 7, 'k_match_final'), ('loss', 4, 'k_multibox')]


def stamps_of(fns, nblk):
    out = {}
    for tu, kid, name in KERNELS:
        n = (kid + 1) * REG
        buf = (ctypes.c_ulonglong * (2 * n))()
        fns[tu](0, buf, n)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)[kid * REG:(kid + 1) * REG]
        a = a[a[:, 0] != 0]
        out[name] = (a[:, 0].astype(np.int64), (a[:, 1] & np.uint64(0xffffffffffff)).astype(np.int64))
    return out


def summary(st, t0):
    s, e = st
    d = (e - s) / 100.0
    es = np.sort(e)
    return {'blocks': int(len(s)), 'first_start_us': round((s.min() - t0) / 100.0, 2),
            'ramp_us': round((s.max() - s.min()) / 100.0, 2),
            'dur_us_p10_p50_p90_max': [round(float(np.percentile(d, q)), 2) for q in (10, 50, 90, 100)],
            'end_us': round((e.max() - t0) / 100.0, 2),
            'tail_us': round((es[-1] - es[-2]) / 100.0, 2) if len(es) > 1 else 0.0,
            'span_us': round((e.max() - s.min()) / 100.0, 2)}


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    lib = L.lib()
    fns = {}
    for tu in ('match', 'loss'):
        f = getattr(lib, 'sbod_debug_stamps_' + tu)
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        fns[tu] = f
    arm = sum(1 << kid for _, kid, _ in KERNELS)
    res = {}
    for label, B, dt in (('c2_bf16_b16', 16, torch.bfloat16), ('c1_f32_b32', 32, torch.float32),
                         ('bf16_b32', 32, torch.bfloat16)):
        st = BM.Step(dev, B, 0, 1, graph=False, n_batches=6, dtype=dt, priority='detect')
        for _ in range(4):
            st.eager_half('criterion')
        torch.cuda.synchronize()
        runs = []
        for _ in range(5):
            for f in fns.values():
                f(arm, None, 0)
            st.eager_half('criterion')
            torch.cuda.synchronize()
            sm = stamps_of(fns, None)
            for f in fns.values():
                f(0, None, 0)
            t0 = min(v[0].min() for v in sm.values() if len(v[0]))
            runs.append({k: summary(v, t0) for k, v in sm.items() if len(v[0])})
        res[label] = runs
        print(label, json.dumps(runs[-1]), flush=True)
        del st
        torch.cuda.synchronize()
    if '--out' in sys.argv:
        with open(sys.argv[sys.argv.index('--out') + 1], 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
