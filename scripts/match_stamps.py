#!/usr/bin/env python3
"""Where k_match_tile's time goes (diagnostic; stamps build: bash scripts/build_stamps_lib.sh, then
SBOD_LIB=<lib/variants/libsbod_hip_stamps*.so>).

One eager criterion half (matcher + loss pass) alone on the GPU per resident batch, SSD512 B=32.
Per k_match_tile workgroup: start / end (s_memrealtime, 100 MHz) and wave 0's four marks
(match.hip MATCH_WAVE_MARK: anchors reduced, first object chunk's ballot, object loop done, keys
flushed).  Prints the dispatch ramp (start spread), per-workgroup phase medians and the span.

    SBOD_LIB=... python scripts/match_stamps.py [--reps 6]
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
KID = 5   # k_match_tile's stamp id in the match translation unit


def pct(a, qs=(10, 50, 90, 99, 100)):
    return [round(float(np.percentile(a, q)), 2) for q in qs]


def main():
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 6
    dev = torch.device('cuda', 0)
    lib = L.lib()
    lib.sbod_debug_stamps_match.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    lib.sbod_debug_match_marks.argtypes = [ctypes.c_void_p, ctypes.c_int]
    st = BM.Step(dev, 32, 0, 1, graph=False, n_batches=6, dtype=torch.float32, priority='detect')
    P = st.P
    for _ in range(6):
        st.eager_half('criterion')
    torch.cuda.synchronize()
    out = []
    for r in range(reps):
        lib.sbod_debug_stamps_match(1 << KID, None, 0)
        lib.sbod_debug_match_marks(None, 0)
        st.eager_half('criterion')
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (2 * (KID + 1) * REG))()
        lib.sbod_debug_stamps_match(0, buf, (KID + 1) * REG)
        stp = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)[KID * REG:(KID + 1) * REG]
        n = int((stp[:, 0] != 0).sum())
        stp = stp[:n]
        mk = (ctypes.c_ulonglong * (4 * REG))()
        lib.sbod_debug_match_marks(mk, REG)
        marks = np.frombuffer(mk, dtype=np.uint64).reshape(-1, 4)[:n].astype(np.int64)
        start = stp[:, 0].astype(np.int64)
        end = (stp[:, 1] & np.uint64(0xffffffffffff)).astype(np.int64)
        t0 = start.min()
        rel = lambda v: (v - start) / 100.0
        row = {'rep': r, 'blocks': n, 'span_us': round((end.max() - t0) / 100.0, 2),
               'start_us': pct((start - t0) / 100.0), 'end_us': pct((end - t0) / 100.0),
               'dur_us': pct((end - start) / 100.0),
               'm0_anchors_us': pct(rel(marks[:, 0])), 'm1_gt_us': pct(rel(marks[:, 1])),
               'm2_loop_us': pct(rel(marks[:, 2])), 'm3_flush_us': pct(rel(marks[:, 3])),
               'loop_only_us': pct((marks[:, 2] - marks[:, 1]) / 100.0),
               'flush_only_us': pct((marks[:, 3] - marks[:, 2]) / 100.0),
               'tail_us': pct((end - marks[:, 3]) / 100.0)}
        nt = n // 32   # grid (tiles, B): block i = tile i % nt of image i // nt
        slow = np.argsort(end - start)[-8:]
        row['slowest_tiles_tile_img_us'] = [[int(i % nt), int(i // nt), round(float(end[i] - start[i]) / 100.0, 2)]
                                            for i in slow]
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
