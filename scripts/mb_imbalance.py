#!/usr/bin/env python3
"""Which k_multibox workgroups are slow, and why (diagnostic; stamps build:
bash scripts/build_stamps_lib.sh, then SBOD_LIB=$PWD/variants/libsbod_hip_stamps.so).

One eager criterion half (matcher + loss pass) alone on the GPU, per resident batch, for the
headline (SSD512 B=32 f32) and C2 (B=16 bf16).  Per workgroup of k_multibox: start / end
(s_memrealtime, 100 MHz), the hardware CU / SE / XCD it ran on, its eight phase marks
(loss.hip MB_MARK: tile committed, positive list, wave 0's box regression, each wave's rows,
tile stored), and from the matcher's outputs of the same batch its positive rows, focal rows
(positives + negatives) and ignored rows.  Prints the correlations; --out writes every row.

    SBOD_LIB=... python scripts/mb_imbalance.py [--out gpurun_out/mb_imbalance.json]
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
from shape_based_object_detection_amd import core  # noqa: E402

REG = 4096
KID = 4   # k_multibox's stamp id in the loss translation unit


def read(lib, nblk):
    buf = (ctypes.c_ulonglong * (2 * (KID + 1) * REG))()
    lib.sbod_debug_stamps_loss(0, buf, (KID + 1) * REG)
    st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)[KID * REG:KID * REG + nblk]
    mk = (ctypes.c_ulonglong * (8 * REG))()
    lib.sbod_debug_mb_marks(mk, REG)
    marks = np.frombuffer(mk, dtype=np.uint64).reshape(-1, 8)[:nblk].astype(np.int64)
    start = st[:, 0].astype(np.int64)
    end = (st[:, 1] & np.uint64(0xffffffffffff)).astype(np.int64)
    hw = (st[:, 1] >> np.uint64(48)).astype(np.int64)
    return start, end, hw, marks


def tile_stats(st, bt, P):
    """positives / focal rows / ignored rows per (image, 256-prior tile), from the matcher itself"""
    gt = bt.stage.stage(bt.boxes, bt.labels)
    obj, ovl, npos = core.match(gt, st.crit.priors_xy, P, st.crit.threshold)
    ov = ovl.float().cpu().numpy()
    B = ov.shape[0]
    nt = (P + 255) // 256
    pad = np.full((B, nt * 256), np.nan, dtype=np.float32)
    pad[:, :P] = ov
    pad = pad.reshape(B, nt, 256)
    pos = (pad >= 0.5).sum(2)
    neg = (pad < 0.4).sum(2)
    rows = np.isfinite(pad).sum(2)
    return pos.reshape(-1), neg.reshape(-1), rows.reshape(-1)   # blk = x + nt * y order


def corr(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    if a.std() == 0 or b.std() == 0:
        return 0.0
    return float(np.corrcoef(a, b)[0, 1])


def analyse(rows):
    d = {k: np.array([r[k] for r in rows]) for k in rows[0]}
    dur = d['dur_us']
    out = {'blocks': len(dur), 'dur_p10_p50_p90_p99_max': [round(float(np.percentile(dur, q)), 2)
                                                           for q in (10, 50, 90, 99, 100)]}
    for k in ('pos', 'focal', 'start_us', 'per_cu', 'tile_x', 'commit_us', 'plist_us', 'regress_us',
              'rows_w0_us', 'rows_w123_us', 'store_us'):
        out['corr_dur_' + k] = round(corr(dur, d[k]), 3)
    out['dur_by_pos'] = {}
    for lo, hi in ((0, 0), (1, 8), (9, 32), (33, 64), (65, 256)):
        m = (d['pos'] >= lo) & (d['pos'] <= hi)
        if m.any():
            out['dur_by_pos']['%d-%d' % (lo, hi)] = [int(m.sum()), round(float(dur[m].mean()), 2),
                                                    round(float(d['regress_us'][m].mean()), 2)]
    out['dur_by_xcd'] = {int(x): round(float(dur[d['xcd'] == x].mean()), 2) for x in np.unique(d['xcd'])}
    out['dur_by_per_cu'] = {int(x): [int((d['per_cu'] == x).sum()), round(float(dur[d['per_cu'] == x].mean()), 2)]
                            for x in np.unique(d['per_cu'])}
    slow = dur >= np.percentile(dur, 95)
    out['slowest_5pct'] = {k: round(float(d[k][slow].mean()), 2) for k in
                           ('pos', 'focal', 'start_us', 'per_cu', 'commit_us', 'plist_us', 'regress_us',
                            'rows_w0_us', 'rows_w123_us', 'store_us', 'end_us')}
    out['median_all'] = {k: round(float(np.median(d[k])), 2) for k in
                         ('pos', 'focal', 'start_us', 'per_cu', 'commit_us', 'plist_us', 'regress_us',
                          'rows_w0_us', 'rows_w123_us', 'store_us', 'end_us')}
    # phases as medians of the per-workgroup segments
    return out


def run(label, B, dtype, reps=6):
    dev = torch.device('cuda', 0)
    lib = L.lib()
    for n, a in (('sbod_debug_stamps_loss', [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]),
                 ('sbod_debug_mb_marks', [ctypes.c_void_p, ctypes.c_int]),
                 ('sbod_debug_fin_marks', [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p])):
        getattr(lib, n).argtypes = a
    st = BM.Step(dev, B, 0, 1, graph=False, n_batches=6, dtype=dtype, priority='detect')
    P = st.P
    nt = (P + 255) // 256
    nblk = nt * B
    for _ in range(6):
        st.eager_half('criterion')
    torch.cuda.synchronize()
    rows, spans, fins = [], [], []
    for r in range(reps):
        lib.sbod_debug_stamps_loss(1 << KID, None, 0)
        lib.sbod_debug_mb_marks(None, 0)
        lib.sbod_debug_fin_marks(None, 0, None)
        st.eager_half('criterion')
        torch.cuda.synchronize()
        bt = st.batches[(st.k - 1) % len(st.batches)]
        start, end, hw, marks = read(lib, nblk)
        seen = (ctypes.c_ulonglong * REG)()
        fm = (ctypes.c_ulonglong * 8)()
        lib.sbod_debug_fin_marks(seen, REG, fm)
        seen = np.frombuffer(seen, dtype=np.uint64)[:nblk].astype(np.int64)
        fm = np.frombuffer(fm, dtype=np.uint64).astype(np.int64)
        lib.sbod_debug_stamps_loss(0, None, 0)
        pos, neg, nrow = tile_stats(st, bt, P)
        t0 = start.min()
        spans.append(round((end.max() - t0) / 100.0, 2))
        if fm[0]:
            # the fused finish: when each record was published (its block's mark 7, after the
            # record store) and when the gatherer first saw it
            pub = marks[:, 7]
            lag = (seen - pub) / 100.0
            last = int(np.argmax(pub))
            fins.append({'rep': r, 'enter_us': (fm[0] - t0) / 100.0, 'first_sweep_us': (fm[1] - t0) / 100.0,
                         'all_folded_us': (fm[2] - t0) / 100.0, 'written_us': (fm[3] - t0) / 100.0,
                         'sweeps_t0': int(fm[4]), 'last_pub_us': (pub.max() - t0) / 100.0,
                         'last_seen_us': (seen.max() - t0) / 100.0,
                         'lag_p50_p90_max_us': [round(float(np.percentile(lag, q)), 2) for q in (50, 90, 100)],
                         'lag_of_last_published_us': round(float(lag[last]), 2),
                         'kernel_end_us': (end.max() - t0) / 100.0})
        cu_count = {}
        for h in hw:
            cu_count[int(h)] = cu_count.get(int(h), 0) + 1
        for i in range(nblk):
            m = marks[i]
            rel = lambda v: (v - start[i]) / 100.0 if v else float('nan')
            w = [rel(m[3 + k]) for k in range(4)]
            rows.append({'rep': r, 'blk': i, 'tile_x': i % nt, 'img': i // nt, 'pos': int(pos[i]),
                         'focal': int(neg[i] + pos[i]), 'rows': int(nrow[i]),
                         'start_us': (start[i] - t0) / 100.0, 'end_us': (end[i] - t0) / 100.0,
                         'dur_us': (end[i] - start[i]) / 100.0, 'hw': int(hw[i]), 'cu': int(hw[i] & 0xf),
                         'se': int((hw[i] >> 4) & 0x3), 'xcd': int(hw[i] >> 6), 'per_cu': cu_count[int(hw[i])],
                         'commit_us': rel(m[0]), 'plist_us': rel(m[1]), 'regress_us': rel(m[2]),
                         'rows_w0_us': w[0], 'rows_w123_us': float(np.nanmax(w[1:])), 'store_us': rel(m[7])})
    res = {'label': label, 'B': B, 'spans_us': spans, 'finish': fins, 'analysis': analyse(rows)}
    print(json.dumps(res), flush=True)
    del st
    torch.cuda.synchronize()
    return res, rows


def main():
    out = {}
    allrows = {}
    for label, B, dt in (('headline_f32_b32', 32, torch.float32), ('c2_bf16_b16', 16, torch.bfloat16)):
        res, rows = run(label, B, dt)
        out[label] = res
        allrows[label] = rows
    if '--out' in sys.argv:
        path = sys.argv[sys.argv.index('--out') + 1]
        with open(path, 'w') as f:
            json.dump({'summary': out, 'rows': allrows}, f)


if __name__ == '__main__':
    main()
