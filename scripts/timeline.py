#!/usr/bin/env python3
"""Per-workgroup timeline of one dispatch of each hot-path kernel (diagnostic library built with
-DSBOD_BLOCK_STAMPS: SBOD_LIB=.../libsbod_hip_stamps.so).  For each kernel: dispatch span, how
the workgroup starts spread (launch ramp / later rounds), per-workgroup duration, the tail.

    SBOD_LIB=$PWD/shape_based_object_detection_amd/lib/libsbod_hip_stamps.so python scripts/timeline.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import _lib as L, core, synth  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402


class Cfg(dict):
    __getattr__ = dict.__getitem__


def main():
    dev = torch.device('cuda')
    B, C = 32, 21
    Pn = prior_table('SSD512')
    P = Pn.shape[0]
    pri = torch.from_numpy(Pn).to(dev)
    import bench
    batches = [bench.Batch(B, 100 * i, dev) for i in range(6)]   # rotated: inputs come from HBM
    cfg = Cfg(reg_weights=1.0, device=dev, n_classes=C, reg_loss='diou', cls_loss='focal')
    crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
    k = [0, 0]

    def crit_step():
        bt = batches[k[0] % 6]
        k[0] += 1
        bt.locs.grad = None
        bt.scores.grad = None
        crit(bt.locs, bt.scores, bt.boxes, bt.labels).backward()

    def det_step():
        bt = batches[k[1] % 6]
        k[1] += 1
        core.detect(bt.locs.detach(), bt.det_scores, 0.01, 0.45, 200, pri)

    lib = L.lib()
    kernels = [('match', 5, 'k_match_tile', crit_step, B * ((P + 255) // 256)),
               ('loss', 4, 'k_multibox', crit_step, B * ((P + 255) // 256)),
               ('nms', 1, 'k_det_prepare', det_step, B * ((P + 255) // 256)),
               ('nms', 2, 'k_det_segment_w4', det_step, B * (C - 1)),
               ('nms', 3, 'k_det_merge', det_step, B)]
    for _ in range(20):
        crit_step()
        det_step()
    torch.cuda.synchronize()
    out = {}
    for tu, kid, name, fn, nblk in kernels:
        f = getattr(lib, 'sbod_debug_stamps_' + tu)
        f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        res = []
        for rep in range(3):
            f(1 << kid, None, 0)
            fn()
            torch.cuda.synchronize()
            reg = 4096   # SBOD_STAMP_REGION: kernel id k owns workgroups [k * reg, (k + 1) * reg)
            buf = np.zeros(2 * 16 * reg, dtype=np.uint64)
            f(0, buf.ctypes.data, 16 * reg)
            buf = buf[2 * kid * reg: 2 * (kid * reg + min(nblk, reg))]
            st = (buf[0::2] & np.uint64(0xffffffffffff)).astype(np.int64)
            en_raw = buf[1::2]
            ok = st > 0
            en = (en_raw & np.uint64(0xffffffffffff)).astype(np.int64)
            cu = (en_raw >> np.uint64(48)).astype(np.int64)
            st, en, cu = st[ok], en[ok], cu[ok]
            t0 = st.min()
            s_us, e_us = (st - t0) / 100.0, (en - t0) / 100.0
            d_us = e_us - s_us
            pct = lambda x: [round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 100)]
            res.append({'blocks': int(ok.sum()), 'span_us': round(float(e_us.max()), 2),
                        'start_pct': pct(s_us), 'dur_pct': pct(d_us), 'end_pct': pct(e_us),
                        'distinct_cu_ids': int(len(np.unique(cu)))})
        out[name] = res[-1]
        print(name, json.dumps(res[-1]), flush=True)


if __name__ == '__main__':
    main()
