#!/usr/bin/env python3
"""Back-to-back (GPU-bound) timing of each hot-path component, to separate kernel speed from
host overhead.  Run on the GPU box, optionally under rocprofv3 --kernel-trace --stats.

    python scripts/microbench.py [--iters 200] [--batch 32]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import _lib as L, core, synth  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402


class Cfg(dict):
    __getattr__ = dict.__getitem__


def timeit(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3, (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--batch', type=int, default=32)
    a = ap.parse_args()
    dev = torch.device('cuda')
    B = a.batch
    Pn = prior_table('SSD512')
    P = Pn.shape[0]
    pri = torch.from_numpy(Pn).to(dev)
    boxes, labels = synth.make_gt(B, seed=0)
    locs, scores = synth.make_preds(B, P, 21, seed=0)
    det = scores.clone()
    det[:, :, 0] += 6.0
    bx, lb = [b.to(dev) for b in boxes], [l.to(dev) for l in labels]
    locs, scores, det = locs.to(dev), scores.to(dev), det.to(dev)
    cfg = Cfg(reg_weights=1.0, device=dev, n_classes=21, reg_loss='diou', cls_loss='focal')
    crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
    lo = locs.clone().requires_grad_(True)
    sc = scores.clone().requires_grad_(True)
    gt = core.pack_gt(bx, lb)
    pxy = crit.priors_xy
    out = {}

    def crit_step():
        lo.grad = None
        sc.grad = None
        crit(lo, sc, bx, lb).backward()
    out['criterion_fwd_bwd'] = timeit(crit_step, a.iters)
    out['match_only'] = timeit(lambda: core.match(gt, pxy, P), a.iters)
    obj, ovl, npos = core.match(gt, pxy, P)
    spec = crit._spec()

    def fused_only():
        with torch.no_grad():
            core.fused_criterion(lo, sc, gt, obj, ovl, npos, npos[B:], pri, spec, 0.5, 0.4)
    out['fused_loss_fwd_only'] = timeit(fused_only, a.iters)

    # detect kernels without the host sync (outputs preallocated)
    top_k = 200
    ob = torch.empty(B, top_k, 4, device=dev)
    ol = torch.empty(B, top_k, dtype=torch.int64, device=dev)
    os_ = torch.empty(B, top_k, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    nb = L.lib().sbod_detect_workspace_bytes(B, P, 21)
    ws = core.workspace(nb, dev, 'detect')
    stream = L.stream_of(det)

    def det_kernels():
        L.call('sbod_detect_f32', L.ptr(locs), L.ptr(det), B, P, 21, L.ptr(pri), None, 0, 0, 0.01, 0.45,
               top_k, -1.0, 0, 0, L.ptr(ob), L.ptr(ol), L.ptr(os_), L.ptr(cnt), None, None, None, L.ptr(ws), nb, stream)
    out['detect_kernels_only'] = timeit(det_kernels, a.iters)
    out['detect_api'] = timeit(lambda: core.detect(locs, det, 0.01, 0.45, top_k, pri), a.iters)
    print(json.dumps({k: {'gpu_us': round(v[0], 2), 'wall_us': round(v[1], 2)} for k, v in out.items()}))


if __name__ == '__main__':
    main()
