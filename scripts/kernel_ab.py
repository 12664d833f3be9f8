#!/usr/bin/env python3
"""Per-kernel device time (HIP events via sbod_timing_*) of the bench step's kernels, GPU-bound
(criterion fwd+bwd + detect back to back, 200 iterations over 6 HBM-resident batches).  Select the library with SBOD_LIB to
A/B two builds on one box:  SBOD_LIB=.../libsbod_hip_old.so python scripts/kernel_ab.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L, core  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402

dev = torch.device('cuda')
pri = torch.from_numpy(prior_table('SSD512')).to(dev)
cfg = bench.Cfg(reg_weights=1.0, device=dev, n_classes=21, reg_loss='diou', cls_loss='focal')
crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
# six resident batches rotated step by step, as bench.py does: every launch reads from HBM
batches = [bench.Batch(32, 100 * i, dev) for i in range(6)]
k = [0]


def step():
    bt = batches[k[0] % len(batches)]
    k[0] += 1
    bt.locs.grad = None
    bt.scores.grad = None
    crit(bt.locs, bt.scores, bt.boxes, bt.labels).backward()
    core.detect(bt.locs.detach(), bt.det_scores, 0.01, 0.45, 200, pri)


for _ in range(20):
    step()
torch.cuda.synchronize()
L.timing_enable('*')
for _ in range(200):
    step()
torch.cuda.synchronize()
out = {'lib': os.path.basename(L.LIB_PATH)}
for k in bench.ALL_KERNELS:
    n, ms = L.timing_query(k)
    if n:
        out[k] = round(ms / n * 1e3, 2)
L.timing_enable(None)
print(json.dumps(out), flush=True)
