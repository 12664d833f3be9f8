#!/usr/bin/env python3
"""cProfile of the bench step's host side on the GPU box (where does the Python time go)."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR, utils as MU  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402

dev = torch.device('cuda')
Pn = prior_table('SSD512')
pri = torch.from_numpy(Pn).to(dev)
cfg = bench.Cfg(reg_weights=1.0, device=dev, n_classes=21, reg_loss='diou', cls_loss='focal',
                focal_type='softmax', model={'box_type': 'offset'})
crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
boxes, labels, locs0, scores0, det = bench.make_batch(32, 0, dev)
locs = locs0.clone().requires_grad_(True)
scores = scores0.clone().requires_grad_(True)


def step():
    locs.grad = None
    scores.grad = None
    crit(locs, scores, boxes, labels).backward()
    MU.detect(locs.detach(), det, 0.01, 0.45, 200, pri, cfg)


for _ in range(20):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumulative").print_stats(40)
