"""One bench-shaped criterion fwd+bwd and detect call (B=32 SSD512, +6 background for detect) on
the phase-clock debug library (SBOD_LIB=.../libsbod_hip_phase.so): the kernels print per-phase
cycle stamps of a few blocks."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core, synth  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402


class Cfg(dict):
    __getattr__ = dict.__getitem__


dev = torch.device('cuda')
Pn = prior_table('SSD512')
pri = torch.from_numpy(Pn).to(dev)
import bench  # noqa: E402
batches = [bench.Batch(32, 100 * i, dev) for i in range(6)]   # rotated: inputs come from HBM
crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=Cfg(reg_weights=1.0, device=dev, n_classes=21,
                                                       reg_loss='diou', cls_loss='focal'))
for i in range(8):      # the last iterations' lines are the steady state
    bt = batches[i % 6]
    print('== iteration %d' % i, flush=True)
    crit(bt.locs, bt.scores, bt.boxes, bt.labels).backward()
    core.detect(bt.locs.detach(), bt.det_scores, 0.01, 0.45, 200, pri)
    torch.cuda.synchronize()
print('done', flush=True)
