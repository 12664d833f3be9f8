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
boxes, labels = synth.make_gt(32, seed=0)
locs, scores = synth.make_preds(32, Pn.shape[0], 21, seed=0)
det = scores.clone()
det[:, :, 0] += 6.0
locs, scores, det = locs.to(dev), scores.to(dev), det.to(dev)
crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=Cfg(reg_weights=1.0, device=dev, n_classes=21,
                                                       reg_loss='diou', cls_loss='focal'))
lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
for _ in range(2):
    crit(lo, sc, [b.to(dev) for b in boxes], [l.to(dev) for l in labels]).backward()
    core.detect(locs, det, 0.01, 0.45, 200, pri)
torch.cuda.synchronize()
print('done', flush=True)
