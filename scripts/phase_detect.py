"""One bench-shaped detect call (B=32 SSD512, +6 background) on the phase-clock debug library
(SBOD_LIB=.../libsbod_hip_phase.so): the kernels print per-phase cycle stamps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core, synth  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402

dev = torch.device('cuda')
Pn = prior_table('SSD512')
pri = torch.from_numpy(Pn).to(dev)
locs, scores = synth.make_preds(32, Pn.shape[0], 21, seed=0)
scores[:, :, 0] += 6.0
locs, scores = locs.to(dev), scores.to(dev)
for _ in range(2):
    core.detect(locs, scores, 0.01, 0.45, 200, pri)
torch.cuda.synchronize()
print('done', flush=True)
