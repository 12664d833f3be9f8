"""BASELINE config C1: SSD300 on 4 synthetic VOC-format images, one criterion step.

The batch comes through the reference's data path (VOC JSON files -> PascalVOCDataset ->
DataLoader with collate_fn); its host lists go to the device in ONE copy
(GtStaging's host path) and MultiBoxLoss300 runs fwd+bwd on the HIP path.  Checked against the
oracle on the same lists (loss and gradients within 1e-4 relative; gradients with a 1e-8 absolute
floor for entries that are ~0)."""
import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader

from oracle import loss_ref as LR
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.dataset import Datasets as D
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('reg,cls', [('smoothl1', 'ce'), ('diou', 'focal')])
def test_c1_ssd300_voc_batch_step(tmp_path, reg, cls):
    folder = D.write_synthetic_voc(str(tmp_path), 4, size=(300, 300), split='TRAIN', seed=11)
    ds = D.PascalVOCDataset(folder, 'train', (300, 300),
                            {'model': {'operation_list': ['expand', 'random_crop'], 'return_percent_coords': True}})
    torch.manual_seed(1)
    images, boxes, labels, _, _ = next(iter(DataLoader(ds, batch_size=4, shuffle=False,
                                                       collate_fn=ds.collate_fn)))
    assert images.shape == (4, 3, 300, 300)
    P = torch.from_numpy(prior_table('SSD300'))
    assert P.shape[0] == 8732
    stage = core.GtStaging(4, 16, DEV)
    gt = stage.stage(boxes, labels)                       # host lists -> one host->device copy
    locs, scores = synth.make_preds(4, P.shape[0], 21, seed=11)
    crit = CR.MultiBoxLoss300(priors_cxcy=P.to(DEV), config={'reg_weights': 1.0, 'device': DEV,
                                                             'n_classes': 21, 'reg_loss': reg,
                                                             'cls_loss': cls})
    lo = locs.to(DEV).requires_grad_(True)
    sc = scores.to(DEV).requires_grad_(True)
    loss = crit(lo, sc, gt, None)
    loss.backward()
    # the same step with the lists moved image by image (train_anchor.py:266-268)
    lo2 = locs.to(DEV).requires_grad_(True)
    sc2 = scores.to(DEV).requires_grad_(True)
    loss2 = crit(lo2, sc2, [b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    loss2.backward()
    assert loss.item() == loss2.item()
    assert torch.equal(lo.grad, lo2.grad) and torch.equal(sc.grad, sc2.grad)
    rl, rs = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    oreg = 'l1' if reg == 'smoothl1' else reg
    ref = LR.criterion('ssd300', P, rl, rs, boxes, labels, oreg, cls)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-4)
    np.testing.assert_allclose(lo.grad.cpu().numpy(), rl.grad.numpy(), rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(sc.grad.cpu().numpy(), rs.grad.numpy(), rtol=1e-4, atol=1e-8)
