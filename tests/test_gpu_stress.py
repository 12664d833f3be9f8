"""Parity at the largest sizes SURVEY §8 names: RetinaNet's generator on 896x896 maps
(P = 100,254 anchors, the C3 stress size) and config C3 itself (RetinaNet 512², B = 32,
P = 32,736).  The HIP path against the oracle on the same seeded inputs: matcher outputs
bit-exact, criterion loss and gradients within 1e-4 relative (north_star's fp32
tolerance), detect bit-exact on the kernels' own activations."""
import numpy as np
import pytest
import torch

from oracle import loss_ref as LR
from oracle import match_ref as M
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = 'cuda'


class Cfg(dict):
    __getattr__ = dict.__getitem__


def test_match_stress_100k_anchors():
    Pn = prior_table('RETINA896')
    assert Pn.shape[0] == 100254
    pxy = M.cxcy_to_xy(Pn)
    B = 4
    boxes, labels = synth.make_gt(B, seed=11, max_objects=40)
    gt = core.pack_gt([b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    obj, ovl, npos = core.match(gt, torch.from_numpy(pxy).to(DEV), Pn.shape[0])
    cls, neg, _, _ = core.match_expand(gt, obj, ovl, torch.from_numpy(Pn).to(DEV), want=('cls', 'neg'))
    tot = 0
    for b in range(B):
        o, v, c, n = M.match_criterion(boxes[b].numpy(), labels[b].numpy(), pxy)
        np.testing.assert_array_equal(obj[b].cpu().numpy(), o)
        np.testing.assert_array_equal(ovl[b].cpu().numpy(), v)
        np.testing.assert_array_equal(cls[b].cpu().numpy(), c)
        np.testing.assert_array_equal(neg[b].cpu().numpy(), n)
        tot += int((c > 0).sum())
    assert int(npos[B]) == tot


def _criterion(arch, B, reg, cls, seed):
    P = torch.from_numpy(prior_table(arch))
    C = 21
    boxes, labels = synth.make_gt(B, seed=seed)
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=seed)
    cfg = Cfg(reg_weights=1.0, device=DEV, n_classes=C, reg_loss=reg, cls_loss=cls)
    crit = CR.RetinaFocalLoss(priors_cxcy=P.to(DEV), config=cfg)
    lo = locs.to(DEV).requires_grad_(True)
    sc = scores.to(DEV).requires_grad_(True)
    loss = crit(lo, sc, [b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    loss.backward()
    rl, rs = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    ref = LR.criterion('retina', P, rl, rs, boxes, labels, reg, cls)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-4)
    np.testing.assert_allclose(lo.grad.cpu().numpy(), rl.grad.numpy(), rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(sc.grad.cpu().numpy(), rs.grad.numpy(), rtol=1e-4, atol=1e-8)


@pytest.mark.parametrize('reg,cls', [('diou', 'focal'), ('smoothl1', 'ce')])
def test_retina_criterion_stress_100k_anchors(reg, cls):
    _criterion('RETINA896', 2, reg, cls, seed=21)


def test_retina_criterion_config_c3_full_batch():
    _criterion('RETINA', 32, 'diou', 'focal', seed=22)


def test_detect_stress_100k_anchors():
    Pn = prior_table('RETINA896')
    P = torch.from_numpy(Pn).to(DEV)
    locs, scores = synth.make_preds(2, Pn.shape[0], 21, seed=31, bg_shift=7.0)
    (ob, ol, os_), probs, boxes = core.detect(locs.to(DEV), scores.to(DEV), 0.01, 0.45, 200, P,
                                              debug=True)
    rb, rl, rs = M.detect(probs.cpu().numpy(), boxes.cpu().numpy(), 0.01, 0.45, 200, nms_variant='tv')
    for b in range(2):
        assert ob[b].shape[0] == 200
        np.testing.assert_array_equal(ol[b].cpu().numpy(), rl[b])
        np.testing.assert_array_equal(os_[b].cpu().numpy(), rs[b])
        np.testing.assert_array_equal(ob[b].cpu().numpy(), rb[b])
