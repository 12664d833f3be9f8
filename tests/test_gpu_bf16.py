"""Config C2 (SSD512 batch=16 bf16) and config C4's criterion at full size, against the oracle.

bf16 semantics of the HIP path: bf16 locs/scores are read as bf16 and computed in fp32 (the
exact upcast), gradients are rounded to bf16 once at the store.  The reference never runs bf16
(no autocast / half anywhere), so parity is defined on the same bf16-rounded inputs
upcast to fp32 and run through the oracle:
  * loss within 1e-4 relative (north_star's fp32 loss tolerance);
  * every gradient element within ONE bf16 ulp of the oracle's fp32 gradient (one rounding of a
    value that agrees with the oracle to ~1e-6 relative can land on either neighbour);
  * detect on bf16 inputs bit-exact vs the oracle's NMS on the activations the kernel produced.
"""
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


def bf16_ulp(x):
    """One bf16 ulp at |x| (8 significant bits); normal-range floor for |x| ~ 0."""
    a = np.maximum(np.abs(x.astype(np.float64)), 2.0 ** -126)
    return 2.0 ** (np.floor(np.log2(a)) - 7)


def assert_within_one_bf16_ulp(got_bf16, ref_f32, what):
    """|got - ref| <= one bf16 ulp of ref, with an absolute floor of 2^-20 x max|ref|: elements
    that are tiny through cancellation (a DIoU gradient near 0) carry fp32 rounding of the
    O(max) terms they cancel, in the oracle as much as here."""
    got = got_bf16.float().cpu().numpy().astype(np.float64)
    ref = ref_f32.astype(np.float64)
    err = np.abs(got - ref)
    tol = np.maximum(bf16_ulp(ref), 2.0 ** -20 * np.abs(ref).max())
    bad = err > tol
    assert not bad.any(), '%s: %d of %d elements beyond one bf16 ulp (worst %g at ref %g)' % (
        what, int(bad.sum()), bad.size, float(err[bad].max()), float(ref[bad][np.argmax(err[bad])]))


@pytest.mark.parametrize('reg,cls', [('diou', 'focal'), ('smoothl1', 'ce')])
def test_c2_ssd512_b16_bf16_criterion_vs_oracle(reg, cls):
    P = torch.from_numpy(prior_table('SSD512'))
    B, C = 16, 21
    boxes, labels = synth.make_gt(B, seed=216)
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=216)
    lo16, sc16 = locs.bfloat16(), scores.bfloat16()
    crit = CR.MultiBoxLoss512(priors_cxcy=P.to(DEV), config=Cfg(reg_weights=1.0, device=DEV, n_classes=C,
                                                                  reg_loss=reg, cls_loss=cls))
    lo = lo16.to(DEV).requires_grad_(True)
    sc = sc16.to(DEV).requires_grad_(True)
    loss = crit(lo, sc, [b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    loss.backward()
    assert lo.grad.dtype == torch.bfloat16 and sc.grad.dtype == torch.bfloat16
    rl = lo16.float().requires_grad_(True)
    rs = sc16.float().requires_grad_(True)
    ref = LR.criterion('ssd512', P, rl, rs, boxes, labels, reg, cls)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-4)
    assert_within_one_bf16_ulp(lo.grad, rl.grad.numpy(), 'grad_locs')
    assert_within_one_bf16_ulp(sc.grad, rs.grad.numpy(), 'grad_scores')


def test_c2_detect_bf16_bit_exact_on_shared_activations():
    P = torch.from_numpy(prior_table('SSD512'))
    B, C = 16, 21
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=217, bg_shift=6.0)
    lo16, sc16 = locs.bfloat16().to(DEV), scores.bfloat16().to(DEV)
    (ob, ol, os_), probs, bxs = core.detect(lo16, sc16, 0.01, 0.45, 200, P.to(DEV), debug=True)
    # the activations are those of the bf16 values (exact upcast): softmax within ~1e-6 of torch
    ref_p = torch.softmax(sc16.float().cpu(), 2).numpy()
    np.testing.assert_allclose(probs.cpu().numpy(), ref_p, rtol=1e-5, atol=1e-7)
    rb, rl, rs = M.detect(probs.cpu().numpy(), bxs.cpu().numpy(), 0.01, 0.45, 200)
    for b in range(B):
        np.testing.assert_array_equal(ol[b].cpu().numpy(), rl[b])
        np.testing.assert_array_equal(os_[b].cpu().numpy(), rs[b])
        np.testing.assert_array_equal(ob[b].cpu().numpy(), rb[b])


def test_c4_refinedet_full_size_vs_oracle():
    """RefineDetLoss at config C4's size: P = 16,320 priors, B = 16, VOC classes."""
    P = torch.from_numpy(prior_table('REFINEDET'))
    B, C = 16, 21
    n = P.shape[0]
    boxes, labels = synth.make_gt(B, seed=416)
    arm_l, arm_s = synth.make_preds(B, n, 2, seed=416)
    odm_l, odm_s = synth.make_preds(B, n, C, seed=417)
    crit = CR.RefineDetLoss(priors_cxcy=P.to(DEV), config=Cfg(reg_weights=1.0, device=DEV, n_classes=C))
    ts = [t.to(DEV).requires_grad_(True) for t in (arm_l, arm_s, odm_l, odm_s)]
    loss = crit(*ts, [b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    loss.backward()
    rs = [t.clone().requires_grad_(True) for t in (arm_l, arm_s, odm_l, odm_s)]
    ref = LR.refinedet(P, *rs, boxes, labels)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-4)
    for name, t, r in zip(('arm_locs', 'arm_scores', 'odm_locs', 'odm_scores'), ts, rs):
        np.testing.assert_allclose(t.grad.cpu().numpy(), r.grad.numpy(), rtol=1e-4, atol=1e-8,
                                   err_msg=name)


@pytest.mark.parametrize('box_type', ['offset', 'corner'])
def test_c2_detect_native_bf16_equals_widened_fp32(box_type):
    """bf16 locs/scores go to the kernels as they are (SBOD_DETECT_INPUT_BF16, widened exactly on
    load): boxes, labels and scores are bit-identical to detect on the fp32-widened tensors, and
    the corner form's in-place clamp (models/utils.py:224) lands in the caller's bf16 tensor."""
    P = torch.from_numpy(prior_table('SSD512'))
    B, C = 16, 21
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=218, bg_shift=6.0)
    if box_type == 'corner':
        locs = locs * 5 + 0.5                  # xyxy-ish values, many outside [0, 1]
    lo16, sc16 = locs.bfloat16().to(DEV), scores.bfloat16().to(DEV)
    lo32 = lo16.float()
    nat = core.detect(lo16, sc16, 0.01, 0.45, 200, P.to(DEV), box_type=box_type)
    wid = core.detect(lo32, sc16.float(), 0.01, 0.45, 200, P.to(DEV), box_type=box_type)
    for x, y in zip(nat, wid):
        for b in range(B):
            assert torch.equal(x[b], y[b])
    if box_type == 'corner':
        assert lo16.dtype == torch.bfloat16
        assert torch.equal(lo16.float(), lo32)      # both clamped in place, identically
        assert float(lo16.min()) >= 0.0 and float(lo16.max()) <= 1.0
