"""The one-launch focal criterion (sbod_criterion_focal: matcher + forced match + normaliser +
fused loss pass in one launch, k_multibox<..., true>) against the same call as two launches
(k_match_tile + k_match_final, then k_multibox) and against the oracle.

The one-launch form lost its A/B and its workgroups wait for each other, so it
is built into a VARIANT library only (EXTRA=-DSBOD_VARIANT_ONE_LAUNCH bash
scripts/build_lib_variant.sh onelaunch; run this file with SBOD_LIB pointing at it).  With the
product library these tests skip; tests/test_cpu_host.py checks the product library has none of it.

The two forms run the same per-prior arithmetic and exact fixed-point finishes of the same
per-workgroup partials, so the matcher outputs, the positive counts, the loss vector and every
gradient must be bit-identical; the oracle comparison is the north_star's 1e-4 relative."""
import numpy as np
import pytest
import torch

from oracle import loss_ref as LR
from shape_based_object_detection_amd import _lib as L
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table


def _variant_built():
    try:
        return bool(L.lib().sbod_build_variants() & L.VARIANT_ONE_LAUNCH_CRITERION)
    except L.SbodError:
        return False


pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not _variant_built(), reason='one-launch criterion: variant library only '
                                                              '(SBOD_LIB=.../libsbod_hip_onelaunch.so)')]
DEV = 'cuda'


class Cfg(dict):
    __getattr__ = dict.__getitem__


CLASSES = {'ssd512': CR.MultiBoxLoss512, 'ssd300': CR.MultiBoxLoss300, 'retina': CR.RetinaFocalLoss}


def _both(kind, arch, B, reg, seed, max_objects=16, dtype=torch.float32, C=21):
    P = torch.from_numpy(prior_table(arch))
    boxes, labels = synth.make_gt(B, seed=seed, max_objects=max_objects, n_classes=C)
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=seed)
    crit = CLASSES[kind](priors_cxcy=P.to(DEV), config=Cfg(reg_weights=1.0, device=DEV, n_classes=C, reg_loss=reg,
                                                           cls_loss='focal'))
    spec = crit._spec()
    gt = core.pack_gt([b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    res = []
    for two in (False, True):
        lo = locs.to(DEV, dtype).requires_grad_(True)
        sc = scores.to(DEV, dtype).requires_grad_(True)
        loss, comps, (obj, ovl, npos) = core.criterion_focal(lo, sc, gt, crit.priors_cxcy, crit.priors_xy, spec,
                                                             crit.threshold, crit.threshold - 0.1, two_launch=two)
        loss.backward()
        res.append(dict(loss=loss.item(), comps=comps.cpu().numpy(), obj=obj.cpu().numpy(), ovl=ovl.cpu().numpy(),
                        npos=npos.cpu().numpy(), gl=lo.grad.float().cpu().numpy(), gs=sc.grad.float().cpu().numpy()))
    assert core.criterion_status(DEV) == 0
    one, two = res
    for k in ('obj', 'ovl', 'npos', 'comps', 'gl', 'gs'):
        np.testing.assert_array_equal(one[k], two[k], err_msg=k)
    assert one['loss'] == two['loss']
    return P, boxes, labels, locs, scores, one


@pytest.mark.parametrize('kind,arch,B,reg', [('ssd512', 'SSD512', 32, 'diou'), ('ssd512', 'SSD512', 3, 'smoothl1'),
                                             ('ssd300', 'SSD300', 8, 'diou'), ('ssd300', 'SSD300', 4, 'l1'),
                                             ('retina', 'RETINA', 8, 'diou')])
def test_one_launch_equals_two_launches_and_oracle(kind, arch, B, reg):
    P, boxes, labels, locs, scores, one = _both(kind, arch, B, reg, seed=B + 17)
    lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    ref = LR.criterion(kind, P, lo, sc, boxes, labels, reg, 'focal')
    ref.backward()
    np.testing.assert_allclose(one['loss'], ref.item(), rtol=1e-4)
    np.testing.assert_allclose(one['gl'], lo.grad.numpy(), rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(one['gs'], sc.grad.numpy(), rtol=1e-4, atol=1e-8)


def test_one_launch_many_objects_lds_forced_match():
    """Up to 150 objects: the forced match's LDS form (Gmax > 64) inside the launch."""
    _both('ssd512', 'SSD512', 4, 'diou', seed=9, max_objects=150)


def test_one_launch_single_object_images_and_bf16():
    _both('ssd512', 'SSD512', 16, 'diou', seed=3, max_objects=1)
    _both('ssd512', 'SSD512', 16, 'diou', seed=4, dtype=torch.bfloat16)


def test_one_launch_forced_collisions():
    """Objects that share their best prior (last writer wins with the FILTERED j) and objects with
    no positive overlap (never forced): the image's forced list, applied in other workgroups."""
    P = torch.from_numpy(prior_table('SSD512'))
    pri = P.to(DEV)
    cfg = Cfg(reg_weights=1.0, device=DEV, n_classes=21, reg_loss='diou', cls_loss='focal')
    crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
    c = torch.tensor([0.31, 0.47])
    tiny = torch.cat([torch.tile(c - 1e-3, (4, 1)), torch.tile(c + 1e-3, (4, 1))], 1)   # 4 identical boxes
    far = torch.tensor([[1.5, 1.5, 1.6, 1.6]])                                           # outside every prior
    boxes = [torch.cat([tiny, far, tiny[:1] + 0.2]), torch.cat([far, tiny[:2]])]
    labels = [torch.tensor([3, 5, 7, 9, 11, 2]), torch.tensor([4, 6, 8])]
    locs, scores = synth.make_preds(2, P.shape[0], 21, seed=5)
    gt = core.pack_gt([b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    spec = crit._spec()
    outs = []
    for two in (False, True):
        lo = locs.to(DEV).requires_grad_(True)
        sc = scores.to(DEV).requires_grad_(True)
        loss, comps, (obj, ovl, npos) = core.criterion_focal(lo, sc, gt, crit.priors_cxcy, crit.priors_xy, spec,
                                                             crit.threshold, crit.threshold - 0.1, two_launch=two)
        loss.backward()
        outs.append((obj.cpu(), ovl.cpu(), npos.cpu(), comps.cpu(), sc.grad.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    ref = LR.criterion('ssd512', P, lo, sc, boxes, labels, 'diou', 'focal')
    ref.backward()
    np.testing.assert_allclose(float(outs[0][3][0]), ref.item(), rtol=1e-4)


def test_criterion_class_uses_one_launch_and_captures():
    """MultiBoxLoss512(focal) with ``one_launch`` set takes the one-launch form; replayed from a
    hipGraph (nothing else running beside it) it gives the eager results."""
    P = torch.from_numpy(prior_table('SSD512')).to(DEV)
    B = 8
    boxes, labels = synth.make_gt(B, seed=77)
    locs, scores = synth.make_preds(B, P.shape[0], 21, seed=77)
    crit = CR.MultiBoxLoss512(priors_cxcy=P, config=Cfg(reg_weights=1.0, device=DEV, n_classes=21, reg_loss='diou',
                                                        cls_loss='focal'))
    crit.one_launch = True   # opt-in (the default is the matcher and loss launches)
    bx, lb = [b.to(DEV) for b in boxes], [l.to(DEV) for l in labels]
    stage = core.GtStaging(B, 16, DEV)
    lo = locs.to(DEV).requires_grad_(True)
    sc = scores.to(DEV).requires_grad_(True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            lo.grad = sc.grad = None
            eager = crit(lo, sc, stage.stage(bx, lb), None)
            eager.backward(core.unit_grad(DEV))
        e_loss, e_gl, e_gs = eager.item(), lo.grad.clone(), sc.grad.clone()
        lo.grad = sc.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            loss = crit(lo, sc, stage.stage(bx, lb), None)
            loss.backward(core.unit_grad(DEV))
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        assert core.criterion_status(DEV) == 0   # (the capture stream's workspace)
    assert loss.item() == e_loss
    assert torch.equal(lo.grad, e_gl) and torch.equal(sc.grad, e_gs)


def test_timed_out_wait_poisons_gradients_and_next_call_is_clean():
    """a one-launch call whose in-launch wait gives up (the grid not co-resident: a
    long kernel of another stream holds the CUs) returns a NaN loss AND NaN gradients in the
    workgroups that gave up, and the timeout word is cleared by that call's finish — the next
    call on the same workspace (alone on the device) is finite and equals the two-launch form.
    Whether the first call times out depends on the other stream's timing; the sticky diagnostics
    word (sbod_criterion_status) says whether it did."""
    P = torch.from_numpy(prior_table('SSD512')).to(DEV)
    B = 32
    boxes, labels = synth.make_gt(B, seed=5)
    locs, scores = synth.make_preds(B, P.shape[0], 21, seed=5)
    crit = CR.MultiBoxLoss512(priors_cxcy=P, config=Cfg(reg_weights=1.0, device=DEV, n_classes=21, reg_loss='diou',
                                                        cls_loss='focal'))
    spec = crit._spec()
    gt = core.pack_gt([b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    hog_a = torch.randn(8192, 8192, device=DEV)
    other = torch.cuda.Stream()
    outs = []
    for k in range(2):
        lo = locs.to(DEV).requires_grad_(True)
        sc = scores.to(DEV).requires_grad_(True)
        if k == 0:   # a long GEMM on another stream first: the launch may not get every CU
            with torch.cuda.stream(other):
                for _ in range(4):
                    hog_a = hog_a @ hog_a
                    hog_a = hog_a / hog_a.abs().max()
        loss, comps, _ = core.criterion_focal(lo, sc, gt, crit.priors_cxcy, crit.priors_xy, spec, crit.threshold,
                                              crit.threshold - 0.1, two_launch=False)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.item(), sc.grad.clone(), core.criterion_status(DEV)))
    first_loss, first_gs, first_status = outs[0]
    if first_status != 0:
        assert first_loss != first_loss and bool(torch.isnan(first_gs).any())
    lo = locs.to(DEV).requires_grad_(True)
    sc = scores.to(DEV).requires_grad_(True)
    ref, _, _ = core.criterion_focal(lo, sc, gt, crit.priors_cxcy, crit.priors_xy, spec, crit.threshold,
                                     crit.threshold - 0.1, two_launch=True)
    ref.backward()
    assert outs[1][0] == ref.item()
    assert torch.equal(outs[1][1], sc.grad)
