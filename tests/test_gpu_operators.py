"""The operators.* / metrics / transforms API on the HIP path vs the reference's golden vectors."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import match_ref as M
from shape_based_object_detection_amd import metrics
from shape_based_object_detection_amd import synth
from shape_based_object_detection_amd.dataset import transforms as T
from shape_based_object_detection_amd.models.priors import prior_table
from shape_based_object_detection_amd.operators import Loss as LS
from shape_based_object_detection_amd.operators import iou_utils as IU

pytestmark = pytest.mark.gpu
DEV = 'cuda'
RTOL = 1e-4


def t(x):
    return torch.from_numpy(np.asarray(x)).to(DEV)


def test_overlaps_and_iou_losses():
    d = load_golden('losses.npz')
    p, tt = t(d['box_p']), t(d['box_t'])
    for name in ['iou', 'giou', 'diou', 'ciou']:
        pp = p.clone().requires_grad_(True)
        o = getattr(IU, 'bbox_overlaps_' + name)(pp, tt)
        o.sum().backward()
        np.testing.assert_allclose(o.detach().cpu().numpy(), d['ov_' + name], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(pp.grad.cpu().numpy(), d['ov_%s_grad' % name], rtol=1e-4, atol=1e-5)
    w = None
    for lt in ['Iou', 'Giou', 'Diou', 'Ciou']:
        for red in ['mean', 'sum']:
            pp = p.clone().requires_grad_(True)
            loss = LS.IouLoss(pred_mode='Corner', reduce=red, losstype=lt)(pp, tt)
            loss.backward()
            np.testing.assert_allclose(loss.item(), d['iouloss_%s_%s' % (lt, red)], rtol=RTOL)
            np.testing.assert_allclose(pp.grad.cpu().numpy(), d['iouloss_%s_%s_grad' % (lt, red)],
                                       rtol=1e-4, atol=1e-6)
    loc = t(d['center_loc']).requires_grad_(True)
    loss = LS.IouLoss(pred_mode='Center', variances=[0.1, 0.2], losstype='Diou')(loc, tt, prior_data=t(d['center_priors']))
    loss.backward()
    np.testing.assert_allclose(loss.item(), d['iouloss_center'], rtol=RTOL)
    np.testing.assert_allclose(loc.grad.cpu().numpy(), d['iouloss_center_grad'], rtol=1e-4, atol=1e-6)
    empty = IU.bbox_overlaps_diou(torch.zeros(0, 4, device=DEV), torch.zeros(0, 4, device=DEV))
    assert tuple(empty.shape) == (0, 0)


def test_smooth_l1_and_focals():
    d = load_golden('losses.npz')
    a, b = t(d['sl1_a']), t(d['sl1_b'])
    for red in ['mean', 'sum']:
        aa = a.clone().requires_grad_(True)
        loss = LS.SmoothL1Loss(reduction=red)(aa, b)
        loss.backward()
        np.testing.assert_allclose(loss.item(), d['sl1_' + red], rtol=RTOL)
        np.testing.assert_allclose(aa.grad.cpu().numpy(), d['sl1_%s_grad' % red], rtol=1e-5, atol=1e-7)
    aa = a.clone().requires_grad_(True)
    loss = LS.SmoothL1Loss()(aa, b, weights=t(d['sl1_w'])[:, None])
    loss.backward()
    np.testing.assert_allclose(loss.item(), d['sl1_w_loss'], rtol=RTOL)
    np.testing.assert_allclose(aa.grad.cpu().numpy(), d['sl1_w_grad'], rtol=1e-5, atol=1e-7)
    # gradient w.r.t. the target as well (autograd reaches both inputs in the reference): the
    # loss depends on (pred - target) only, so d/dtarget is exactly -d/dpred
    aa, bb = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    LS.SmoothL1Loss()(aa, bb).backward()
    np.testing.assert_allclose(aa.grad.cpu().numpy(), d['sl1_mean_grad'], rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(bb.grad.cpu().numpy(), -aa.grad.cpu().numpy())
    x, y = t(d['logits']), t(d['y'])

    class C:
        device = DEV
    cases = [('focal', lambda z: LS.focal_loss(z, y, device=DEV)),
             ('focal_b', lambda z: LS.focal_loss(z, y, alpha=[0.3, 0.6], gamma=1.5, device=DEV)),
             ('sfocal', lambda z: LS.SigmoidFocalLoss(2.0, 0.25, C())(z, y)),
             ('bfocal', lambda z: LS.FocalLoss()(z, y))]
    for key, fn in cases:
        z = x.clone().requires_grad_(True)
        loss = fn(z)
        loss.backward()
        np.testing.assert_allclose(loss.item(), d[key], rtol=RTOL, err_msg=key)
        np.testing.assert_allclose(z.grad.cpu().numpy(), d[key + '_grad'], rtol=1e-4, atol=1e-6, err_msg=key)


def test_metrics_and_jaccard():
    d = load_golden('jaccard.npz')
    for k in range(int(d['n_cases'])):
        gt, an = t(d['c%d_gt' % k]), t(d['c%d_anchors' % k])
        np.testing.assert_array_equal(metrics.find_jaccard_overlap(gt, an).cpu().numpy(), d['c%d_metrics' % k])
        np.testing.assert_array_equal(IU.jaccard(gt, an).cpu().numpy(), d['c%d_plain' % k])
        inter = metrics.intersect(gt, an).cpu().numpy()
        g, a = d['c%d_gt' % k][:, None], d['c%d_anchors' % k][None]
        ref = (np.maximum(np.minimum(g[..., 2], a[..., 2]) - np.maximum(g[..., 0], a[..., 0]), np.float32(0)) *
               np.maximum(np.minimum(g[..., 3], a[..., 3]) - np.maximum(g[..., 1], a[..., 1]), np.float32(0)))
        np.testing.assert_array_equal(inter, ref)


def test_codecs_and_match_api():
    d = load_golden('codecs.npz')
    p, bx, lc = t(d['priors']), t(d['boxes']), t(d['locs'])
    np.testing.assert_array_equal(T.xy_to_cxcy(bx).cpu().numpy(), d['xy_to_cxcy'])
    np.testing.assert_array_equal(T.cxcy_to_xy(p).cpu().numpy(), d['cxcy_to_xy'])
    np.testing.assert_array_equal(IU.point_form(p).cpu().numpy(), d['point_form'])
    np.testing.assert_allclose(T.cxcy_to_gcxgcy(T.xy_to_cxcy(bx), p).cpu().numpy(), d['cxcy_to_gcxgcy'], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(T.gcxgcy_to_cxcy(lc, p).cpu().numpy(), d['gcxgcy_to_cxcy'], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(IU.encode(bx, p, [0.1, 0.2]).cpu().numpy(), d['encode'], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(IU.decode(lc, p, [0.1, 0.2]).cpu().numpy(), d['decode'], rtol=1e-6, atol=1e-7)
    with pytest.raises(TypeError):
        IU.center_size(p)
    m = load_golden('match_iou_utils.npz')
    P = t(prior_table('SSD300'))
    loc_t = torch.zeros(2, P.shape[0], 4, device=DEV)
    conf_t = torch.zeros(2, P.shape[0], dtype=torch.long, device=DEV)
    for i in range(2):
        IU.match(0.5, t(m['b%d_boxes' % i]), P, [0.1, 0.2], t(m['b%d_labels' % i]), loc_t, conf_t, i)
    np.testing.assert_array_equal(conf_t.cpu().numpy(), m['match_conf'])
    np.testing.assert_allclose(loc_t.cpu().numpy(), m['match_loc'], rtol=1e-5, atol=1e-5)


def test_cpu_and_device_paths_agree():
    """CPU tensors take the host path (DataLoader workers); device tensors the HIP
    kernel: bit-identical IoU.  Mixed devices raise; the C-ABI wrappers reject CPU tensors."""
    from shape_based_object_detection_amd import _lib as L
    from shape_based_object_detection_amd.operators import iou_utils as IU
    g = torch.rand(7, 2)
    gt = torch.cat([g, g + torch.rand(7, 2) * 0.5], 1)
    a = torch.rand(300, 2)
    an = torch.cat([a, a + torch.rand(300, 2) * 0.3], 1)
    an[5, 2:] = an[5, :2]                        # a zero-size anchor (-1 mask)
    host = metrics.find_jaccard_overlap(gt, an)
    dev = metrics.find_jaccard_overlap(gt.cuda(), an.cuda()).cpu()
    assert torch.equal(host, dev)
    assert torch.equal(IU.jaccard(gt, an), IU.jaccard(gt.cuda(), an.cuda()).cpu())
    with pytest.raises(RuntimeError):
        metrics.find_jaccard_overlap(gt, an.cuda())
    from shape_based_object_detection_amd import core
    with pytest.raises(L.SbodError):
        core.nms(torch.rand(4, 4), torch.rand(4), 0.5)


@pytest.mark.parametrize('kind', ['iou', 'giou', 'diou', 'ciou'])
def test_overlap_gradients_both_box_sets(kind):
    """Autograd reaches BOTH box sets in the reference (iou_utils.py:6-164): d/d bboxes2 vs the
    oracle's torch-fp32 restatement of the same graph (with ties and the clamp masks)."""
    from oracle import loss_ref as LR
    d = load_golden('losses.npz')
    p, q = torch.from_numpy(d['box_p']), torch.from_numpy(d['box_t'])
    q = q.clone()
    q[-3:, 0] = p[-3:, 0]                                 # exact min / max ties on x1 and y2
    q[-3:, 3] = p[-3:, 3]
    a, b = p.to(DEV).requires_grad_(True), q.to(DEV).requires_grad_(True)
    o = getattr(IU, 'bbox_overlaps_' + kind)(a, b)
    (o * torch.linspace(0.5, 1.5, o.numel(), device=DEV)).sum().backward()
    ra, rb = p.clone().requires_grad_(True), q.clone().requires_grad_(True)
    ro = LR.aligned_overlap(kind, ra, rb)
    (ro * torch.linspace(0.5, 1.5, ro.numel())).sum().backward()
    np.testing.assert_allclose(o.detach().cpu().numpy(), ro.detach().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(a.grad.cpu().numpy(), ra.grad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(b.grad.cpu().numpy(), rb.grad.numpy(), rtol=1e-4, atol=1e-5)
    # the reference exchanges the sets when rows > cols (and transposes back): a [1,4] x [n,4]
    # call broadcasts the single box, whose gradient is the sum over the rows
    one = p[:1].to(DEV).requires_grad_(True)
    bb = q.to(DEV).requires_grad_(True)
    getattr(IU, 'bbox_overlaps_' + kind)(bb, one).sum().backward()
    r1, rbb = p[:1].clone().requires_grad_(True), q.clone().requires_grad_(True)
    LR.aligned_overlap(kind, r1.expand_as(rbb), rbb).sum().backward()
    np.testing.assert_allclose(one.grad.cpu().numpy(), r1.grad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(bb.grad.cpu().numpy(), rbb.grad.numpy(), rtol=1e-4, atol=1e-5)
