"""The drop-in modules on CPU tensors (the reference's ``device = 'cpu'``, train_anchor.py:65-71):
criteria, loss operators, NMS / detect, DeformConv2d and calculate_mAP through the host path
(``hostpath.py``), pinned to the golden vectors the reference itself produced
(tests/golden/make_golden.py).  Config C1 — one SSD300 step on 4 VOC-format images on the CPU —
runs here as stated.  Tolerances are the north_star's: losses 1e-4 relative, gradients 1e-4
relative (+ a small absolute floor), indices / labels / counts exact."""
import hashlib

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader

from conftest import load_golden
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.dataset import Datasets as D
from shape_based_object_detection_amd.detect_scripts import detect_tools as DT
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models import utils as MU
from shape_based_object_detection_amd.models.priors import prior_table
from shape_based_object_detection_amd.operators import Loss as LS
from shape_based_object_detection_amd.operators import iou_utils as IU
from shape_based_object_detection_amd.operators.Deformable_convolution import DeformConv2d

RTOL = 1e-4


class Cfg(dict):
    __getattr__ = dict.__getitem__


CLASSES = {'ssd512': CR.MultiBoxLoss512, 'ssd300': CR.MultiBoxLoss300, 'retina': CR.RetinaFocalLoss}
NAMES = ['ssd512_sl1_ce', 'ssd512_diou_focal', 'ssd300_l1_ce', 'ssd300_diou_focal',
         'retina_diou_focal', 'retina_sl1_ce', 'ssd512full_diou_focal', 'ssd512full_sl1_ce']


def test_metrics_import_surface():
    """train_anchor.py:21 / eval.py:23 import these names from the metrics module."""
    from shape_based_object_detection_amd.metrics import AverageMeter, accuracy, calculate_mAP  # noqa: F401
    m = AverageMeter()
    for v, n in ((2.0, 1), (4.0, 3)):
        m.update(v, n)
    assert (m.val, m.sum, m.count, m.avg) == (4.0, 14.0, 4, 3.5)
    m.reset()
    assert (m.val, m.sum, m.count, m.avg) == (0, 0, 0, 0)
    scores = torch.tensor([[0.1, 0.7, 0.2], [0.5, 0.1, 0.4], [0.2, 0.3, 0.5], [0.6, 0.3, 0.1]])
    targets = torch.tensor([1, 2, 0, 0])
    assert accuracy(scores, targets, 1) == 50.0
    assert accuracy(scores, targets, 2) == 75.0


@pytest.mark.parametrize('name', NAMES)
def test_criteria_golden_on_cpu(name):
    d = load_golden('crit_%s.npz' % name)
    kind = name.split('_')[0].replace('full', '')
    reg, cls = name.split('_')[1:]
    P = torch.from_numpy(prior_table(str(d['arch']))[::int(d['prior_stride'])].copy())
    B, C = int(d['batch']), int(d['n_classes'])
    boxes = [torch.from_numpy(d['b%d_boxes' % i]) for i in range(B)]
    labels = [torch.from_numpy(d['b%d_labels' % i]) for i in range(B)]
    if 'locs' in d.files:
        locs, scores = torch.from_numpy(d['locs']), torch.from_numpy(d['scores'])
    else:
        locs, scores = synth.make_preds(B, P.shape[0], C, seed=61)
        assert hashlib.sha256(locs.numpy().tobytes()).hexdigest() == str(d['locs_sha'])
    crit = CLASSES[kind](priors_cxcy=P, config=Cfg(reg_weights=1.0, device='cpu', n_classes=C, reg_loss=reg,
                                                   cls_loss=cls))
    lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    loss = crit(lo, sc, boxes, labels)
    loss.backward()
    np.testing.assert_allclose(loss.item(), d['loss'], rtol=RTOL)
    gl, gs = lo.grad.numpy(), sc.grad.numpy()
    if 'grad_locs' in d.files:
        np.testing.assert_allclose(gl, d['grad_locs'], rtol=1e-4, atol=1e-7)
        np.testing.assert_allclose(gs, d['grad_scores'], rtol=1e-4, atol=1e-7)
    else:
        np.testing.assert_allclose(gl.reshape(-1, 4)[d['grad_locs_rows']], d['grad_locs_at_rows'], rtol=1e-4, atol=1e-8)
        np.testing.assert_allclose(gs.reshape(-1, C)[d['grad_scores_rows']], d['grad_scores_at_rows'],
                                   rtol=1e-4, atol=1e-8)


def test_refinedet_golden_on_cpu():
    d = load_golden('crit_refinedet.npz')
    P = torch.from_numpy(prior_table('REFINEDET')[::int(d['prior_stride'])].copy())
    boxes = [torch.from_numpy(d['b%d_boxes' % i]) for i in range(3)]
    labels = [torch.from_numpy(d['b%d_labels' % i]) for i in range(3)]
    ts = [torch.from_numpy(d[n]).requires_grad_(True) for n in ['arm_locs', 'arm_scores', 'odm_locs', 'odm_scores']]
    crit = CR.RefineDetLoss(priors_cxcy=P, config=Cfg(reg_weights=1.0, device='cpu', n_classes=6))
    loss = crit(*ts, boxes, labels)
    loss.backward()
    np.testing.assert_allclose(loss.item(), d['loss'], rtol=RTOL)
    for n, t in zip(['arm_locs', 'arm_scores', 'odm_locs', 'odm_scores'], ts):
        np.testing.assert_allclose(t.grad.numpy(), d[n + '_grad'], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize('reg,cls', [('smoothl1', 'ce'), ('diou', 'focal')])
def test_c1_ssd300_voc_step_on_cpu(tmp_path, reg, cls):
    """BASELINE config C1 as stated: 4 synthetic VOC-format 300x300 images through the reference's
    data path (JSON -> PascalVOCDataset -> DataLoader/collate_fn), one MultiBoxLoss300 step on the
    CPU.  The same batch on the golden-pinned host path twice gives identical results, and its
    loss is finite with gradients on every positive / mined row."""
    folder = D.write_synthetic_voc(str(tmp_path), 4, size=(300, 300), split='TRAIN', seed=11)
    ds = D.PascalVOCDataset(folder, 'train', (300, 300),
                            {'model': {'operation_list': ['expand', 'random_crop'], 'return_percent_coords': True}})
    torch.manual_seed(1)
    images, boxes, labels, _, _ = next(iter(DataLoader(ds, batch_size=4, shuffle=False, collate_fn=ds.collate_fn)))
    assert images.shape == (4, 3, 300, 300) and not images.is_cuda
    P = torch.from_numpy(prior_table('SSD300'))
    locs, scores = synth.make_preds(4, P.shape[0], 21, seed=11)
    crit = CR.MultiBoxLoss300(priors_cxcy=P, config={'reg_weights': 1.0, 'device': 'cpu', 'n_classes': 21,
                                                     'reg_loss': reg, 'cls_loss': cls})
    out = []
    for _ in range(2):
        lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
        loss = crit(lo, sc, boxes, labels)
        loss.backward()
        out.append((loss.item(), lo.grad, sc.grad))
    assert np.isfinite(out[0][0]) and out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])
    assert int((out[0][1].abs().sum(2) > 0).sum()) > 0


def test_loss_operators_golden_on_cpu():
    d = load_golden('losses.npz')
    p, tt = torch.from_numpy(d['box_p']), torch.from_numpy(d['box_t'])
    for name in ['iou', 'giou', 'diou', 'ciou']:
        pp = p.clone().requires_grad_(True)
        o = getattr(IU, 'bbox_overlaps_' + name)(pp, tt)
        o.sum().backward()
        np.testing.assert_allclose(o.detach().numpy(), d['ov_' + name], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(pp.grad.numpy(), d['ov_%s_grad' % name], rtol=1e-5, atol=1e-6)
    for lt in ['Iou', 'Giou', 'Diou', 'Ciou']:
        for red in ['mean', 'sum']:
            pp = p.clone().requires_grad_(True)
            loss = LS.IouLoss(pred_mode='Corner', reduce=red, losstype=lt)(pp, tt)
            loss.backward()
            np.testing.assert_allclose(loss.item(), d['iouloss_%s_%s' % (lt, red)], rtol=RTOL)
            np.testing.assert_allclose(pp.grad.numpy(), d['iouloss_%s_%s_grad' % (lt, red)], rtol=1e-4, atol=1e-6)
    a, b = torch.from_numpy(d['sl1_a']), torch.from_numpy(d['sl1_b'])
    for red in ['mean', 'sum']:
        aa = a.clone().requires_grad_(True)
        loss = LS.SmoothL1Loss(reduction=red)(aa, b)
        loss.backward()
        np.testing.assert_allclose(loss.item(), d['sl1_' + red], rtol=RTOL)
        np.testing.assert_allclose(aa.grad.numpy(), d['sl1_%s_grad' % red], rtol=1e-5, atol=1e-7)
    x, y = torch.from_numpy(d['logits']), torch.from_numpy(d['y'])

    class C:
        device = 'cpu'
    cases = [('focal', lambda z: LS.focal_loss(z, y, device='cpu')),
             ('focal_b', lambda z: LS.focal_loss(z, y, alpha=[0.3, 0.6], gamma=1.5, device='cpu')),
             ('sfocal', lambda z: LS.SigmoidFocalLoss(2.0, 0.25, C())(z, y)),
             ('bfocal', lambda z: LS.FocalLoss()(z, y))]
    for key, fn in cases:
        z = x.clone().requires_grad_(True)
        loss = fn(z)
        loss.backward()
        np.testing.assert_allclose(loss.item(), d[key], rtol=RTOL, err_msg=key)
        np.testing.assert_allclose(z.grad.numpy(), d[key + '_grad'], rtol=1e-4, atol=1e-6, err_msg=key)


def test_nms_golden_on_cpu():
    d = load_golden('nms.npz')
    for k in range(int(d['n_cases'])):
        b, s = torch.from_numpy(d['c%d_boxes' % k]), torch.from_numpy(d['c%d_scores' % k])
        thr, tk = float(d['c%d_thr' % k]), int(d['c%d_topk' % k])
        keep, count = IU.nms(b, s, thr, tk)
        assert count == int(d['c%d_count' % k])
        np.testing.assert_array_equal(keep.numpy(), d['c%d_keep' % k])
        keep, count = IU.diounms(b, s, thr, tk)
        assert count == int(d['c%d_dcount' % k])
        np.testing.assert_array_equal(keep.numpy(), d['c%d_dkeep' % k])
    empty = IU.nms(torch.zeros(0, 4), torch.zeros(0))
    assert isinstance(empty, torch.Tensor) and bool(d['empty_is_tensor'])


def test_detect_golden_on_cpu():
    d = load_golden('detect.npz')
    P = torch.from_numpy(prior_table('SSD512')[::int(d['prior_stride'])].copy())
    for k in range(int(d['n_cases'])):
        fn, bt, ft = str(d['c%d_fn' % k]), str(d['c%d_box_type' % k]), str(d['c%d_focal_type' % k])
        ms, mo, tk = d['c%d_params' % k]
        locs = torch.from_numpy(d['c%d_locs' % k]).clone()
        scores = torch.from_numpy(d['c%d_scores' % k])
        pos = torch.from_numpy(d['c%d_pos' % k]).bool() if ('c%d_pos' % k) in d.files else None
        if fn == 'utils':
            res = MU.detect(locs, scores, ms, mo, int(tk), P, Cfg(device='cpu', focal_type=ft, model={'box_type': bt}),
                            prior_positives_idx=pos)
        elif fn == 'tools':
            res = DT.detect(locs, scores, ms, mo, int(tk), P)
        else:
            res = DT.detect_refine(locs, scores, ms, mo, int(tk), P, prior_positives_idx=pos)
        ob, ol, os_ = res
        np.testing.assert_array_equal([x.shape[0] for x in ob], d['c%d_counts' % k], err_msg='case %d' % k)
        np.testing.assert_array_equal(torch.cat(ol).numpy(), d['c%d_labels' % k], err_msg='case %d' % k)
        np.testing.assert_allclose(torch.cat(ob).numpy(), d['c%d_boxes' % k], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(torch.cat(os_).numpy(), d['c%d_scores_out' % k], rtol=1e-5, atol=1e-7)
        np.testing.assert_array_equal(locs.numpy(), d['c%d_locs_after' % k])


def test_dcn_golden_on_cpu():
    d = load_golden('dcn.npz')
    for k in range(int(d['n_cases'])):
        pre = 'c%d_' % k
        B, C, O, H, W, stride = [int(v) for v in d[pre + 'shape']]
        m = DeformConv2d(C, O, kernel_size=3, padding=1, stride=stride)
        with torch.no_grad():
            for n, p in m.named_parameters():
                p.copy_(torch.from_numpy(d[pre + 'w_' + n.replace('.', '_')]))
        x = torch.from_numpy(d[pre + 'x']).requires_grad_(True)
        out = m(x)
        out.backward(torch.from_numpy(d[pre + 'gout']))
        np.testing.assert_allclose(out.detach().numpy(), d[pre + 'out'], rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(x.grad.numpy(), d[pre + 'gx'], rtol=1e-4, atol=1e-5)
        for n, p in m.named_parameters():
            np.testing.assert_allclose(p.grad.numpy(), d[pre + 'g_' + n.replace('.', '_')], rtol=1e-4, atol=1e-4,
                                       err_msg=pre + n)


def test_map_golden_on_cpu():
    from shape_based_object_detection_amd import metrics
    d = load_golden('map.npz')
    for k in range(int(d['n_cases'])):
        B, C, thr, _ = d['c%d_params' % k]
        B, C = int(B), int(C)
        lists = [[torch.from_numpy(np.ascontiguousarray(d['c%d_%s%d' % (k, key, i)])) for i in range(B)]
                 for key in ('db', 'dl', 'ds', 'tb', 'tl', 'td')]
        lm = {'background': 0}
        lm.update({'c%d' % c: c for c in range(1, C)})
        aps, m = metrics.calculate_mAP(*lists, float(thr), lm, device='cpu')
        got = np.array([aps['c%d' % c] for c in range(1, C)], np.float32)
        np.testing.assert_allclose(got, d['c%d_ap' % k], rtol=1e-6, atol=0, err_msg='case %d' % k)
        np.testing.assert_allclose(m, d['c%d_map' % k], rtol=1e-6)


def test_kernels_stay_device_only():
    """The C-ABI wrappers in core never take CPU tensors: the host path is chosen by the drop-in
    modules, not by a fallback inside the HIP path."""
    from shape_based_object_detection_amd import _lib as L
    with pytest.raises(L.SbodError, match='ROCm device'):
        core.nms(torch.rand(4, 4), torch.rand(4), 0.5)
    with pytest.raises(L.SbodError, match='ROCm device'):
        core.detect(torch.rand(1, 8, 4), torch.rand(1, 8, 3), 0.01, 0.45, 5, torch.rand(8, 4))
