"""The GT packing folded into the matcher (sbod_match_lists_f32 / sbod_criterion_focal_lists): the
first matcher launch reads each image's rows in place from the collate_fn lists and writes the
packed copy the later launches read.  Against sbod_gt_pack followed by the packed entry points on
the same inputs, every output must be bit-identical (the same per-prior arithmetic on the same
rows); the packed copy must equal torch.cat of the lists; and batches the list form does not take
(an empty image, more than 64 images, more objects than Gmax) are refused with SBOD_E_INVALID."""
import numpy as np
import pytest
import torch

from shape_based_object_detection_amd import _lib as L
from shape_based_object_detection_amd import synth
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = 'cuda'
E_INVALID = -1   # SBOD_E_INVALID


class Cfg(dict):
    __getattr__ = dict.__getitem__


def _lists(B, seed, max_objects=16, C=21):
    boxes, labels = synth.make_gt(B, seed=seed, max_objects=max_objects, n_classes=C)
    return [b.to(DEV).contiguous() for b in boxes], [l.to(DEV).contiguous() for l in labels]


_KEEP = []


def _ptr_arrays(boxes, labels):
    """Host arrays of device pointers / counts (as sbod_gt_pack takes them), as addresses."""
    bp = np.array([b.data_ptr() for b in boxes], np.uint64)
    lp = np.array([l.data_ptr() for l in labels], np.uint64)
    cnt = np.array([b.shape[0] for b in boxes], np.int32)
    _KEEP[:] = [bp, lp, cnt]
    return bp.ctypes.data, lp.ctypes.data, cnt.ctypes.data


def _packed_out(cap, B):
    return (torch.full((cap, 4), -7.0, device=DEV), torch.full((cap,), -7, dtype=torch.int64, device=DEV),
            torch.full((B + 1,), -7, dtype=torch.int32, device=DEV))


def _criterion(boxes, labels, kind, arch, reg, dtype, fold, seed, C=21):
    P = torch.from_numpy(prior_table(arch)).to(DEV)
    cls = {'ssd512': CR.MultiBoxLoss512, 'retina': CR.RetinaFocalLoss}[kind]
    crit = cls(priors_cxcy=P, config=Cfg(reg_weights=1.0, device=DEV, n_classes=C, reg_loss=reg, cls_loss='focal'))
    spec = crit._spec()
    B, NP = len(boxes), P.shape[0]
    locs, scores = synth.make_preds(B, NP, C, seed=seed)
    locs, scores = locs.to(DEV, dtype).contiguous(), scores.to(DEV, dtype).contiguous()
    dt = L.DT_F32 if dtype == torch.float32 else L.DT_BF16
    cap = sum(b.shape[0] for b in boxes) + 5
    gb, gl_, go = _packed_out(cap, B)
    gmax = max(b.shape[0] for b in boxes)
    obj = torch.empty(B, NP, dtype=torch.int32, device=DEV)
    ovl = torch.empty(B, NP, dtype=torch.float32, device=DEV)
    npos = torch.empty(B + 1, dtype=torch.int32, device=DEV)
    g_locs, g_scores = torch.empty_like(locs), torch.empty_like(scores)
    out = torch.empty(4, device=DEV)
    lib = L.lib()
    nb = lib.sbod_criterion_workspace_bytes(B, gmax, NP)
    ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
    stream = L.stream_of(locs)
    bp, lp, cnt = _ptr_arrays(boxes, labels)
    flags = (spec.flags & L.LOSS_FOCAL_NORM) | L.CRIT_TWO_LAUNCH
    tail = (gmax, float(crit.threshold), float(crit.threshold - 0.1), spec.reg, flags, float(spec.reg_weight),
            float(spec.alpha), float(spec.gamma), L.ptr(obj), L.ptr(ovl), L.ptr(npos), L.ptr(g_locs),
            L.ptr(g_scores), L.ptr(out), L.ptr(ws), nb, stream)
    if fold:
        L.call('sbod_criterion_focal_lists', bp, lp, cnt, cap, L.ptr(locs), L.ptr(scores), dt, B, NP, C,
               L.ptr(crit.priors_cxcy), L.ptr(crit.priors_xy), L.ptr(gb), L.ptr(gl_), L.ptr(go), *tail)
    else:
        L.call('sbod_gt_pack', bp, lp, cnt, B, cap, L.ptr(gb), L.ptr(gl_), L.ptr(go), stream)
        L.call('sbod_criterion_focal', L.ptr(locs), L.ptr(scores), dt, B, NP, C, L.ptr(crit.priors_cxcy),
               L.ptr(crit.priors_xy), L.ptr(gb), L.ptr(gl_), L.ptr(go), *tail)
    torch.cuda.synchronize()
    n = int(go[B].item())
    return dict(obj=obj, ovl=ovl, npos=npos, out=out, gl=g_locs, gs=g_scores, gb=gb[:n], glab=gl_[:n], go=go)


@pytest.mark.parametrize('kind,arch,B,reg,dtype,maxo', [
    ('ssd512', 'SSD512', 32, 'diou', torch.float32, 16), ('ssd512', 'SSD512', 64, 'smoothl1', torch.float32, 8),
    ('ssd512', 'SSD512', 5, 'diou', torch.bfloat16, 16), ('ssd512', 'SSD512', 4, 'diou', torch.float32, 150),
    ('retina', 'RETINA', 8, 'diou', torch.float32, 1)])
def test_criterion_lists_equals_pack_then_criterion(kind, arch, B, reg, dtype, maxo):
    boxes, labels = _lists(B, seed=B + 3, max_objects=maxo)
    a = _criterion(boxes, labels, kind, arch, reg, dtype, True, seed=B)
    b = _criterion(boxes, labels, kind, arch, reg, dtype, False, seed=B)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(a['gb'], torch.cat(boxes)) and torch.equal(a['glab'], torch.cat(labels))
    offs = np.concatenate([[0], np.cumsum([x.shape[0] for x in boxes])])
    np.testing.assert_array_equal(a['go'].cpu().numpy(), offs)


@pytest.mark.parametrize('flags', [0, L.MATCH_BINARY, L.MATCH_ODM])
def test_match_lists_equals_pack_then_match(flags):
    """Plain (SSD / RetinaNet), binary (RefineDet ARM) and ODM (RefineDet: anchors = the ARM locs
    decoded against the priors, easy negatives from the ARM scores) matcher forms."""
    B = 16
    boxes, labels = _lists(B, seed=41, max_objects=40)
    P = torch.from_numpy(prior_table('SSD512')).to(DEV)
    pxy = torch.cat([P[:, :2] - P[:, 2:] / 2, P[:, :2] + P[:, 2:] / 2], 1).contiguous()
    NP = P.shape[0]
    pri, arm_sc = None, None
    if flags == L.MATCH_ODM:
        g = torch.Generator(device=DEV).manual_seed(5)
        pxy = (torch.randn(B, NP, 4, device=DEV, generator=g) * 0.5).contiguous()    # ARM locs (gcxgcy)
        pri = P.contiguous()
        arm_sc = torch.randn(B, NP, 2, device=DEV, generator=g).contiguous()
    cap = sum(b.shape[0] for b in boxes)
    gmax = max(b.shape[0] for b in boxes)
    nb = L.lib().sbod_match_workspace_bytes_p(B, gmax, NP)
    stream = L._raw_stream(0)
    bp, lp, cnt = _ptr_arrays(boxes, labels)
    res = []
    for fold in (True, False):
        gb, gl_, go = _packed_out(cap, B)
        obj = torch.empty(B, NP, dtype=torch.int32, device=DEV)
        ovl = torch.empty(B, NP, dtype=torch.float32, device=DEV)
        npos = torch.empty(B + 1, dtype=torch.int32, device=DEV)
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        tail = (L.ptr(pxy), L.ptr(pri), L.ptr(arm_sc), NP, 0.5, 0.01, flags, L.ptr(obj), L.ptr(ovl), L.ptr(npos),
                L.ptr(ws), nb, stream)
        if fold:
            L.call('sbod_match_lists_f32', bp, lp, cnt, cap, L.ptr(gb), L.ptr(gl_), L.ptr(go), B, gmax, *tail)
        else:
            L.call('sbod_gt_pack', bp, lp, cnt, B, cap, L.ptr(gb), L.ptr(gl_), L.ptr(go), stream)
            L.call('sbod_match_f32', L.ptr(gb), L.ptr(gl_), L.ptr(go), B, gmax, *tail)
        torch.cuda.synchronize()
        res.append((obj, ovl, npos, gb, gl_, go))
    for x, y in zip(*res):
        assert torch.equal(x, y)


def test_lists_form_refuses_what_it_does_not_take():
    P = torch.from_numpy(prior_table('SSD300')).to(DEV)
    pxy = torch.cat([P[:, :2] - P[:, 2:] / 2, P[:, :2] + P[:, 2:] / 2], 1).contiguous()
    NP = P.shape[0]
    stream = L._raw_stream(0)

    def run(boxes, labels, gmax):
        B = len(boxes)
        cap = max(sum(b.shape[0] for b in boxes), 1)
        gb, gl_, go = _packed_out(cap, B)
        obj = torch.empty(B, NP, dtype=torch.int32, device=DEV)
        ovl = torch.empty(B, NP, device=DEV)
        npos = torch.empty(B + 1, dtype=torch.int32, device=DEV)
        nb = L.lib().sbod_match_workspace_bytes_p(B, gmax, NP)
        ws = torch.zeros(nb, dtype=torch.uint8, device=DEV)
        bp, lp, cnt = _ptr_arrays(boxes, labels)
        return L.lib().sbod_match_lists_f32(bp, lp, cnt, cap, L.ptr(gb), L.ptr(gl_), L.ptr(go), B, gmax, L.ptr(pxy),
                                            None, None, NP, 0.5, 0.01, 0, L.ptr(obj), L.ptr(ovl), L.ptr(npos),
                                            L.ptr(ws), nb, stream)

    boxes, labels = _lists(4, seed=5, max_objects=6)
    assert run(boxes, labels, 16) == 0
    e_box, e_lab = torch.zeros(0, 4, device=DEV), torch.zeros(0, dtype=torch.int64, device=DEV)
    assert run(boxes[:2] + [e_box], labels[:2] + [e_lab], 16) == E_INVALID          # an empty image
    many_b, many_l = _lists(65, seed=6, max_objects=2)
    assert run(many_b, many_l, 16) == E_INVALID                                       # > 64 images
    assert run(boxes, labels, 1) == E_INVALID or max(b.shape[0] for b in boxes) == 1  # > Gmax objects
    torch.cuda.synchronize()
