"""HIP matcher parity (bit-exact) against the oracle and the reference's golden vectors."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import match_ref as M
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd import _lib as L
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _gt(boxes, labels):
    return core.pack_gt([torch.as_tensor(b).to(DEV) for b in boxes],
                        [torch.as_tensor(l).to(DEV) for l in labels])


def test_jaccard_golden():
    d = load_golden('jaccard.npz')
    for k in range(int(d['n_cases'])):
        gt = _gt([d['c%d_gt' % k]], [np.zeros(d['c%d_gt' % k].shape[0], np.int64)])
        an = torch.from_numpy(d['c%d_anchors' % k]).to(DEV)
        out = core.iou_pairwise(gt, an)[0].cpu().numpy()
        np.testing.assert_array_equal(out, d['c%d_metrics' % k])
        out = core.iou_pairwise(gt, an, mode=L.IOU_PLAIN)[0].cpu().numpy()
        np.testing.assert_array_equal(out, d['c%d_plain' % k])


def test_match_golden():
    d = load_golden('match_ssd512.npz')
    P = prior_table('SSD512')
    pri = torch.from_numpy(P).to(DEV)
    pxy = core.codec('cxcy_to_xy', pri)
    np.testing.assert_array_equal(pxy.cpu().numpy(), M.cxcy_to_xy(P))
    for k in range(int(d['n_cases'])):
        gt = _gt([d['c%d_boxes' % k]], [d['c%d_labels' % k]])
        obj, ovl, npos = core.match(gt, pxy, P.shape[0])
        np.testing.assert_array_equal(obj[0].cpu().numpy(), d['c%d_obj' % k])
        np.testing.assert_array_equal(ovl[0].cpu().numpy(), d['c%d_ovl' % k])
        cls, neg, txy, enc = core.match_expand(gt, obj, ovl, pri)
        np.testing.assert_array_equal(cls[0].cpu().numpy(), d['c%d_cls' % k])
        np.testing.assert_array_equal(neg[0].cpu().numpy(), d['c%d_neg' % k])
        pos = d['c%d_cls' % k] > 0
        assert int(npos[0]) == int(pos.sum()) == int(npos[1])
        np.testing.assert_allclose(enc[0].cpu().numpy()[pos], d['c%d_enc_pos' % k], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('arch,B,seed,maxg', [('SSD512', 32, 0, 16), ('SSD300', 4, 1, 16),
                                              ('RETINA', 32, 2, 16), ('REFINEDET', 16, 3, 40),
                                              ('SSD512', 5, 4, 200), ('SSD512', 3, 5, 600),
                                              ('SSD300', 2, 6, 4096)])
def test_match_vs_oracle(arch, B, seed, maxg):
    """maxg > 256: objects reduced in several LDS chunks per tile; 4096 = the ABI's maximum."""
    P = prior_table(arch)
    pri = torch.from_numpy(P).to(DEV)
    pxy_np = M.cxcy_to_xy(P)
    boxes, labels = synth.make_gt(B, seed=seed, max_objects=maxg)
    gt = _gt(boxes, labels)
    obj, ovl, npos = core.match(gt, torch.from_numpy(pxy_np).to(DEV), P.shape[0])
    obj2, ovl2, npos2 = core.match(gt, torch.from_numpy(pxy_np).to(DEV), P.shape[0])
    assert torch.equal(obj, obj2) and torch.equal(ovl, ovl2) and torch.equal(npos, npos2)
    cls, neg, _, _ = core.match_expand(gt, obj, ovl, pri, want=('cls', 'neg'))
    tot = 0
    for b in range(B):
        o, v, c, n = M.match_criterion(boxes[b].numpy(), labels[b].numpy(), pxy_np)
        np.testing.assert_array_equal(obj[b].cpu().numpy(), o)
        np.testing.assert_array_equal(ovl[b].cpu().numpy(), v)
        np.testing.assert_array_equal(cls[b].cpu().numpy(), c)
        np.testing.assert_array_equal(neg[b].cpu().numpy(), n)
        assert int(npos[b]) == int((c > 0).sum())
        tot += int((c > 0).sum())
    assert int(npos[B]) == tot


def _check_oracle(boxes, labels, obj, ovl, npos, pxy_np):
    tot = 0
    for b in range(len(boxes)):
        o, v, c, n = M.match_criterion(boxes[b], labels[b], pxy_np)
        np.testing.assert_array_equal(obj[b].cpu().numpy(), o)
        np.testing.assert_array_equal(ovl[b].cpu().numpy(), v)
        assert int(npos[b]) == int((c > 0).sum())
        tot += int((c > 0).sum())
    assert int(npos[len(boxes)]) == tot


def test_match_forced_collisions_and_counter_reuse():
    """Objects that share a best prior (identical boxes, tiny boxes around one point): the forced
    match's last writer wins and the positive count follows it.  Calls with different batch
    sizes on one workspace: the in-launch arrival counters are left zero by every call."""
    P = prior_table('SSD512')
    pxy_np = M.cxcy_to_xy(P)
    pxy = torch.from_numpy(pxy_np).to(DEV)
    rng = np.random.default_rng(7)
    boxes, labels = [], []
    for b in range(6):
        xy = rng.uniform(0, 0.6, (5, 2)).astype(np.float32)
        wh = rng.uniform(0.05, 0.35, (5, 2)).astype(np.float32)
        base = np.concatenate([xy, xy + wh], 1)
        c = rng.uniform(0.2, 0.8, 2).astype(np.float32)
        tiny = np.concatenate([np.tile(c - 1e-3, (4, 1)), np.tile(c + 1e-3, (4, 1))], 1)
        tiny[:, :2] -= np.arange(4, dtype=np.float32)[:, None] * 1e-4
        bx = np.concatenate([np.repeat(base[:2], 3, 0), base[2:], tiny]).astype(np.float32)
        boxes.append(bx)
        labels.append(rng.integers(1, 21, bx.shape[0]).astype(np.int64))
    for sel in (range(6), range(2), range(6), [5]):
        bs, ls = [boxes[i] for i in sel], [labels[i] for i in sel]
        obj, ovl, npos = core.match(_gt(bs, ls), pxy, P.shape[0])
        _check_oracle(bs, ls, obj, ovl, npos, pxy_np)


def test_refinedet_arm_odm():
    P = prior_table('REFINEDET')
    pri = torch.from_numpy(P).to(DEV)
    B = 3
    boxes, labels = synth.make_gt(B, seed=21)
    arm_locs, arm_scores = synth.make_preds(B, P.shape[0], 2, seed=21)
    d = load_golden('match_refinedet.npz')
    gt = _gt(boxes, labels)
    pxy = core.codec('cxcy_to_xy', pri)
    obj, ovl, npos = core.match(gt, pxy, P.shape[0], flags=L.MATCH_BINARY)
    cls, _, _, _ = core.match_expand(gt, obj, ovl, pri, flags=L.MATCH_BINARY, want=('cls',))
    np.testing.assert_array_equal(cls.cpu().numpy(), d['arm_cls'])
    al, asc = arm_locs.to(DEV), arm_scores.to(DEV)
    obj, ovl, npos = core.match(gt, al, P.shape[0], flags=L.MATCH_ODM, priors_cxcy=pri, arm_scores=asc)
    cls, _, _, enc = core.match_expand(gt, obj, ovl, pri, flags=L.MATCH_ODM, arm_locs=al,
                                       want=('cls', 'enc'))
    np.testing.assert_array_equal(cls.cpu().numpy(), d['odm_cls'])
    # shared decode: oracle matched against the GPU's decoded anchors is bit-identical
    dec = core.codec('decode_tenfive_xy', al, pri).cpu().numpy()
    for b in range(B):
        o, v, c, _ = M.match_criterion(boxes[b].numpy(), labels[b].numpy(), dec[b])
        np.testing.assert_array_equal(obj[b].cpu().numpy(), o)
    assert int(npos[B]) == int(d['odm_pos'].sum())
    odm_cls = d['odm_cls']
    np.testing.assert_allclose(enc.cpu().numpy()[odm_cls > 0], d['odm_enc_pos'], rtol=1e-4, atol=1e-5)


def test_iou_utils_match_golden():
    d = load_golden('match_iou_utils.npz')
    P = prior_table('SSD300')
    pri = torch.from_numpy(P).to(DEV)
    for i in range(2):
        tr = torch.from_numpy(d['b%d_boxes' % i]).to(DEV)
        lb = torch.from_numpy(d['b%d_labels' % i]).to(DEV)
        for enc, lk, ck in [(1, 'match_loc', 'match_conf'), (0, 'match_ious_loc', 'match_ious_conf')]:
            loc = torch.zeros(P.shape[0], 4, device=DEV)
            conf = torch.zeros(P.shape[0], dtype=torch.int64, device=DEV)
            nb = 1 << 20
            ws = core.workspace(nb, DEV)
            L.call('sbod_match_ssd_f32', L.ptr(tr), L.ptr(lb), tr.shape[0], L.ptr(pri), P.shape[0],
                   0.5, 0.1, 0.2, enc, L.ptr(loc), L.ptr(conf), L.ptr(ws), nb, L.stream_of(tr))
            np.testing.assert_array_equal(conf.cpu().numpy(), d[ck][i])
            np.testing.assert_allclose(loc.cpu().numpy(), d[lk][i], rtol=1e-5, atol=1e-5)


def test_codecs_golden():
    d = load_golden('codecs.npz')
    p = torch.from_numpy(d['priors']).to(DEV)
    bx = torch.from_numpy(d['boxes']).to(DEV)
    lc = torch.from_numpy(d['locs']).to(DEV)
    np.testing.assert_array_equal(core.codec('xy_to_cxcy', bx).cpu().numpy(), d['xy_to_cxcy'])
    np.testing.assert_array_equal(core.codec('cxcy_to_xy', p).cpu().numpy(), d['cxcy_to_xy'])
    np.testing.assert_allclose(core.codec('encode_tenfive', core.codec('xy_to_cxcy', bx), p).cpu().numpy(),
                               d['cxcy_to_gcxgcy'], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(core.codec('decode_tenfive', lc, p).cpu().numpy(), d['gcxgcy_to_cxcy'],
                               rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(core.codec('encode_var', bx, p).cpu().numpy(), d['encode'], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(core.codec('decode_var', lc, p).cpu().numpy(), d['decode'], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('counts', [(64, 1, 64), (1, 63, 64, 65, 127, 128, 129), (65, 2)])
def test_match_object_count_boundaries(counts):
    """Object counts at the 64-object chunk of k_match_tile and the register / LDS switch of
    k_match_final (Gmax <= 64 vs > 64), in one batch; an object repeated across a chunk boundary
    (objects 10 and 70 identical) so the forced match's last writer sits in another chunk."""
    P = prior_table('SSD512')
    pxy_np = M.cxcy_to_xy(P)
    pxy = torch.from_numpy(pxy_np).to(DEV)
    rng = np.random.default_rng(sum(counts))
    boxes, labels = [], []
    for g in counts:
        xy = rng.uniform(0, 0.7, (g, 2)).astype(np.float32)
        wh = rng.uniform(0.02, 0.3, (g, 2)).astype(np.float32)
        bx = np.concatenate([xy, np.minimum(xy + wh, 1.0)], 1).astype(np.float32)
        if g > 70:
            bx[70] = bx[10]
        boxes.append(bx)
        labels.append(rng.integers(1, 21, g).astype(np.int64))
    obj, ovl, npos = core.match(_gt(boxes, labels), pxy, P.shape[0])
    _check_oracle(boxes, labels, obj, ovl, npos, pxy_np)
