"""numpy restatement of the reference's integer / index work (TEST INFRASTRUCTURE ONLY).

float32 element-wise arithmetic in numpy rounds exactly like torch-CPU's kernels for
+, -, *, /, min, max, so the IoU matrices, argmax assignments and NMS decisions here are the
reference's bit for bit (pinned by tests/golden).  log/exp (box codecs) agree to ~1 ulp only.

Thresholds given as Python floats are compared as float32 (torch casts the scalar to the
tensor dtype — probed: ``torch.tensor([1e-5f]) < 1e-5`` is False).
"""
import numpy as np

F32 = np.float32
EPS = F32(1e-5)


# ----------------------------------------------------------------------------- pairwise IoU
def find_jaccard_overlap(gt, anchors):
    """``metrics.py:208-252``: [G,P] IoU with the +1e-5 denominator and degenerate masks
    (zero GT → 0, zero anchor → −1, the anchor mask applied last)."""
    gt = np.asarray(gt, F32)[:, None, :]
    an = np.asarray(anchors, F32)[None, :, :]
    iw = np.minimum(gt[..., 2], an[..., 2]) - np.maximum(gt[..., 0], an[..., 0])
    iw[iw < 0] = 0
    ih = np.minimum(gt[..., 3], an[..., 3]) - np.maximum(gt[..., 1], an[..., 1])
    ih[ih < 0] = 0
    gx = gt[..., 2] - gt[..., 0]
    gy = gt[..., 3] - gt[..., 1]
    g_area = gx * gy
    g_zero = (np.abs(gx) < EPS) & (np.abs(gy) < EPS)
    ax = an[..., 2] - an[..., 0]
    ay = an[..., 3] - an[..., 1]
    a_area = ax * ay
    a_zero = (ax < EPS) & (ay < EPS)
    inner = iw * ih
    with np.errstate(divide='ignore', invalid='ignore'):
        ov = inner / (g_area + a_area - inner + EPS)
    ov = np.broadcast_to(ov, np.broadcast_shapes(g_zero.shape, a_zero.shape)).copy()
    ov[np.broadcast_to(g_zero, ov.shape)] = 0
    ov[np.broadcast_to(a_zero, ov.shape)] = -1
    return ov.astype(F32)


def jaccard_plain(a, b):
    """``operators/iou_utils.py:192-233``: plain IoU, no EPS and no masks."""
    a = np.asarray(a, F32)[:, None, :]
    b = np.asarray(b, F32)[None, :, :]
    w = np.maximum(np.minimum(a[..., 2], b[..., 2]) - np.maximum(a[..., 0], b[..., 0]), F32(0))
    h = np.maximum(np.minimum(a[..., 3], b[..., 3]) - np.maximum(a[..., 1], b[..., 1]), F32(0))
    inter = w * h
    area_a = (a[..., 2] - a[..., 0]) * (a[..., 3] - a[..., 1])
    area_b = (b[..., 2] - b[..., 0]) * (b[..., 3] - b[..., 1])
    with np.errstate(divide='ignore', invalid='ignore'):
        return (inter / (area_a + area_b - inter)).astype(F32)


# ----------------------------------------------------------------------------- codecs
def xy_to_cxcy(xy):          # dataset/transforms.py:26-34
    xy = np.asarray(xy, F32)
    return np.concatenate([(xy[:, 2:] + xy[:, :2]) / F32(2), xy[:, 2:] - xy[:, :2]], 1)


def cxcy_to_xy(c):           # dataset/transforms.py:37-45
    c = np.asarray(c, F32)
    return np.concatenate([c[:, :2] - c[:, 2:] / F32(2), c[:, :2] + c[:, 2:] / F32(2)], 1)


def cxcy_to_gcxgcy(c, p):    # dataset/transforms.py:48-66
    c, p = np.asarray(c, F32), np.asarray(p, F32)
    with np.errstate(divide='ignore', invalid='ignore'):
        return np.concatenate([(c[:, :2] - p[:, :2]) / (p[:, 2:] / F32(10)),
                               np.log(c[:, 2:] / p[:, 2:]) * F32(5)], 1)


def gcxgcy_to_cxcy(g, p):    # dataset/transforms.py:69-83
    g, p = np.asarray(g, F32), np.asarray(p, F32)
    return np.concatenate([g[:, :2] * p[:, 2:] / F32(10) + p[:, :2],
                           np.exp(g[:, 2:] / F32(5)) * p[:, 2:]], 1)


def point_form(p):           # operators/iou_utils.py:167-177
    p = np.asarray(p, F32)
    return np.concatenate([p[:, :2] - p[:, 2:] / F32(2), p[:, :2] + p[:, 2:] / F32(2)], 1)


def encode_var(matched, priors, v):   # operators/iou_utils.py:324-345
    m, p = np.asarray(matched, F32), np.asarray(priors, F32)
    g = (m[:, :2] + m[:, 2:]) / F32(2) - p[:, :2]
    g = g / (F32(v[0]) * p[:, 2:])
    with np.errstate(divide='ignore', invalid='ignore'):
        wh = np.log((m[:, 2:] - m[:, :2]) / p[:, 2:]) / F32(v[1])
    return np.concatenate([g, wh], 1)


def decode_var(loc, priors, v):       # operators/iou_utils.py:349-368
    loc, p = np.asarray(loc, F32), np.asarray(priors, F32)
    c = p[:, :2] + loc[:, :2] * F32(v[0]) * p[:, 2:]
    wh = p[:, 2:] * np.exp(loc[:, 2:] * F32(v[1]))
    xy = c - wh / F32(2)
    return np.concatenate([xy, wh + xy], 1)


# ----------------------------------------------------------------------------- matching
def match_criterion(gt, labels, anchors_xy, threshold=0.5, neg_delta=0.1, binary=False):
    """The criteria's per-image matching block, ``models/SSD512.py:535-563`` (identical in
    ``SSD300.py:504-533``, ``RetinaNet.py:412-441``, ``RefineDet512.py:749-781`` (binary) and
    ``:851-878`` (vs decoded ARM boxes)).

    Returns (obj [P] int64, ovl [P] f32, cls [P] int64, neg [P] int64 (−1 / label)).
    Forced match: ``j`` indexes the FILTERED object list, last writer wins."""
    ov = find_jaccard_overlap(gt, anchors_xy)
    ovl = ov.max(0).copy()
    obj = ov.argmax(0).astype(np.int64)          # first index on ties (torch CPU semantics)
    best_pri = ov.argmax(1)
    pri_f = best_pri[ov.max(1) > 0]
    if len(pri_f):
        ovl[pri_f] = F32(1.0)
    for j, p in enumerate(pri_f):
        obj[p] = j
    labels = np.asarray(labels, np.int64)
    cls = labels[obj].copy()
    neg = labels[obj].copy()
    cls[ovl < F32(threshold)] = 0
    neg[ovl < F32(threshold - neg_delta)] = -1
    if binary:
        cls = (cls > 0).astype(np.int64)
    return obj, ovl, cls, neg


def match_iou_utils(threshold, truths, priors, variances, labels, encode=True):
    """``operators/iou_utils.py:236-321`` (``match`` / ``match_ious``): plain jaccard vs
    point_form(priors), forced-match fill value 2, UNFILTERED j, ``conf = labels + 1``."""
    ov = jaccard_plain(truths, point_form(priors))
    best_pri = ov.argmax(1)
    bto = ov.max(0).copy()
    bti = ov.argmax(0).astype(np.int64)
    bto[best_pri] = F32(2)
    for j in range(best_pri.shape[0]):
        bti[best_pri[j]] = j
    matches = np.asarray(truths, F32)[bti]
    conf = np.asarray(labels, np.int64)[bti] + 1
    conf[bto < F32(threshold)] = 0
    loc = encode_var(matches, priors, variances) if encode else matches
    return loc, conf


# ----------------------------------------------------------------------------- NMS
def _stable_desc(scores):
    return np.argsort(-np.asarray(scores, np.float64), kind='stable')


def nms_greedy(boxes, scores, overlap, top_k=None, variant='tv', beta1=1.0):
    """Greedy NMS; returns kept indices in descending-score order.

    variant 'ref'  — ``operators/iou_utils.py:385-450``: keep top_k before suppressing,
                      union = (area_j − inter) + area_i, keep iff IoU <= thr (NaN suppressed).
    variant 'tv'   — torchvision.ops.nms semantics (``models/utils.py:265``): union =
                      (area_i + area_j) − inter, suppress iff IoU > thr (NaN kept).
    variant 'diou' — ``iou_utils.py:453-530`` incl. the ``center_y2 = (yy2 + yy2)/2`` quirk.
    Ties: stable descending order (lower index first) — the documented tie rule."""
    b = np.asarray(boxes, F32)
    n = b.shape[0]
    if n == 0:
        return np.zeros(0, np.int64)
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    area = (x2 - x1) * (y2 - y1)
    order = _stable_desc(scores)
    if top_k is not None:
        order = order[:top_k]
    thr = F32(overlap)
    keep = []
    alive = order
    while alive.size:
        i = alive[0]
        keep.append(int(i))
        rest = alive[1:]
        if rest.size == 0:
            break
        xx1 = np.maximum(x1[rest], x1[i])
        yy1 = np.maximum(y1[rest], y1[i])
        xx2 = np.minimum(x2[rest], x2[i])
        yy2 = np.minimum(y2[rest], y2[i])
        w = np.maximum(xx2 - xx1, F32(0))
        h = np.maximum(yy2 - yy1, F32(0))
        inter = w * h
        with np.errstate(divide='ignore', invalid='ignore'):
            if variant == 'tv':
                iou = inter / ((area[i] + area[rest]) - inter)
                alive = rest[~(iou > thr)]
                continue
            iou = inter / ((area[rest] - inter) + area[i])
            if variant == 'diou':
                cx1 = (x1[i] + x2[i]) / F32(2)
                cy1 = (y1[i] + y2[i]) / F32(2)
                cx2 = (x1[rest] + x2[rest]) / F32(2)
                cy2 = (y2[rest] + y2[rest]) / F32(2)
                d = (cx1 - cx2) ** 2 + (cy1 - cy2) ** 2
                ex1 = np.minimum(x1[rest], x1[i])
                ey1 = np.minimum(y1[rest], y1[i])
                ex2 = np.maximum(x2[rest], x2[i])
                ey2 = np.maximum(y2[rest], y2[i])
                c = (ex2 - ex1) ** 2 + (ey2 - ey1) ** 2
                u = d / c
                iou = iou - (u if beta1 == 1.0 else u ** F32(beta1))
        alive = rest[iou <= thr]
    return np.asarray(keep, np.int64)


# ----------------------------------------------------------------------------- detect
def detect(probs, boxes, min_score, max_overlap, top_k, pos=None, final_nms=None,
           nms_variant='tv'):
    """``models/utils.py:181-297`` on PRE-ACTIVATED probabilities [B,P,C] and PRE-DECODED,
    clamped boxes [B,P,4] (parity is pinned on shared activations/decodes: SURVEY §8(c)).
    ``final_nms=0.7`` gives ``detect_scripts/detect_tools.py:202-205`` / ``:324-327``.
    Returns lists of (boxes [K,4] f32, labels [K] int64, scores [K] f32)."""
    probs = np.asarray(probs, F32)
    boxes = np.asarray(boxes, F32)
    B, P, C = probs.shape
    out_b, out_l, out_s = [], [], []
    for b in range(B):
        if pos is not None:
            sel = np.flatnonzero(np.asarray(pos[b]).astype(bool))
            sc_all, bx_all = probs[b][sel], boxes[b][sel]
        else:
            sc_all, bx_all = probs[b], boxes[b]
        ib, il, is_ = [], [], []
        for c in range(1, C):
            s = sc_all[:, c]
            cand = np.flatnonzero(s > F32(min_score))
            if cand.size == 0:
                continue
            cs, cb = s[cand], bx_all[cand]
            keep = nms_greedy(cb, cs, max_overlap, variant=nms_variant)
            ib.append(cb[keep])
            il.append(np.full(keep.size, c, np.int64))
            is_.append(cs[keep])
        if not ib:
            ib, il, is_ = [np.array([[0, 0, 1, 1]], F32)], [np.zeros(1, np.int64)], [np.zeros(1, F32)]
        ib, il, is_ = np.concatenate(ib), np.concatenate(il), np.concatenate(is_)
        n_objects = is_.size
        if final_nms is not None:
            k = nms_greedy(ib, is_, final_nms, variant=nms_variant)
            ib, il, is_ = ib[k], il[k], is_[k]
        if n_objects > top_k:
            o = _stable_desc(is_)
            ib, il, is_ = ib[o][:top_k], il[o][:top_k], is_[o][:top_k]
        out_b.append(ib)
        out_l.append(il)
        out_s.append(is_)
    return out_b, out_l, out_s


def softmax_np(x, axis=-1):
    x = np.asarray(x, np.float64)
    e = np.exp(x - x.max(axis, keepdims=True))
    return (e / e.sum(axis, keepdims=True)).astype(F32)


def decode_boxes(locs, priors_cxcy, box_type):
    """Per-image decode + clamp of ``models/utils.py:218-224``."""
    locs = np.asarray(locs, F32)
    out = []
    for b in range(locs.shape[0]):
        if box_type == 'offset':
            d = cxcy_to_xy(gcxgcy_to_cxcy(locs[b], priors_cxcy))
        elif box_type == 'center':
            d = cxcy_to_xy(locs[b])
        else:
            d = locs[b].copy()
        out.append(np.clip(d, F32(0), F32(1)))
    return np.stack(out)
