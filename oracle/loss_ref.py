"""torch-CPU fp32 restatement of the loss family and criteria (TEST INFRASTRUCTURE ONLY).

Floating-point kernels are checked against a plain torch fp32 reference with autograd for
the gradients; assignment (integer) work comes from ``match_ref`` (numpy, bit-exact).
Each function follows the cited reference lines' operation order.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import match_ref as M


def _t(x):
    return torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x


# ----------------------------------------------------------------------------- aligned overlaps
def aligned_overlap(kind, b1, b2):
    """Row-wise IoU / GIoU / DIoU / CIoU, ``operators/iou_utils.py:6-164``."""
    w1 = b1[:, 2] - b1[:, 0]
    h1 = b1[:, 3] - b1[:, 1]
    w2 = b2[:, 2] - b2[:, 0]
    h2 = b2[:, 3] - b2[:, 1]
    a1, a2 = w1 * h1, w2 * h2
    imax = torch.min(b1[:, 2:], b2[:, 2:])
    imin = torch.max(b1[:, :2], b2[:, :2])
    inter = torch.clamp(imax - imin, min=0)
    ia = inter[:, 0] * inter[:, 1]
    union = a1 + a2 - ia
    if kind == 'iou':
        return torch.clamp(ia / union, min=0, max=1.0)
    omax = torch.max(b1[:, 2:], b2[:, 2:])
    omin = torch.min(b1[:, :2], b2[:, :2])
    outer = torch.clamp(omax - omin, min=0)
    if kind == 'giou':
        closure = outer[:, 0] * outer[:, 1]
        return torch.clamp(ia / union - (closure - union) / closure, min=-1.0, max=1.0)
    cx1 = (b1[:, 2] + b1[:, 0]) / 2
    cy1 = (b1[:, 3] + b1[:, 1]) / 2
    cx2 = (b2[:, 2] + b2[:, 0]) / 2
    cy2 = (b2[:, 3] + b2[:, 1]) / 2
    idiag = (cx2 - cx1) ** 2 + (cy2 - cy1) ** 2
    odiag = outer[:, 0] ** 2 + outer[:, 1] ** 2
    if kind == 'diou':
        return torch.clamp(ia / union - idiag / odiag, min=-1.0, max=1.0)
    u = idiag / odiag
    iou = ia / union
    with torch.no_grad():                       # iou_utils.py:86-91
        arctan = torch.atan(w2 / h2) - torch.atan(w1 / h1)
        v = (4 / (math.pi ** 2)) * torch.pow(arctan, 2)
        alpha = v / ((1 - iou) + v)
        w_temp = 2 * w1
    ar = (8 / (math.pi ** 2)) * arctan * ((w1 - w_temp) * h1)
    return torch.clamp(iou - (u + alpha * ar), min=-1.0, max=1.0)


def iou_loss(kind, loc_p, loc_t, mode='Corner', variances=None, priors=None, weights=None,
             reduce='mean'):
    """``operators/Loss.py:164-200``."""
    num = loc_p.shape[0]
    if mode == 'Center':
        c = torch.cat([priors[:, :2] + loc_p[:, :2] * variances[0] * priors[:, 2:],
                       priors[:, 2:] * torch.exp(loc_p[:, 2:] * variances[1])], 1)
        xy = c[:, :2] - c[:, 2:] / 2
        boxes = torch.cat([xy, c[:, 2:] + xy], 1)
    else:
        boxes = loc_p
    loss = 1.0 - aligned_overlap(kind.lower(), boxes, loc_t)
    if weights is not None and weights.sum() > 1e-6:
        return (loss * weights).sum() / weights.sum()
    return loss.sum() / num if reduce == 'mean' else loss.sum()


def smooth_l1(pred, target, beta=1.0 / 9.0, weights=None, reduction='mean'):
    """``operators/Loss.py:203-226``."""
    x = (pred - target).abs()
    l = torch.where(x >= beta, x - 0.5 * beta, 0.5 * x ** 2 / beta)
    if weights is not None and weights.sum() > 1e-6:
        return (l * weights).sum() / weights.sum()
    return l.sum() / pred.size(0) if reduction == 'mean' else l.sum()


def focal_softmax(logits, y, alpha=0.25, gamma=2.0):
    """``operators/Loss.py:9-38``: background rows weighted by p_bg (sic), α_bg = 1 − α."""
    if isinstance(alpha, (list, tuple)):
        fa, ba = alpha[0], alpha[1]
    else:
        fa, ba = alpha, 1 - alpha
    onehot = torch.eye(logits.shape[-1], dtype=logits.dtype)[y]
    p = F.softmax(logits, dim=1)
    af = torch.cat([onehot[:, :1] * ba, onehot[:, 1:] * fa], 1)
    fw = torch.cat([onehot[:, :1] * p[:, :1], onehot[:, 1:] * (1 - p[:, 1:])], 1)
    return (af * fw ** gamma * (-1 * torch.log(p))).sum()


def focal_sigmoid(logits, y, gamma=2.0, alpha=0.25):
    """``operators/Loss.py:41-80``: background (t == 0) rows contribute nothing."""
    C = logits.shape[1]
    ids = torch.arange(1, C, dtype=y.dtype).unsqueeze(0)
    t = y.unsqueeze(1)
    p = torch.sigmoid(logits[:, 1:])
    term1 = (1 - p) ** gamma * torch.log(p)
    term2 = p ** gamma * torch.log(1 - p)
    loss = -(t == ids).float() * alpha * term1 - ((t != ids) * (t > 0)).float() * (1 - alpha) * term2
    return loss.sum()


def focal_bce(logits, y, alpha=0.25, gamma=2):
    """``operators/Loss.py:83-103`` (one-hot over ALL C columns incl. background)."""
    ids = torch.arange(0, logits.shape[1], dtype=y.dtype).unsqueeze(0)
    tgt = (y.unsqueeze(1) == ids).float()
    pred = logits.sigmoid().clamp(min=1e-4, max=1 - 1e-4)
    ce = F.binary_cross_entropy_with_logits(logits, tgt, reduction='none')
    a = tgt * alpha + (1. - tgt) * (1. - alpha)
    pt = torch.where(tgt == 1, pred, 1 - pred)
    return (a * (1. - pt) ** gamma * ce).sum()


# ----------------------------------------------------------------------------- criteria
def _assign(priors_cxcy, boxes, labels, threshold, anchors_xy=None, binary=False):
    pxy = M.cxcy_to_xy(priors_cxcy.numpy()) if anchors_xy is None else None
    objs, clss, negs = [], [], []
    for i in range(len(boxes)):
        an = pxy if anchors_xy is None else anchors_xy[i]
        obj, _, cls, neg = M.match_criterion(boxes[i].numpy(), labels[i].numpy(), an, threshold,
                                             binary=binary)
        objs.append(obj)
        clss.append(cls)
        negs.append(neg)
    return np.stack(objs), torch.from_numpy(np.stack(clss)), torch.from_numpy(np.stack(negs))


def _decode_t(locs, priors):
    c = torch.cat([locs[:, :2] * priors[:, 2:] / 10 + priors[:, :2],
                   torch.exp(locs[:, 2:] / 5) * priors[:, 2:]], 1)
    return torch.cat([c[:, :2] - c[:, 2:] / 2, c[:, :2] + c[:, 2:] / 2], 1)


def _encode_t(xy, priors):
    c = torch.cat([(xy[:, 2:] + xy[:, :2]) / 2, xy[:, 2:] - xy[:, :2]], 1)
    return torch.cat([(c[:, :2] - priors[:, :2]) / (priors[:, 2:] / 10),
                      torch.log(c[:, 2:] / priors[:, 2:]) * 5], 1)


def _hnm_sum(ce, pool_mask, n_hard):
    """Σ of the top-n_hard[b] entries of ce[b] restricted to pool (others count as 0)."""
    vals = torch.where(pool_mask, ce, torch.zeros_like(ce))
    tot = ce.new_zeros(())
    for b in range(ce.shape[0]):
        k = int(n_hard[b])
        if k > 0:
            tot = tot + torch.topk(vals[b], min(k, vals.shape[1])).values.sum()
    return tot


def local_npos(priors_cxcy, boxes, labels, threshold=0.5):
    """Positives of this (shard of the) batch — the quantity data parallelism all-reduces."""
    _, cls, _ = _assign(priors_cxcy, boxes, labels, threshold)
    return int((cls > 0).sum())


def ssd300_pool(priors_cxcy, scores, boxes, labels, threshold=0.5):
    """MultiBoxLoss300's mining pool of this (shard of the) batch, flattened [B*P]: the CE of
    negative priors (SSD300.py:571-580), -1 elsewhere — what data-parallel ranks exchange."""
    B, P, C = scores.shape
    _, cls, neg = _assign(priors_cxcy, boxes, labels, threshold)
    ce = F.cross_entropy(scores.detach().reshape(-1, C), cls.reshape(-1), reduction='none')
    return torch.where(torch.as_tensor(neg == -1).reshape(-1), ce, torch.full_like(ce, -1.0))


def criterion(kind, priors_cxcy, locs, scores, boxes, labels, reg_loss, cls_loss,
              threshold=0.5, neg_pos_ratio=3, reg_weights=1.0, npos_total=None, pool_all=None,
              local_off=0):
    """kind: 'ssd512' (``models/SSD512.py:508-626``), 'ssd300' (``SSD300.py:477-594``),
    'retina' (``RetinaNet.py:385-506``).  ``locs``/``scores`` are autograd leaves.
    ``npos_total`` overrides the batch positive count in every normaliser (a data-parallel shard
    normalised by the global count; summing shard losses gives the full-batch loss).
    ``pool_all``/``local_off`` (ssd300 CE, data-parallel): every rank's ``ssd300_pool``
    concatenated rank-major and this shard's offset in it — the hard negatives are the global
    top ratio*npos_total (ties: lowest global index first), summed over this shard's rows."""
    B, P, C = scores.shape
    obj, cls, neg = _assign(priors_cxcy, boxes, labels, threshold)
    pos = cls > 0
    negm = neg == -1
    n_pos = pos.sum(1)
    n_tot = n_pos.sum().float() if npos_total is None else torch.tensor(float(npos_total))
    if reg_loss.upper() == 'DIOU':
        dec = torch.stack([_decode_t(locs[b], priors_cxcy) for b in range(B)])
        tl = torch.stack([boxes[b][torch.from_numpy(obj[b])] for b in range(B)])
        loc_loss = (1.0 - aligned_overlap('diou', dec[pos].view(-1, 4), tl[pos].view(-1, 4))).sum() / n_tot
    else:
        enc = torch.stack([_encode_t(boxes[b][torch.from_numpy(obj[b])], priors_cxcy) for b in range(B)])
        if kind == 'ssd300':
            loc_loss = (locs[pos].view(-1, 4) - enc[pos].view(-1, 4)).abs().sum() / (4 * n_tot)
        else:
            loc_loss = smooth_l1(locs[pos].view(-1, 4), enc[pos].view(-1, 4), reduction='sum') / n_tot
    if cls_loss.upper() == 'FOCAL':
        rows = torch.cat([scores[pos], scores[negm]], 0)
        tgt = torch.cat([cls[pos], cls[negm]], 0)
        conf = focal_softmax(rows.view(-1, C), tgt.view(-1))
        if kind == 'retina':
            conf = conf / n_tot
    else:
        ce = F.cross_entropy(scores.view(-1, C), cls.view(-1), reduction='none').view(B, P)
        n_hard = neg_pos_ratio * n_pos
        if kind == 'ssd300' and pool_all is not None:
            k = neg_pos_ratio * int(n_tot)
            vals = pool_all.detach().cpu().numpy()
            order = np.argsort(-vals, kind='stable')              # value desc, index asc on ties
            sel = order[vals[order] >= 0][:k]
            mine = sel[(sel >= local_off) & (sel < local_off + B * P)] - local_off
            hard = ce.reshape(-1)[torch.from_numpy(mine)].sum()
        elif kind == 'ssd300':
            negs = ce[negm]
            k = int(n_hard.sum())
            hard = torch.topk(negs, min(k, negs.numel())).values.sum() if k > 0 else ce.new_zeros(())
        elif kind == 'retina':
            hard = _hnm_sum(ce, negm, n_hard)
        else:
            hard = _hnm_sum(ce, ~pos, n_hard)
        conf = (hard + ce[pos].sum()) / n_tot
    return conf + reg_weights * loc_loss


def refinedet(priors_cxcy, arm_locs, arm_scores, odm_locs, odm_scores, boxes, labels,
              threshold=0.5, neg_pos_ratio=3, theta=0.01, reg_weights=1.0):
    """``models/RefineDet512.py:730-956`` (ARM binary loss + ODM loss on detached ARM)."""
    B, P, _ = arm_locs.shape
    # ARM
    obj, cls, _ = _assign(priors_cxcy, boxes, labels, threshold, binary=True)
    pos = cls > 0
    n_pos = pos.sum(1)
    enc = torch.stack([_encode_t(boxes[b][torch.from_numpy(obj[b])], priors_cxcy) for b in range(B)])
    loc = smooth_l1(arm_locs[pos].view(-1, 4), enc[pos].view(-1, 4))
    ce = F.cross_entropy(arm_scores.view(-1, 2), cls.view(-1), reduction='none').view(B, P)
    hard = _hnm_sum(ce, ~pos, neg_pos_ratio * n_pos)
    arm = (hard + ce[pos].sum()) / n_pos.sum().float() + reg_weights * loc
    # ODM
    al = arm_locs.detach()
    dec = [_decode_t(al[b], priors_cxcy) for b in range(B)]
    obj, cls, _ = _assign(None, boxes, labels, threshold, anchors_xy=[d.numpy() for d in dec])
    easy = F.softmax(arm_scores.detach(), dim=2)[:, :, 1] < theta
    pos = (cls > 0) & ~easy
    n_pos = pos.sum(1)
    enc = torch.stack([_encode_t(boxes[b][torch.from_numpy(obj[b])],
                                 torch.cat([(dec[b][:, 2:] + dec[b][:, :2]) / 2, dec[b][:, 2:] - dec[b][:, :2]], 1))
                       for b in range(B)])
    loc = smooth_l1(odm_locs[pos].view(-1, 4), enc[pos].view(-1, 4))
    C = odm_scores.shape[2]
    ce = F.cross_entropy(odm_scores.view(-1, C), cls.view(-1), reduction='none').view(B, P)
    hard = _hnm_sum(ce, ~pos & ~easy, neg_pos_ratio * n_pos)
    odm = (hard + ce[pos].sum()) / n_pos.sum().float() + reg_weights * loc
    return arm + odm
