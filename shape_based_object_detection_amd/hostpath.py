"""Host (CPU-tensor) path of the criteria, the loss operators, NMS / detect, DeformConv2d and
calculate_mAP: what the reference runs when it picks ``device = 'cpu'`` (train_anchor.py:65-71,
eval.py:68-74) — BASELINE config C1 is exactly that, one SSD300 step on the CPU.

Product code, not the test oracle (it imports nothing from ``oracle/``): plain torch-CPU
arithmetic in the reference's evaluation order, batched over images where the reference loops
(one [B, P] label / target pass, one box-loss pass, one class-loss pass), with autograd
providing the backward exactly as it does for the reference's own ops.  The matching block's
forced match keeps its per-object loop (last writer wins, FILTERED j — models/SSD512.py:546-553).
Device tensors never come here: each drop-in module picks this path only when its inputs are
CPU tensors, and raises on a mix (``metrics.on_host``); there is no fallback in either
direction.  NMS follows torchvision.ops.nms (descending score, ties by lower index, suppress
IoU > thr, union a_i + a_j - inter) for ``detect``, and iou_utils.nms / diounms for those names.
"""
import math

import torch
import torch.nn.functional as F

from . import host

# ----------------------------------------------------------------------------- aligned overlaps


def _aligned_parts(b1, b2):
    """Shared terms of iou_utils.py:6-164 for row-paired boxes (b1 / b2 already exchanged)."""
    w1, h1 = b1[:, 2] - b1[:, 0], b1[:, 3] - b1[:, 1]
    w2, h2 = b2[:, 2] - b2[:, 0], b2[:, 3] - b2[:, 1]
    inner = torch.clamp(torch.min(b1[:, 2:], b2[:, 2:]) - torch.max(b1[:, :2], b2[:, :2]), min=0)
    outer = torch.clamp(torch.max(b1[:, 2:], b2[:, 2:]) - torch.min(b1[:, :2], b2[:, :2]), min=0)
    ia = inner[:, 0] * inner[:, 1]
    union = w1 * h1 + w2 * h2 - ia
    return w1, h1, w2, h2, ia, union, outer


def _centre_dist(b1, b2, outer):
    dx = (b2[:, 2] + b2[:, 0]) / 2 - (b1[:, 2] + b1[:, 0]) / 2
    dy = (b2[:, 3] + b2[:, 1]) / 2 - (b1[:, 3] + b1[:, 1]) / 2
    return (dx ** 2 + dy ** 2) / ((outer[:, 0] ** 2) + (outer[:, 1] ** 2))


def aligned_overlap(kind, bboxes1, bboxes2):
    """Row-wise IoU / GIoU / DIoU / CIoU of iou_utils.py:6-164 (rows > cols exchange the sets,
    empty input -> a [rows, cols] zero matrix, as the reference returns)."""
    rows, cols = bboxes1.shape[0], bboxes2.shape[0]
    if rows * cols == 0:
        return torch.zeros((rows, cols))
    b1, b2 = (bboxes2, bboxes1) if rows > cols else (bboxes1, bboxes2)
    w1, h1, w2, h2, ia, union, outer = _aligned_parts(b1, b2)
    if kind == 'iou':
        return torch.clamp(ia / union, min=0, max=1.0)
    if kind == 'giou':
        closure = outer[:, 0] * outer[:, 1]
        return torch.clamp(ia / union - (closure - union) / closure, min=-1.0, max=1.0)
    u = _centre_dist(b1, b2, outer)
    if kind == 'diou':
        return torch.clamp(ia / union - u, min=-1.0, max=1.0)
    iou = ia / union
    with torch.no_grad():   # CIoU's trade-off term is a constant (iou_utils.py:86-91)
        atan_d = torch.atan(w2 / h2) - torch.atan(w1 / h1)
        v = (4 / (math.pi ** 2)) * torch.pow(atan_d, 2)
        alpha = v / ((1 - iou) + v)
        w_const = 2 * w1
    ar = (8 / (math.pi ** 2)) * atan_d * ((w1 - w_const) * h1)
    return torch.clamp(iou - (u + alpha * ar), min=-1.0, max=1.0)


# ----------------------------------------------------------------------------- loss operators
def focal_softmax(y_pred, y_true, alpha=0.25, gamma=2.0):
    """Loss.py:9-38, summed: one-hot from an identity matrix, softmax, alpha_bg = 1 - alpha on the
    background column, weight p_bg for background rows and 1 - p for foreground ones."""
    fore_alpha, back_alpha = (alpha[0], alpha[1]) if isinstance(alpha, (list, tuple)) else (alpha, 1 - alpha)
    onehot = torch.eye(y_pred.shape[-1])[y_true]
    p = F.softmax(y_pred, dim=1)
    bg_t, fg_t = onehot[:, :1], onehot[:, 1:]
    a = torch.cat([bg_t * back_alpha, fg_t * fore_alpha], dim=1)
    w = torch.cat([bg_t * p[:, :1], fg_t * (1 - p[:, 1:])], dim=1)
    return (a * (w ** gamma) * (-1 * torch.log(p))).sum()


def focal_sigmoid(out, target, alpha, gamma):
    """Loss.py:41-80: sigmoid focal over classes 1..C-1; rows with target 0 contribute nothing."""
    ids = torch.arange(1, out.shape[1], dtype=target.dtype).unsqueeze(0)
    t = target.unsqueeze(1)
    p = torch.sigmoid(out[:, 1:])
    term1 = (1 - p) ** gamma * torch.log(p)
    term2 = p ** gamma * torch.log(1 - p)
    return (-(t == ids).float() * alpha * term1 - ((t != ids) * (t > 0)).float() * (1 - alpha) * term2).sum()


def focal_bce(logits, targets, alpha, gamma):
    """Loss.py:83-103: BCE-with-logits focal over all one-hot columns, prediction clamped."""
    ids = torch.arange(0, logits.shape[1], dtype=targets.dtype).unsqueeze(0)
    tgt = (targets.unsqueeze(1) == ids).float()
    pred = logits.sigmoid().clamp(min=1e-4, max=1 - 1e-4)
    ce = F.binary_cross_entropy_with_logits(logits, tgt, reduction='none')
    a = tgt * alpha + (1. - tgt) * (1. - alpha)
    pt = torch.where(tgt == 1, pred, 1 - pred)
    return (a * (1. - pt) ** gamma * ce).sum()


def smooth_l1_elementwise(pred, target, beta):
    """Loss.py:213-217 element-wise."""
    x = (pred - target).abs()
    return torch.where(x >= beta, x - 0.5 * beta, 0.5 * x ** 2 / beta)


def _mean_rows(loss, rows):
    return loss.sum() / rows


# ----------------------------------------------------------------------------- matching
def match_image(boxes, labels, anchors_xy, threshold, binary=False):
    """The criteria's per-image matching block (models/SSD512.py:535-563; binary ARM labels
    RefineDet512.py:777-781): (object per prior, overlap per prior, class, negative-marked class)."""
    overlap = host.find_jaccard_overlap(boxes, anchors_xy)
    ovl, obj = overlap.max(dim=0)
    best_ovl, best_prior = overlap.max(dim=1)
    forced = best_prior[best_ovl > 0]
    if len(forced) > 0:
        ovl.index_fill_(0, forced, 1.0)
    for j in range(forced.size(0)):       # FILTERED j, last writer wins
        obj[forced[j]] = j
    lab = labels[obj]
    cls = lab.clone()
    cls[ovl < threshold] = 0
    if binary:
        cls = (cls > 0).long()
    neg = lab.clone()
    neg[ovl < threshold - 0.1] = -1
    return obj, ovl, cls, neg


def _match_batch(boxes, labels, anchors, threshold, binary=False):
    """[B, P] obj / cls / neg over the batch; ``anchors`` shared [P,4] or a per-image list."""
    objs, clss, negs = [], [], []
    for i in range(len(boxes)):
        an = anchors[i] if isinstance(anchors, (list, tuple)) else anchors
        obj, _, cls, neg = match_image(boxes[i], labels[i].long(), an, threshold, binary)
        objs.append(obj)
        clss.append(cls)
        negs.append(neg)
    return torch.stack(objs), torch.stack(clss), torch.stack(negs)


def _true_xy(boxes, obj):
    return torch.stack([boxes[i][obj[i]] for i in range(len(boxes))])


def _hard_negative_sum(ce, excluded, n_hard):
    """Per image: the n_hard[b] largest CE values outside ``excluded`` (which count as 0), by the
    reference's descending sort and rank mask (SSD512.py:610-619, RetinaNet.py:490-499)."""
    neg = ce.clone()
    neg[excluded] = 0.
    neg, _ = neg.sort(dim=1, descending=True)
    ranks = torch.arange(ce.shape[1]).unsqueeze(0).expand_as(neg)
    return neg[ranks < n_hard.unsqueeze(1)].sum()


def anchor_criterion(kind, priors_cxcy, priors_xy, locs, scores, boxes, labels, reg_loss, cls_loss,
                     threshold=0.5, neg_pos_ratio=3, reg_weight=1.0):
    """MultiBoxLoss512 (models/SSD512.py:508-626), MultiBoxLoss300 (SSD300.py:477-594) and
    RetinaFocalLoss (RetinaNet.py:385-506) on CPU tensors; returns the 0-d loss with autograd."""
    B, P, C = scores.shape
    obj, cls, neg = _match_batch(boxes, labels, priors_xy, threshold)
    pos = cls > 0
    negm = neg == -1
    n_pos = pos.sum(dim=1)
    txy = _true_xy(boxes, obj)
    if str(reg_loss).upper() == 'DIOU':
        dec = host.cxcy_to_xy(host.gcxgcy_to_cxcy(locs, priors_cxcy))
        d, t = dec[pos].view(-1, 4), txy[pos].view(-1, 4)
        loc_loss = _mean_rows(1.0 - aligned_overlap('diou', d, t), d.shape[0])
    else:
        enc = host.cxcy_to_gcxgcy(host.xy_to_cxcy(txy), priors_cxcy)
        lp, lt = locs[pos].view(-1, 4), enc[pos].view(-1, 4)
        if kind == 'ssd300':                                   # nn.L1Loss: mean over elements
            loc_loss = F.l1_loss(lp, lt)
        else:                                                  # SmoothL1Loss: sum / rows
            loc_loss = _mean_rows(smooth_l1_elementwise(lp, lt, 1.0 / 9.0), lp.shape[0])
    if str(cls_loss).upper() == 'FOCAL':
        rows = torch.cat([scores[pos], scores[negm]], dim=0)
        tgt = torch.cat([cls[pos], cls[negm]], dim=0)
        conf = focal_softmax(rows.view(-1, C), tgt.view(-1))
        if kind == 'retina':
            conf = conf / n_pos.sum().float()
    else:
        ce = F.cross_entropy(scores.view(-1, C), cls.view(-1), reduction='none').view(B, P)
        n_hard = neg_pos_ratio * n_pos
        if kind == 'ssd300':          # one pool over the batch's negatives (SSD300.py:580-588)
            pool, _ = ce[negm].sort(dim=-1, descending=True)
            hard = pool[:n_hard.sum().long()].sum()
        elif kind == 'retina':        # negatives only, per image
            hard = _hard_negative_sum(ce, ~negm, n_hard)
        else:                         # every non-positive, per image
            hard = _hard_negative_sum(ce, pos, n_hard)
        conf = (hard + ce[pos].sum()) / n_pos.sum().float()
    return conf + reg_weight * loc_loss


def refinedet_arm(priors_cxcy, priors_xy, arm_locs, arm_scores, boxes, labels, threshold=0.5,
                  neg_pos_ratio=3, reg_weight=1.0):
    """RefineDetLoss.compute_arm_loss (RefineDet512.py:730-820): binary labels, smooth-L1 vs the
    fixed priors, CE with per-image mining over the non-positives."""
    B, P, C = arm_scores.shape
    obj, cls, _ = _match_batch(boxes, labels, priors_xy, threshold, binary=True)
    pos = cls > 0
    n_pos = pos.sum(dim=1)
    enc = host.cxcy_to_gcxgcy(host.xy_to_cxcy(_true_xy(boxes, obj)), priors_cxcy)
    lp = arm_locs[pos].view(-1, 4)
    loc = _mean_rows(smooth_l1_elementwise(lp, enc[pos].view(-1, 4), 1.0 / 9.0), lp.shape[0])
    ce = F.cross_entropy(arm_scores.view(-1, C), cls.view(-1), reduction='none').view(B, P)
    conf = (_hard_negative_sum(ce, pos, neg_pos_ratio * n_pos) + ce[pos].sum()) / n_pos.sum().float()
    return conf + reg_weight * loc


def refinedet_odm(priors_cxcy, arm_locs, arm_scores, odm_locs, odm_scores, boxes, labels, threshold=0.5,
                  neg_pos_ratio=3, reg_weight=1.0, theta=0.01):
    """RefineDetLoss.compute_odm_loss (RefineDet512.py:822-939): matching against each image's
    decoded ARM boxes, targets encoded relative to them, easy negatives (softmax(ARM)[..., 1] <
    theta) removed from the positives and from the mining pool."""
    B, P, C = odm_scores.shape
    dec = host.cxcy_to_xy(host.gcxgcy_to_cxcy(arm_locs, priors_cxcy))
    obj, cls, _ = _match_batch(boxes, labels, list(dec), threshold)
    enc = host.cxcy_to_gcxgcy(host.xy_to_cxcy(_true_xy(boxes, obj)), host.xy_to_cxcy(dec))
    easy = F.softmax(arm_scores, dim=2)[:, :, 1] < theta
    pos = (cls > 0) & ~easy
    lp = odm_locs[pos].view(-1, 4)
    loc = _mean_rows(smooth_l1_elementwise(lp, enc[pos].view(-1, 4), 1.0 / 9.0), lp.shape[0])
    n_pos = pos.sum(dim=1)
    ce = F.cross_entropy(odm_scores.view(-1, C), cls.view(-1), reduction='none').view(B, P)
    conf = (_hard_negative_sum(ce, pos | easy, neg_pos_ratio * n_pos) + ce[pos].sum()) / n_pos.sum().float()
    return conf + reg_weight * loc


def match_ssd(threshold, truths, priors, variances, labels, loc_t, conf_t, idx, encode):
    """iou_utils.match / match_ious (:236-321) on CPU tensors: plain jaccard vs point_form(priors),
    each object's best prior filled with 2 (UNFILTERED j, last writer wins), conf = labels + 1,
    in place into loc_t[idx] / conf_t[idx]."""
    ov = host.jaccard(truths, host.point_form(priors))
    _, best_prior = ov.max(1)
    best_ovl, best_obj = ov.max(0)
    best_ovl.index_fill_(0, best_prior, 2)
    for j in range(best_prior.size(0)):
        best_obj[best_prior[j]] = j
    matches = truths[best_obj]
    conf = labels[best_obj] + 1
    conf[best_ovl < threshold] = 0
    loc_t[idx] = host.encode(matches, priors, variances) if encode else matches
    conf_t[idx] = conf


# ----------------------------------------------------------------------------- NMS
def _areas(b):
    return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])


def nms_tv(boxes, scores, thr):
    """torchvision.ops.nms semantics: kept indices in descending score order (ties: lower index
    first), a box suppressed by a kept one with IoU > thr, union a_i + a_j - inter."""
    order = torch.sort(scores, descending=True, stable=True)[1]
    b = boxes[order]
    area = _areas(b)
    alive = torch.ones(len(order), dtype=torch.bool)
    keep = []
    for i in range(len(order)):
        if not alive[i]:
            continue
        keep.append(i)
        rest = alive[i + 1:]
        if not rest.any():
            break
        r = b[i + 1:]
        w = torch.clamp(torch.minimum(b[i, 2], r[:, 2]) - torch.maximum(b[i, 0], r[:, 0]), min=0)
        h = torch.clamp(torch.minimum(b[i, 3], r[:, 3]) - torch.maximum(b[i, 1], r[:, 1]), min=0)
        inter = w * h
        rest &= ~(inter / (area[i] + area[i + 1:] - inter) > thr)
    return order[torch.tensor(keep, dtype=torch.long)]


def nms_ref(boxes, scores, overlap=0.5, top_k=200, diou=False, beta1=1.0):
    """iou_utils.nms / diounms (iou_utils.py:385-530): ascending sort, the top_k largest kept
    before suppression, pop the maximum, keep boxes with IoU <= overlap (union (a_j - inter) + a_i;
    DIoU: IoU - (d / c)^beta1 with the reference's centre_y2 quirk).  Returns (keep, count); the
    bare zero ``keep`` for empty input."""
    keep = scores.new_zeros(scores.size(0), dtype=torch.long)
    if boxes.numel() == 0:
        return keep
    x1, y1, x2, y2 = boxes[:, 0], boxes[:, 1], boxes[:, 2], boxes[:, 3]
    area = torch.mul(x2 - x1, y2 - y1)
    _, idx = scores.sort(0)
    idx = idx[-top_k:]
    count = 0
    while idx.numel() > 0:
        i = idx[-1]
        keep[count] = i
        count += 1
        if idx.size(0) == 1:
            break
        idx = idx[:-1]
        cx1, cy1 = torch.index_select(x1, 0, idx), torch.index_select(y1, 0, idx)
        cx2, cy2 = torch.index_select(x2, 0, idx), torch.index_select(y2, 0, idx)
        w = torch.clamp(torch.clamp(cx2, max=x2[i]) - torch.clamp(cx1, min=x1[i]), min=0.0)
        h = torch.clamp(torch.clamp(cy2, max=y2[i]) - torch.clamp(cy1, min=y1[i]), min=0.0)
        inter = w * h
        rem = torch.index_select(area, 0, idx)
        iou = inter / ((rem - inter) + area[i])
        if diou:
            # centre distance over the enclosing diagonal; the candidate's centre y is
            # (y2 + y2) / 2 in the reference (iou_utils.py:507)
            d = ((x1[i] + x2[i]) / 2 - (cx1 + cx2) / 2) ** 2 + ((y1[i] + y2[i]) / 2 - (cy2 + cy2) / 2) ** 2
            c = ((torch.clamp(cx2, min=x2[i]) - torch.clamp(cx1, max=x1[i])) ** 2 +
                 (torch.clamp(cy2, min=y2[i]) - torch.clamp(cy1, max=y1[i])) ** 2)
            iou = iou - (d / c) ** beta1
        idx = idx[iou.le(overlap)]
    return keep, count


# ----------------------------------------------------------------------------- detect
def detect(locs, scores, min_score, max_overlap, top_k, priors_cxcy, box_type='offset', act='softmax',
           pos_mask=None, final_nms=None):
    """models/utils.py:181-297 (final_nms None) and detect_tools.detect / detect_refine
    (final_nms 0.7, :202-205 / :324-327) on CPU tensors: lists of per-image boxes, labels, scores."""
    B, P, C = scores.shape
    probs = scores.sigmoid() if act == 'sigmoid' else scores.softmax(dim=2)
    out_b, out_l, out_s = [], [], []
    for i in range(B):
        if box_type == 'offset':
            dec = host.cxcy_to_xy(host.gcxgcy_to_cxcy(locs[i], priors_cxcy)).clamp_(0, 1)
        elif box_type == 'center':
            dec = host.cxcy_to_xy(locs[i]).clamp_(0, 1)
        else:
            dec = locs[i].clamp_(0, 1)                      # the caller's tensor, in place (:224)
        cs, db = probs[i], dec
        if pos_mask is not None:
            sel = pos_mask[i].nonzero().squeeze(-1)
            cs, db = cs.index_select(0, sel), db.index_select(0, sel)
        bx, lb, sc = [], [], []
        for c in range(1, C):
            s = cs[:, c]
            above = torch.nonzero(s > min_score).squeeze(1)
            if above.numel() == 0:
                continue
            s, b = s.index_select(0, above), db.index_select(0, above)
            k = nms_tv(b, s, max_overlap)
            bx.append(b[k])
            lb.append(torch.full((k.numel(),), c, dtype=torch.long))
            sc.append(s[k])
        if not bx:
            bx, lb, sc = [torch.tensor([[0., 0., 1., 1.]])], [torch.tensor([0])], [torch.tensor([0.])]
        bx, lb, sc = torch.cat(bx), torch.cat(lb), torch.cat(sc)
        n = sc.numel()
        if final_nms is not None:
            k = nms_tv(bx, sc, final_nms)
            bx, lb, sc = bx[k], lb[k], sc[k]
        if n > top_k:
            sc, order = sc.sort(dim=0, descending=True, stable=True)
            sc, bx, lb = sc[:top_k], bx[order][:top_k], lb[order][:top_k]
        out_b.append(bx)
        out_l.append(lb)
        out_s.append(sc)
    return out_b, out_l, out_s


# ----------------------------------------------------------------------------- DeformConv2d
def deform_conv2d(x, offset, mask_logits, weight, ks=3, padding=1, stride=1):
    """Deformable_convolution.py:33-91 on CPU tensors (autograd gives the backward): sampling
    points p = (1 + stride*h + i - 1 + d_row, 1 + stride*w + j - 1 + d_col) in the zero-padded map,
    corners from floor(p) clamped to the map, p itself clamped, bilinear weights, sigmoid
    modulation, then the k x k contraction with the kernel point n = i*k + j."""
    B, C, H, W = x.shape
    N = ks * ks
    Ho, Wo = offset.shape[2], offset.shape[3]
    xp = F.pad(x, (padding, padding, padding, padding)) if padding else x
    Hp, Wp = xp.shape[2], xp.shape[3]
    r = torch.arange(-(ks - 1) // 2, (ks - 1) // 2 + 1)
    pn_r = r.view(ks, 1).expand(ks, ks).reshape(N).to(x.dtype)
    pn_c = r.view(1, ks).expand(ks, ks).reshape(N).to(x.dtype)
    p0_r = torch.arange(1, Ho * stride + 1, stride).to(x.dtype).view(Ho, 1, 1)
    p0_c = torch.arange(1, Wo * stride + 1, stride).to(x.dtype).view(1, Wo, 1)
    off = offset.permute(0, 2, 3, 1)                          # [B, Ho, Wo, 2N]
    pr = p0_r + pn_r + off[..., :N]
    pc = p0_c + pn_c + off[..., N:]
    fr, fc = pr.detach().floor(), pc.detach().floor()
    r0, r1 = fr.clamp(0, Hp - 1), (fr + 1).clamp(0, Hp - 1)
    c0, c1 = fc.clamp(0, Wp - 1), (fc + 1).clamp(0, Wp - 1)
    pr, pc = pr.clamp(0, Hp - 1), pc.clamp(0, Wp - 1)
    flat = xp.reshape(B, C, Hp * Wp)

    def corner(rr, cc):
        idx = (rr.long() * Wp + cc.long()).reshape(B, 1, -1).expand(B, C, -1)
        return flat.gather(2, idx).view(B, C, Ho, Wo, N)

    w_lt = (1 + (r0 - pr)) * (1 + (c0 - pc))
    w_rb = (1 - (r1 - pr)) * (1 - (c1 - pc))
    w_lb = (1 + (r0 - pr)) * (1 - (c1 - pc))
    w_rt = (1 - (r1 - pr)) * (1 + (c0 - pc))
    cols = (w_lt.unsqueeze(1) * corner(r0, c0) + w_rb.unsqueeze(1) * corner(r1, c1) +
            w_lb.unsqueeze(1) * corner(r0, c1) + w_rt.unsqueeze(1) * corner(r1, c0))
    if mask_logits is not None:
        cols = cols * torch.sigmoid(mask_logits).permute(0, 2, 3, 1).unsqueeze(1)
    return torch.einsum('ocn,bchwn->bohw', weight.reshape(weight.shape[0], C, N), cols)


# ----------------------------------------------------------------------------- mAP
def calculate_mAP(det_boxes, det_labels, det_scores, true_boxes, true_labels, true_difficulties, threshold,
                  n_classes):
    """metrics.py:8-145 on CPU tensors: per class, detections in descending score order (stable)
    matched greedily to the same image's not-yet-detected objects (IoU > threshold; difficult
    objects ignored), cumulative precision / recall, VOC 11-point AP.  Returns ([AP per class
    1..C-1], mAP)."""
    t_img = torch.cat([torch.full((t.shape[0],), i, dtype=torch.long) for i, t in enumerate(true_labels)])
    d_img = torch.cat([torch.full((t.shape[0],), i, dtype=torch.long) for i, t in enumerate(det_labels)])
    tb, tl, td = torch.cat(true_boxes), torch.cat(true_labels), torch.cat(true_difficulties)
    db, dl, ds = torch.cat(det_boxes), torch.cat(det_labels), torch.cat(det_scores)
    aps = torch.zeros(n_classes - 1, dtype=torch.float)
    rthr = torch.arange(start=0, end=1.1, step=.1)
    for c in range(1, n_classes):
        tsel = tl == c
        ci, cb, cd = t_img[tsel], tb[tsel], td[tsel]
        n_easy = (1 - cd).sum().item()
        seen = torch.zeros(cd.shape[0], dtype=torch.uint8)
        dsel = dl == c
        if int(dsel.sum()) == 0:
            continue
        sc, order = torch.sort(ds[dsel], dim=0, descending=True, stable=True)
        di, dbx = d_img[dsel][order], db[dsel][order]
        tp = torch.zeros(sc.shape[0])
        fp = torch.zeros(sc.shape[0])
        for d in range(sc.shape[0]):
            in_img = torch.nonzero(ci == di[d]).squeeze(1)
            if in_img.numel() == 0:
                fp[d] = 1
                continue
            ov = host.find_jaccard_overlap(dbx[d].unsqueeze(0), cb[in_img])
            best, k = torch.max(ov.squeeze(0), dim=0)
            obj = in_img[k]
            if best.item() > threshold:
                if cd[obj] == 0:
                    if seen[obj] == 0:
                        tp[d] = 1
                        seen[obj] = 1
                    else:
                        fp[d] = 1
            else:
                fp[d] = 1
        ctp, cfp = torch.cumsum(tp, dim=0), torch.cumsum(fp, dim=0)
        prec = ctp / (ctp + cfp + 1e-10)
        rec = ctp / n_easy
        pr = torch.zeros(rthr.shape[0])
        for i, t in enumerate(rthr.tolist()):
            above = rec >= t
            pr[i] = prec[above].max() if above.any() else 0.
        aps[c - 1] = pr.mean()
    return aps.tolist(), aps.mean().item()
