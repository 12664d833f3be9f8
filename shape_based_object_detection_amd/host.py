"""Host (CPU-tensor) path of the box utilities that the reference also calls OUTSIDE the training
step: DataLoader worker processes run ``random_crop``, which calls ``find_jaccard_overlap`` on CPU
tensors (dataset/transforms.py:175-176), and the box codecs are used on CPU data the same way.
SURVEY §8(b): the drop-in must keep a CPU path for them.

This is product code, not the test oracle: plain torch-CPU element-wise arithmetic written for
broadcasting ([k,1] x [1,n] operands instead of expanded copies), in the reference's evaluation
order so every element rounds exactly as the reference's CPU path does.  Device tensors never
come here — they go to the HIP kernels (csrc/match.hip, csrc/codec.hip) and there is no silent
fallback between the two: the caller's tensor device picks the path.
"""
import torch

EPS = 1e-5   # metrics.py:233


def _zero_neg(x):
    """``x[x < 0] = 0`` (keeps -0.0 and NaN exactly as the masked assignment does)."""
    return torch.where(x < 0, torch.zeros((), dtype=x.dtype), x)


def find_jaccard_overlap(gt_boxes, anchors):
    """[k, n] IoU of metrics.py:208-252: +1e-5 in the denominator, zero-size GT -> 0, anchors with
    w < 1e-5 and h < 1e-5 -> -1 (applied last)."""
    g = gt_boxes.reshape(-1, 1, 4)
    a = anchors.reshape(1, -1, 4)
    iw = _zero_neg(torch.minimum(g[..., 2], a[..., 2]) - torch.maximum(g[..., 0], a[..., 0]))
    ih = _zero_neg(torch.minimum(g[..., 3], a[..., 3]) - torch.maximum(g[..., 1], a[..., 1]))
    gx, gy = g[..., 2] - g[..., 0], g[..., 3] - g[..., 1]          # [k, 1]
    ax, ay = a[..., 2] - a[..., 0], a[..., 3] - a[..., 1]          # [1, n]
    inner = iw * ih
    ov = inner / (gx * gy + ax * ay - inner + EPS)
    ov = ov.masked_fill((gx.abs() < EPS) & (gy.abs() < EPS), 0)
    return ov.masked_fill((ax < EPS) & (ay < EPS), -1)


def intersect(box_a, box_b):
    """[A, B] intersection areas (metrics.py:186-205 / iou_utils.py:192-212)."""
    a = box_a.reshape(-1, 1, 4)
    b = box_b.reshape(1, -1, 4)
    w = torch.clamp(torch.minimum(a[..., 2], b[..., 2]) - torch.maximum(a[..., 0], b[..., 0]), min=0)
    h = torch.clamp(torch.minimum(a[..., 3], b[..., 3]) - torch.maximum(a[..., 1], b[..., 1]), min=0)
    return w * h


def jaccard(box_a, box_b):
    """[A, B] plain IoU, no EPS and no masks (iou_utils.py:215-233)."""
    inter = intersect(box_a, box_b)
    area_a = ((box_a[:, 2] - box_a[:, 0]) * (box_a[:, 3] - box_a[:, 1]))[:, None]
    area_b = ((box_b[:, 2] - box_b[:, 0]) * (box_b[:, 3] - box_b[:, 1]))[None, :]
    return inter / (area_a + area_b - inter)


def _pairs(x):
    return x[..., :2], x[..., 2:]


def xy_to_cxcy(xy):
    lo, hi = _pairs(xy)
    return torch.cat([(hi + lo) / 2, hi - lo], -1)


def cxcy_to_xy(cxcy):
    c, wh = _pairs(cxcy)
    half = wh / 2
    return torch.cat([c - half, c + half], -1)


def cxcy_to_gcxgcy(cxcy, priors_cxcy):
    c, wh = _pairs(cxcy)
    pc, pwh = _pairs(priors_cxcy)
    return torch.cat([(c - pc) / (pwh / 10), torch.log(wh / pwh) * 5], -1)


def gcxgcy_to_cxcy(gcxgcy, priors_cxcy):
    g, gwh = _pairs(gcxgcy)
    pc, pwh = _pairs(priors_cxcy)
    return torch.cat([g * pwh / 10 + pc, torch.exp(gwh / 5) * pwh], -1)


def point_form(boxes):
    """iou_utils.py:167-177 (same arithmetic as cxcy_to_xy)."""
    return cxcy_to_xy(boxes)


def encode(matched, priors, variances):
    """iou_utils.py:324-345: centre offset / (v0 * prior wh), log(wh / prior wh) / v1."""
    lo, hi = _pairs(matched)
    pc, pwh = _pairs(priors)
    g_c = (lo + hi) / 2 - pc
    g_c = g_c / (variances[0] * pwh)
    g_wh = torch.log((hi - lo) / pwh) / variances[1]
    return torch.cat([g_c, g_wh], -1)


def decode(loc, priors, variances):
    """iou_utils.py:349-368: centre and size, then the in-place corner conversion."""
    l_c, l_wh = _pairs(loc)
    pc, pwh = _pairs(priors)
    c = pc + l_c * variances[0] * pwh
    wh = pwh * torch.exp(l_wh * variances[1])
    lo = c - wh / 2
    return torch.cat([lo, wh + lo], -1)
