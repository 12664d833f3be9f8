"""``metrics.py`` hot-path half on the HIP path: ``find_jaccard_overlap`` and ``intersect``.

``find_jaccard_overlap`` (metrics.py:208-252) is the IoU every criterion and the mAP use:
inner / (gt_area + anchor_area - inner + 1e-5), GT with |w|,|h| < 1e-5 -> 0, anchors with
w,h < 1e-5 -> -1 (applied last).  Bit-exact with the reference's CPU path.
``calculate_mAP`` (VOC 11-point AP bookkeeping) is outside the hot path.
"""
import torch

from . import _lib as L
from . import core


def _single(gt, anchors, mode, what):
    L.require_device(gt, anchors, what=what)
    g = gt.reshape(-1, 4).float().contiguous()
    a = anchors.reshape(-1, 4).float().contiguous()
    G, P = g.shape[0], a.shape[0]
    if G == 0 or P == 0:
        return torch.zeros(G, P, dtype=torch.float32, device=g.device)
    pack = core.GtPack(g, torch.zeros(G, dtype=torch.int64, device=g.device),
                       core._offsets_tensor([G], g.device), [G])
    return core.iou_pairwise(pack, a, mode=mode)[0]


def find_jaccard_overlap(gt_boxes, anchors):
    """[G, P] IoU of metrics.py:208-252."""
    return _single(gt_boxes, anchors, L.IOU_METRICS, 'find_jaccard_overlap')


def intersect(box_a, box_b):
    """[A, B] intersection areas (metrics.py:192-205)."""
    return _single(box_a, box_b, L.IOU_INTER, 'intersect')
