"""``operators/iou_utils.py`` on the HIP path — same names, arguments and return conventions.

  * ``bbox_overlaps_{iou,giou,diou,ciou}`` (:6-164): row-wise overlaps with autograd w.r.t.
    the first box set; the reference's row/col exchange (:13-16) and empty-input zeros (:9-11).
  * ``point_form`` (:167-177), ``center_size`` (:180-189, raises TypeError as the reference does),
    ``intersect`` / ``jaccard`` (:192-233), ``match`` / ``match_ious`` (:236-321, in place into
    ``loc_t[idx]`` / ``conf_t[idx]``), ``encode`` / ``decode`` (:324-368), ``log_sum_exp`` (:371-379),
    ``nms`` / ``diounms`` (:385-530: (keep, count), or the bare zero ``keep`` for empty input).
Device tensors run the HIP kernels.  CPU tensors run the host path (``host.py`` for the box
utilities, ``hostpath.py`` for the overlaps, match and NMS): the reference's own CPU arithmetic.
"""
import torch

from .. import _lib as L
from .. import core
from .. import host
from .. import hostpath
from .. import metrics as _metrics
from ..metrics import on_host


def _overlaps(kind, bboxes1, bboxes2):
    if on_host(bboxes1, bboxes2):
        return hostpath.aligned_overlap(kind, bboxes1, bboxes2)
    rows, cols = bboxes1.shape[0], bboxes2.shape[0]
    if rows * cols == 0:
        return torch.zeros((rows, cols), device=bboxes1.device)
    exchange = rows > cols
    if exchange:
        bboxes1, bboxes2 = bboxes2, bboxes1
    if bboxes1.shape[0] != bboxes2.shape[0]:
        bboxes1, bboxes2 = torch.broadcast_tensors(bboxes1, bboxes2)
    return core.aligned_overlap(kind, bboxes1, bboxes2)


def bbox_overlaps_diou(bboxes1, bboxes2):
    return _overlaps('diou', bboxes1, bboxes2)


def bbox_overlaps_ciou(bboxes1, bboxes2):
    return _overlaps('ciou', bboxes1, bboxes2)


def bbox_overlaps_iou(bboxes1, bboxes2):
    return _overlaps('iou', bboxes1, bboxes2)


def bbox_overlaps_giou(bboxes1, bboxes2):
    return _overlaps('giou', bboxes1, bboxes2)


def point_form(boxes):
    """(cx, cy, w, h) -> (xmin, ymin, xmax, ymax)."""
    if on_host(boxes):
        return host.point_form(boxes)
    L.require_device(boxes, what='point_form')
    return core.codec('cxcy_to_xy', boxes.float())


def center_size(boxes):
    """The reference's ``center_size`` passes three positional tensors to ``torch.cat``
    (iou_utils.py:188-189) and always raises; kept identical."""
    raise TypeError('cat() received an invalid combination of arguments '
                    '[operators/iou_utils.py:188 center_size is broken in the reference]')


def intersect(box_a, box_b):
    """[A, B] intersection areas."""
    return _metrics.intersect(box_a, box_b)


def jaccard(box_a, box_b):
    """[A, B] plain IoU (no EPS, no degenerate masks)."""
    if on_host(box_a, box_b):
        return host.jaccard(box_a, box_b)
    return _metrics._single(box_a, box_b, L.IOU_PLAIN, 'jaccard')


def _match(threshold, truths, priors, variances, labels, loc_t, conf_t, idx, encode):
    if on_host(truths, priors, labels, loc_t, conf_t):
        return hostpath.match_ssd(threshold, truths, priors, variances, labels, loc_t, conf_t, idx, encode)
    L.require_device(truths, priors, labels, loc_t, conf_t, what='match')
    if not (loc_t.is_contiguous() and conf_t.is_contiguous() and loc_t.dtype == torch.float32
            and conf_t.dtype == torch.int64):
        raise TypeError('match: loc_t must be contiguous float32 and conf_t contiguous int64')
    tr = truths.float().contiguous()
    lb = labels.to(torch.int64).contiguous()
    pri = priors.float().contiguous()
    G, P = tr.shape[0], pri.shape[0]
    nb = L.lib().sbod_match_ssd_workspace_bytes(G, P)
    ws = core.workspace(nb, tr.device, 'match_ssd')
    L.call('sbod_match_ssd_f32', L.ptr(tr), L.ptr(lb), G, L.ptr(pri), P, float(threshold),
           float(variances[0]), float(variances[1]), int(encode), L.ptr(loc_t[idx]),
           L.ptr(conf_t[idx]), L.ptr(ws), nb, L.stream_of(tr))


def match_ious(threshold, truths, priors, variances, labels, loc_t, conf_t, idx):
    """Writes the raw matched truths into loc_t[idx] and labels+1 / 0 into conf_t[idx]."""
    _match(threshold, truths, priors, variances, labels, loc_t, conf_t, idx, encode=False)


def match(threshold, truths, priors, variances, labels, loc_t, conf_t, idx):
    """Writes encode(matches, priors, variances) into loc_t[idx] and labels+1 / 0 into conf_t[idx]."""
    _match(threshold, truths, priors, variances, labels, loc_t, conf_t, idx, encode=True)


def encode(matched, priors, variances):
    if on_host(matched, priors):
        return host.encode(matched, priors, variances)
    L.require_device(matched, priors, what='encode')
    return core.codec('encode_var', matched.float(), priors.float(), var=variances)


def decode(loc, priors, variances):
    if on_host(loc, priors):
        return host.decode(loc, priors, variances)
    L.require_device(loc, priors, what='decode')
    return core.codec('decode_var', loc.float(), priors.float(), var=variances)


def log_sum_exp(x):
    """log(sum(exp(x - max), 1)) + max with the GLOBAL max (iou_utils.py:371-379): element-wise
    torch arithmetic on either device."""
    x_max = x.data.max()
    return torch.log(torch.sum(torch.exp(x - x_max), 1, keepdim=True)) + x_max


def _nms(variant, boxes, scores, overlap, top_k, beta1=1.0):
    if on_host(boxes, scores):
        return hostpath.nms_ref(boxes, scores, overlap, top_k, diou=variant == 'diou', beta1=beta1)
    L.require_device(boxes, scores, what=variant)
    if boxes.numel() == 0:
        return scores.new_zeros(scores.size(0), dtype=torch.long)
    keep, count = core.nms(boxes, scores, overlap, top_k=top_k, variant=variant, beta1=beta1)
    return keep, int(count.item())


def nms(boxes, scores, overlap=0.5, top_k=200):
    """Greedy NMS over the top_k highest scores; keep iff IoU <= overlap.  Returns (keep, count)."""
    return _nms('ref', boxes, scores, overlap, top_k)


def diounms(boxes, scores, overlap=0.5, top_k=200, beta1=1.0):
    """DIoU-NMS (iou_utils.py:453-530), including its center_y2 quirk."""
    return _nms('diou', boxes, scores, overlap, top_k, beta1)
