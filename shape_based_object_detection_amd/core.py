"""Host-side orchestration of the HIP hot path (device memory, workspaces, ragged GT packing).

Everything here runs on ROCm device tensors; inputs on the CPU are rejected.  No call in this
module synchronises with the host unless its docstring says so.
"""
import torch

from . import _lib as L


class GtPack:
    """Ragged ground truth packed once per step (dataset/Datasets.py:58-86 list-of-tensors).

    boxes [sum G, 4] f32 xyxy, labels [sum G] int64, offsets [B+1] int32 on the device;
    ``counts`` / ``gmax`` are host ints (taken from tensor shapes: no device sync)."""

    __slots__ = ('boxes', 'labels', 'offsets', 'counts', 'gmax', 'batch')

    def __init__(self, boxes, labels, offsets, counts):
        self.boxes, self.labels, self.offsets, self.counts = boxes, labels, offsets, counts
        self.gmax = max(counts) if counts else 0
        self.batch = len(counts)


_OFFSET_CACHE = {}


def _offsets_tensor(counts, device):
    key = (tuple(counts), str(device))
    t = _OFFSET_CACHE.get(key)
    if t is None:
        offs = [0]
        for c in counts:
            offs.append(offs[-1] + c)
        t = torch.tensor(offs, dtype=torch.int32).pin_memory().to(device, non_blocking=True)
        if len(_OFFSET_CACHE) > 256:
            _OFFSET_CACHE.clear()
        _OFFSET_CACHE[key] = t
    return t


def pack_gt(boxes, labels, device=None, allow_empty=False):
    """Pack per-image lists into a GtPack.  An image with no objects raises like the reference
    does (``overlap.max(dim=0)`` of an empty matrix, models/SSD512.py:538)."""
    if len(boxes) != len(labels):
        raise ValueError('boxes and labels must have the same length')
    counts = [int(b.shape[0]) for b in boxes]
    if not allow_empty and any(c == 0 for c in counts):
        raise RuntimeError('max(): Expected reduction dim 0 to have non-zero size (an image has no '
                           'ground-truth objects, as in the reference criterion)')
    device = device or boxes[0].device
    L.require_device(*boxes, *labels, what='pack_gt')
    gb = torch.cat([b.reshape(-1, 4) for b in boxes]).to(torch.float32).contiguous()
    gl = torch.cat([l.reshape(-1) for l in labels]).to(torch.int64).contiguous()
    return GtPack(gb, gl, _offsets_tensor(counts, device), counts)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def iou_pairwise(gt, anchors, mode=L.IOU_METRICS, anchor_batch_stride=0):
    """out [B, Gmax, P] (rows beyond each image's G are zero)."""
    a = anchors.contiguous()
    P = a.shape[-2]
    out = torch.zeros(gt.batch, gt.gmax, P, dtype=torch.float32, device=a.device)
    L.call('sbod_iou_pairwise_f32', L.ptr(gt.boxes), L.ptr(gt.offsets), gt.batch, gt.gmax,
           L.ptr(a), anchor_batch_stride, P, mode, L.ptr(out), L.stream_of(a))
    return out


def match(gt, anchors, P, threshold=0.5, flags=0, priors_cxcy=None, arm_scores=None, theta=0.01):
    """The criteria's matching block.  Returns (obj [B,P] int32, ovl [B,P] f32, n_pos [B+1] int32).

    ``anchors`` is priors_xy [P,4] (shared) or, with ``flags & MATCH_ODM``, the ARM locs [B,P,4]."""
    dev = anchors.device
    B = gt.batch
    obj = torch.empty(B, P, dtype=torch.int32, device=dev)
    ovl = torch.empty(B, P, dtype=torch.float32, device=dev)
    npos = torch.empty(B + 1, dtype=torch.int32, device=dev)
    nb = L.lib().sbod_match_workspace_bytes(B, gt.gmax)
    ws = workspace(nb, dev)
    L.call('sbod_match_f32', L.ptr(gt.boxes), L.ptr(gt.labels), L.ptr(gt.offsets), B, gt.gmax,
           L.ptr(anchors.contiguous()), L.ptr(priors_cxcy), L.ptr(arm_scores), P, float(threshold),
           float(theta), int(flags), L.ptr(obj), L.ptr(ovl), L.ptr(npos), L.ptr(ws), nb,
           L.stream_of(anchors))
    return obj, ovl, npos


def match_expand(gt, obj, ovl, priors_cxcy=None, threshold=0.5, neg_threshold=0.4, flags=0,
                 arm_locs=None, want=('cls', 'neg', 'true_xy', 'enc')):
    """The reference's per-prior tensors from matcher outputs (true_classes, true_neg_classes,
    true_locs, true_locs_encoded)."""
    B, P = obj.shape
    dev = obj.device
    cls = torch.empty(B, P, dtype=torch.int64, device=dev) if 'cls' in want else None
    neg = torch.empty(B, P, dtype=torch.int64, device=dev) if 'neg' in want else None
    txy = torch.empty(B, P, 4, dtype=torch.float32, device=dev) if 'true_xy' in want else None
    enc = torch.empty(B, P, 4, dtype=torch.float32, device=dev) if 'enc' in want else None
    L.call('sbod_match_expand_f32', L.ptr(gt.boxes), L.ptr(gt.labels), L.ptr(gt.offsets), B,
           L.ptr(obj), L.ptr(ovl), L.ptr(priors_cxcy), L.ptr(arm_locs), P, float(threshold),
           float(neg_threshold), int(flags), L.ptr(cls), L.ptr(neg), L.ptr(txy), L.ptr(enc),
           L.stream_of(obj))
    return cls, neg, txy, enc


def codec(op, x, priors=None, var=(0.1, 0.2), out=None):
    """Row-wise box codec on [n,4] (priors broadcast over leading dims when smaller)."""
    x = x.contiguous()
    n = x.numel() // 4
    prow = 0
    if priors is not None:
        priors = priors.contiguous()
        pr = priors.numel() // 4
        prow = pr if pr != n else 0
    out = torch.empty_like(x) if out is None else out
    L.call('sbod_codec_f32', L.CODEC[op], L.ptr(x), L.ptr(priors), n, prow, float(var[0]),
           float(var[1]), L.ptr(out), L.stream_of(x))
    return out
