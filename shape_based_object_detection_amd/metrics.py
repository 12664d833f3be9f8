"""``metrics.py`` hot-path half on the HIP path: ``find_jaccard_overlap`` and ``intersect``.

``find_jaccard_overlap`` (metrics.py:208-252) is the IoU every criterion and the mAP use:
inner / (gt_area + anchor_area - inner + 1e-5), GT with |w|,|h| < 1e-5 -> 0, anchors with
w,h < 1e-5 -> -1 (applied last).  Bit-exact with the reference's CPU path.  Device tensors run
the HIP kernel; CPU tensors (DataLoader workers: random_crop, dataset/transforms.py:175-176) run
the host path in ``host.py``.
``calculate_mAP`` (metrics.py:8-145): VOC 11-point mAP on the device —
sorts, per-(class, image) greedy TP/FP assignment and per-class AP kernels (csrc/map.hip),
one host sync for the returned Python values, like the reference's ``.item()``/``.tolist()``;
CPU tensors take the host path (``hostpath.calculate_mAP``).
``accuracy`` / ``AverageMeter`` (metrics.py:255-289): the bookkeeping train_anchor.py:21 and
eval.py:23 import from this module, host-side as in the reference.
"""
import torch

from . import _lib as L
from . import core
from . import host
from . import hostpath

_RTHR = {}
_ONE_IMAGE_OFFSETS = {}


def _one_image_offsets(G, device):
    """gt_offsets [0, G] of a single-image call, cached per (G, device)."""
    key = (G, str(device))
    t = _ONE_IMAGE_OFFSETS.get(key)
    if t is None:
        if len(_ONE_IMAGE_OFFSETS) > 1024:
            _ONE_IMAGE_OFFSETS.clear()
        t = torch.tensor([0, G], dtype=torch.int32).pin_memory().to(device, non_blocking=True)
        _ONE_IMAGE_OFFSETS[key] = t
    return t


def on_host(*tensors):
    """True when every tensor is a CPU tensor (the host path); False when all are on the device;
    mixed devices raise as torch's own ops would."""
    cpu = [not t.is_cuda for t in tensors]
    if all(cpu):
        return True
    if any(cpu):
        raise RuntimeError('Expected all tensors to be on the same device, got %s'
                           % [str(t.device) for t in tensors])
    return False


def _single(gt, anchors, mode, what):
    L.require_device(gt, anchors, what=what)
    g = gt.reshape(-1, 4).float().contiguous()
    a = anchors.reshape(-1, 4).float().contiguous()
    G, P = g.shape[0], a.shape[0]
    if G == 0 or P == 0:
        return torch.zeros(G, P, dtype=torch.float32, device=g.device)
    pack = core.GtPack(g, None, _one_image_offsets(G, g.device), [G])
    return core.iou_pairwise(pack, a, mode=mode)[0]


def find_jaccard_overlap(gt_boxes, anchors):
    """[G, P] IoU of metrics.py:208-252."""
    if on_host(gt_boxes, anchors):
        return host.find_jaccard_overlap(gt_boxes, anchors)
    return _single(gt_boxes, anchors, L.IOU_METRICS, 'find_jaccard_overlap')


def intersect(box_a, box_b):
    """[A, B] intersection areas (metrics.py:192-205)."""
    if on_host(box_a, box_b):
        return host.intersect(box_a, box_b)
    return _single(box_a, box_b, L.IOU_INTER, 'intersect')


def _offsets(lists, device):
    offs = [0]
    for t in lists:
        offs.append(offs[-1] + int(t.shape[0]))
    return torch.tensor(offs, dtype=torch.int32).to(device, non_blocking=True), offs[-1]


def calculate_mAP(det_boxes, det_labels, det_scores, true_boxes, true_labels, true_difficulties, threshold,
                  label_map, device='cuda:0'):
    """metrics.py:8-145.  Lists of per-image tensors (ROCm device) -> (dict class name -> AP,
    mAP).  Score ties within a class keep input order (see include/sbod.h)."""
    assert len(det_boxes) == len(det_labels) == len(det_scores) == len(true_boxes) == len(
        true_labels) == len(true_difficulties)
    n_classes = len(label_map)
    B = len(det_boxes)
    rev_label_map = {v: k for k, v in label_map.items()}
    if all(not t.is_cuda for g in (det_boxes, det_labels, det_scores, true_boxes, true_labels,
                                   true_difficulties) for t in g):
        aps, mean_ap = hostpath.calculate_mAP(det_boxes, det_labels, det_scores, true_boxes, true_labels,
                                              true_difficulties, threshold, n_classes)
        return {rev_label_map[c + 1]: v for c, v in enumerate(aps)}, mean_ap
    dev = torch.device(device)
    for group in (det_boxes, det_labels, det_scores, true_boxes, true_labels, true_difficulties):
        L.require_device(*group, what='calculate_mAP')
    db = torch.cat([b.reshape(-1, 4) for b in det_boxes]).to(dev, torch.float32).contiguous()
    dl = torch.cat([l.reshape(-1) for l in det_labels]).to(dev, torch.int64).contiguous()
    ds = torch.cat([s.reshape(-1) for s in det_scores]).to(dev, torch.float32).contiguous()
    tb = torch.cat([b.reshape(-1, 4) for b in true_boxes]).to(dev, torch.float32).contiguous()
    tl = torch.cat([l.reshape(-1) for l in true_labels]).to(dev, torch.int64).contiguous()
    td = torch.cat([d.reshape(-1) for d in true_difficulties]).to(dev, torch.uint8).contiguous()
    doff, D = _offsets(det_labels, dev)
    toff, T = _offsets(true_labels, dev)
    key = str(dev)
    if key not in _RTHR:   # metrics.py:128, float32 arange exactly as the reference builds it
        _RTHR[key] = torch.arange(start=0, end=1.1, step=.1).to(dev)
    ap = torch.empty(n_classes - 1, dtype=torch.float32, device=dev)
    mean = torch.empty(1, dtype=torch.float32, device=dev)
    nb = L.lib().sbod_map_workspace_bytes(D, T)
    ws = core.workspace(nb, dev, 'map')
    L.call('sbod_map_f32', L.ptr(db), L.ptr(dl), L.ptr(ds), L.ptr(doff), L.ptr(tb), L.ptr(tl), L.ptr(td),
           L.ptr(toff), B, n_classes, D, T, float(threshold), L.ptr(_RTHR[key]), L.ptr(ap), L.ptr(mean),
           L.ptr(ws), nb, L.stream_of(db))
    aps = ap.cpu().tolist()
    mean_average_precision = float(mean.cpu().item())
    return {rev_label_map[c + 1]: v for c, v in enumerate(aps)}, mean_average_precision


def accuracy(scores, targets, k):
    """Top-k accuracy in percent (metrics.py:255-268): the share of rows whose target is among
    the k highest scores, times 100."""
    _, ind = scores.topk(k, 1, True, True)
    hits = ind.eq(targets.view(-1, 1).expand_as(ind)).view(-1).float().sum()
    return hits.item() * (100.0 / targets.size(0))


class AverageMeter(object):
    """Latest value, running sum, count and mean of a metric (metrics.py:271-289)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count
