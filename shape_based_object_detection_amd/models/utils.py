"""``models/utils.py`` detection post-processing on the HIP path.

``detect`` (models/utils.py:181-297) keeps the reference's signature, config keys
(``config.model['box_type']``, ``config['focal_type']``, ``config.device``) and outputs: lists
of per-image boxes [K,4] (clamped xyxy), labels [K] int64 and scores [K], K <= top_k, classes in
order 1..C-1 unless more than top_k objects survive (then the top_k by score), the
[[0,0,1,1]] / 0 / 0 placeholder for an image without detections, and the in-place clamp of the
caller's ``predicted_locs`` when box_type is neither 'offset' nor 'center'.
NMS semantics are torchvision.ops.nms's (models/utils.py:5,265): suppress IoU > max_overlap,
ties in score resolved by lower prior index.  CPU tensors (the reference's ``device = 'cpu'``)
take the host path (``hostpath.detect``), ROCm tensors the HIP kernels.
"""
from .. import core
from .. import hostpath
from ..metrics import on_host


def _cfg(config, key, default=None):
    if isinstance(config, dict):
        return config.get(key, default)
    try:
        return config[key]
    except (KeyError, TypeError, IndexError):
        return getattr(config, key, default)


def detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy, config,
           prior_positives_idx=None, async_=False):
    """``async_=True`` (an addition; the reference has no such argument) returns a handle whose
    ``wait()`` gives the lists: the caller can queue the next step's work before the one host sync
    detect needs (its per-image counts)."""
    model = _cfg(config, 'model', {}) or {}
    box_type = model.get('box_type', 'offset') if isinstance(model, dict) else getattr(model, 'box_type')
    focal_type = str(_cfg(config, 'focal_type', 'softmax'))
    act = 'sigmoid' if focal_type.lower() == 'sigmoid' else 'softmax'
    bt = box_type if box_type in ('offset', 'center') else 'corner'
    if on_host(predicted_locs, predicted_scores):
        return hostpath.detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k,
                               priors_cxcy.cpu() if priors_cxcy is not None else None, bt, act,
                               prior_positives_idx)
    return core.detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy,
                       box_type=bt, act=act, pos_mask=prior_positives_idx, async_=async_)


def detect_objects(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy,
                   config):
    """The reference's ``detect_objects`` (models/utils.py:87-178) cannot run: it squeezes dim 1
    of a 1-D tensor (:136).  Kept for API completeness with the same failure."""
    raise IndexError('Dimension out of range (expected to be in range of [-1, 0], but got 1) '
                     '[models/utils.py:136 detect_objects is broken in the reference]')
