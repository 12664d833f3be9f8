"""``detect_scripts/detect_tools.py`` on the HIP path.

``detect`` (:100-219): softmax, offset decode + clamp, per-class NMS, then a final
class-agnostic NMS at IoU 0.7 (:202-205) before top_k — output in descending score order.
``detect_refine`` (:222-341): no decode (boxes are predicted_locs clamped IN PLACE, :264),
optional ``prior_positives_idx`` filter (:271-281), same final NMS.
CPU tensors take the host path (``hostpath.detect``).
"""
from .. import core
from .. import hostpath
from ..metrics import on_host


def detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy):
    if on_host(predicted_locs, predicted_scores):
        return hostpath.detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy.cpu(),
                               'offset', 'softmax', None, 0.7)
    return core.detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy,
                       box_type='offset', act='softmax', final_nms=0.7)


def detect_refine(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy,
                  prior_positives_idx=None):
    if on_host(predicted_locs, predicted_scores):
        return hostpath.detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, None,
                               'corner', 'softmax', prior_positives_idx, 0.7)
    return core.detect(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy,
                       box_type='corner', act='softmax', pos_mask=prior_positives_idx, final_nms=0.7)


def detect_objects(predicted_locs, predicted_scores, min_score, max_overlap, top_k, priors_cxcy):
    """Broken in the reference (mask used as an index, :57-59, then ``exit()``, :69)."""
    raise IndexError('detect_tools.detect_objects is broken in the reference '
                     '(detect_scripts/detect_tools.py:57-69)')
