"""``operators/Loss.py`` on the HIP path — same classes, arguments and reductions.

Per-row values and their derivatives come from the sbod kernels; the reductions stay the
reference's own (sum, ``sum / num`` rows for 'mean', ``Σ(l·w)/Σw`` when ``Σw > 1e-6``) so the
numbers match Loss.py's.  CPU tensors take the host path (``hostpath.py``, the reference's own
torch ops, autograd backward).
"""
import torch
from torch import nn

from .. import core
from .. import hostpath
from ..metrics import on_host
from .iou_utils import bbox_overlaps_ciou, bbox_overlaps_diou, bbox_overlaps_giou, bbox_overlaps_iou


def focal_loss(y_pred, y_true, alpha=0.25, gamma=2., device='cuda:0'):
    """Softmax focal loss, summed (Loss.py:9-38): α_fg·(1-p_t)^γ·(-log p_t) for foreground rows,
    α_bg·p_bg^γ·(-log p_bg) for background rows (the reference's weighting)."""
    if isinstance(alpha, (list, tuple)):
        fore_alpha, back_alpha = alpha[0], alpha[1]
    else:
        fore_alpha, back_alpha = alpha, 1 - alpha
    if on_host(y_pred, y_true):
        return hostpath.focal_softmax(y_pred, y_true, (fore_alpha, back_alpha), gamma)
    return core.focal_rows('softmax', y_pred, y_true, fore_alpha, back_alpha, gamma).sum()


class SigmoidFocalLoss(nn.Module):
    """Loss.py:41-80: sigmoid focal over classes 1..C-1; background rows contribute nothing."""

    def __init__(self, gamma, alpha, config):
        super().__init__()
        self.gamma = gamma
        self.alpha = alpha
        self.device = getattr(config, 'device', None) if not isinstance(config, dict) else config.get('device')

    def forward(self, out, target):
        if on_host(out, target):
            return hostpath.focal_sigmoid(out, target, self.alpha, self.gamma)
        return core.focal_rows('sigmoid', out, target, self.alpha, 1 - self.alpha, self.gamma).sum()


class FocalLoss(nn.Module):
    """Loss.py:83-103: BCE-with-logits focal over all C one-hot columns, prediction clamped."""

    def __init__(self, alpha=0.25, gamma=2):
        super().__init__()
        self.alpha = alpha
        self.gamma = gamma

    def forward(self, pred_logits, targets):
        if on_host(pred_logits, targets):
            return hostpath.focal_bce(pred_logits, targets, self.alpha, self.gamma)
        return core.focal_rows('bce', pred_logits, targets, self.alpha, 1 - self.alpha, self.gamma).sum()


def _decode_center(loc, priors, variances):
    c = torch.cat([priors[:, :2] + loc[:, :2] * variances[0] * priors[:, 2:],
                   priors[:, 2:] * torch.exp(loc[:, 2:] * variances[1])], 1)
    xy = c[:, :2] - c[:, 2:] / 2
    return torch.cat([xy, c[:, 2:] + xy], 1)


class IouLoss(nn.Module):
    """Loss.py:164-200."""

    def __init__(self, pred_mode='Corner', reduce='mean', variances=None, losstype='Diou'):
        super().__init__()
        self.reduce = reduce
        self.pred_mode = pred_mode
        self.variances = variances
        self.loss = losstype

    def forward(self, loc_p, loc_t, prior_data=None, weights=None):
        num = loc_p.shape[0]
        if self.pred_mode == 'Center':
            assert prior_data is not None
            decoded_boxes = _decode_center(loc_p, prior_data, self.variances)
        else:
            decoded_boxes = loc_p
        fn = {'Iou': bbox_overlaps_iou, 'Giou': bbox_overlaps_giou,
              'Diou': bbox_overlaps_diou}.get(self.loss, bbox_overlaps_ciou)
        loss = 1.0 - fn(decoded_boxes, loc_t)
        if weights is not None and weights.sum() > 1e-6:
            return (loss * weights).sum() / weights.sum()
        if self.reduce == 'mean':
            return loss.sum() / num
        return loss.sum()


class SmoothL1Loss(nn.Module):
    """Loss.py:203-226 (beta 1/9; 'mean' = sum / rows)."""

    def __init__(self, beta=1.0 / 9.0, reduction='mean'):
        super().__init__()
        self.beta = beta
        self.reduction = reduction

    def forward(self, pred, target, weights=None):
        num = pred.size(0)
        if on_host(pred, target):
            l1_loss = hostpath.smooth_l1_elementwise(pred, target, self.beta)
        else:
            l1_loss = core.smooth_l1_elementwise(pred, target, self.beta)
        if weights is not None and weights.sum() > 1e-6:
            assert pred.size(0) == target.size(0) == weights.size(0)
            return (l1_loss * weights).sum() / weights.sum()
        if self.reduction == 'mean':
            return l1_loss.sum() / num
        return l1_loss.sum()
