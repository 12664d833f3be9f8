"""Drop-in criteria: the reference's loss classes, same constructor/forward signatures, running
the fused HIP path (matcher kernels + one fused loss pass + mining + finaliser).

  * ``MultiBoxLoss512``  — ``models/SSD512.py:477-626``
  * ``MultiBoxLoss300``  — ``models/SSD300.py:446-594`` (nn.L1Loss box loss, global mining pool)
  * ``RetinaFocalLoss``  — ``models/RetinaNet.py:353-506`` (focal / n_pos, negatives-only pool)
  * ``RefineDetLoss``    — ``models/RefineDet512.py:698-956`` (binary ARM + ODM on decoded ARM)

CPU tensors (the reference's ``device = 'cpu'``, train_anchor.py:65-71; config C1) take the host
path (``hostpath.py``: torch-CPU restatement, autograd backward); ROCm tensors the HIP path.

Constructed as ``criterion(priors_cxcy=model.priors_cxcy, config=config)`` (train_anchor.py:172)
with ``config`` exposing ``reg_weights, device, n_classes, reg_loss, cls_loss``; called as
``criterion(locs [B,P,4], scores [B,P,C], boxes: list of [G_i,4], labels: list of [G_i])``.
Returns a 0-d loss tensor with autograd.  ``last_components`` holds the device vector
{total, conf, loc, n_pos} of the last call (no sync).

Data parallelism: set ``distributed = True`` (optionally ``process_group``) and every rank
normalises by the all-reduced positive count, so a rank's share of the loss is
exactly its images' part of the single-device batch loss and the SUM of the ranks' gradients is
the single-device batch gradient.  DDP AVERAGES gradients over ranks, so with the default
``grad_reduction = 'mean'`` each rank returns world_size x its share (the mean of the returned
values over ranks is the single-device loss, and DDP's averaged gradient is the single-device
gradient).  Set ``grad_reduction = 'sum'`` for a trainer that sums gradients instead.
"""
import torch
from torch import nn

from .. import _lib as L
from .. import core
from .. import hostpath
from ..dataset.transforms import cxcy_to_xy
from ..metrics import on_host


def _cfg(config, key, default=None):
    if isinstance(config, dict):
        return config.get(key, default)
    return getattr(config, key, default)


class _AnchorCriterion(nn.Module):
    KIND = 'ssd512'

    def __init__(self, priors_cxcy, config, threshold=0.5, neg_pos_ratio=3):
        super().__init__()
        self.priors_cxcy = priors_cxcy
        self.priors_xy = cxcy_to_xy(priors_cxcy)
        self.threshold = threshold
        self.neg_pos_ratio = neg_pos_ratio
        self.alpha = _cfg(config, 'reg_weights', 1.0)
        self.device = _cfg(config, 'device')
        self.n_classes = _cfg(config, 'n_classes')
        self.config = config
        self.distributed = False
        self.process_group = None
        self.grad_reduction = 'mean'
        self.force_collectives = False   # run the collectives even in a one-rank group (tests)
        # focal on one device: the matcher and the loss pass as separate launches (default), or as
        # ONE launch (opt-in, variant library only: its workgroups wait for each other, so it needs
        # the whole device — with kernels of other streams sharing the CUs the grid is not
        # co-resident and the bounded wait ends in a NaN loss; measured slower alone too,
        # DESIGN.md round 4)
        self.one_launch = False
        # focal: the workgroups' loss partials are summed by a separate one-block launch after the
        # loss pass (default), or by the loss pass's last workgroup gathering every workgroup's
        # record (False: one launch fewer; its gather waits out the pass's store drain, ~4 us).
        # The same exact fixed-point sum either way: the same loss bit for bit; the same step time
        # (same-box A/B)
        self.separate_finish = True
        self.last_components = None

    def increase_threshold(self, increment=0.1):
        if self.threshold >= 0.7:
            return
        self.threshold += increment

    def _spec(self):
        key = (str(_cfg(self.config, 'reg_loss', 'smoothl1')), str(_cfg(self.config, 'cls_loss', 'ce')),
               self.neg_pos_ratio, self.alpha, self.distributed, self.separate_finish)
        if getattr(self, '_spec_key', None) != key:
            self._spec_cache = self._build_spec()
            self._spec_key = key
        return self._spec_cache

    def _build_spec(self):
        reg_loss = str(_cfg(self.config, 'reg_loss', 'smoothl1')).upper()
        cls_loss = str(_cfg(self.config, 'cls_loss', 'ce')).upper()
        if reg_loss == 'DIOU':
            reg = L.REG['diou']
        else:
            reg = L.REG['l1'] if self.KIND == 'ssd300' else L.REG['smoothl1']
        if cls_loss == 'FOCAL':
            cls = L.CLS['focal']
            flags = L.LOSS_FOCAL_NORM if self.KIND == 'retina' else 0
            if self.separate_finish:
                flags |= L.LOSS_UNFUSED_FINISH
        else:
            cls = L.CLS['ce']
            flags = {'ssd512': L.POOL['nonpos'], 'ssd300': L.POOL['global_neg'],
                     'retina': L.POOL['neg']}[self.KIND]
        return core.CriterionSpec(reg, cls, flags, self.neg_pos_ratio, float(self.alpha))

    def forward(self, predicted_locs, predicted_scores, boxes, labels):
        B, P, _ = predicted_scores.shape
        n_priors = self.priors_cxcy.size(0)
        assert n_priors == predicted_locs.size(1) == predicted_scores.size(1)
        if not self.distributed and on_host(predicted_locs, predicted_scores):
            # the reference's CPU device (train_anchor.py:65-71): the host path, no kernels
            # (data parallelism is the ROCm path's: its RCCL exchange steps need device tensors)
            return hostpath.anchor_criterion(self.KIND, self.priors_cxcy.cpu(), self.priors_xy.cpu(),
                                             predicted_locs, predicted_scores, boxes, labels,
                                             _cfg(self.config, 'reg_loss', 'smoothl1'),
                                             _cfg(self.config, 'cls_loss', 'ce'), self.threshold,
                                             self.neg_pos_ratio, self.alpha)
        spec = self._spec()
        if spec.cls == L.CLS['focal'] and not self.distributed and not self.one_launch:
            # the whole call natively (GT packing, the launches, a C++ autograd node), once the
            # Python path below has set up this stream's buffers
            r = core.criterion_focal_fast(predicted_locs, predicted_scores, boxes, labels, self.priors_cxcy,
                                          self.priors_xy, spec, self.threshold, self.threshold - 0.1)
            if r is not None:
                self.last_components = r[1]
                return r[0]
        gt = core.pack_gt(boxes, labels, reuse=True)   # consumed by this call's launches only
        if spec.cls == L.CLS['focal'] and not self.distributed:
            # one device, no mining: the matcher and the loss pass in one C call (the matcher's
            # launches then the loss launch; ONE launch with ``one_launch``)
            loss, comps, _ = core.criterion_focal(predicted_locs, predicted_scores, gt, self.priors_cxcy,
                                                  self.priors_xy, spec, self.threshold, self.threshold - 0.1,
                                                  two_launch=not self.one_launch, fresh_match=False)
            self.last_components = comps
            return loss
        obj, ovl, npos = core.match(gt, self.priors_xy, P, self.threshold)
        tot = (core.allreduce_npos(npos, self.process_group, self.force_collectives)
               if self.distributed else npos[B:])
        # SSD300's CE mines over the whole batch: data-parallel, the pools are exchanged
        exchange = (core.allgather_pool(self.process_group)
                    if self.distributed and (spec.flags & L.POOL['global_neg']) else None)
        loss, comps = core.fused_criterion(predicted_locs, predicted_scores, gt, obj, ovl, npos, tot,
                                           self.priors_cxcy, spec, self.threshold,
                                           self.threshold - 0.1, exchange=exchange)
        self.last_components = comps
        return _dp_scale(self, loss)


def _dp_scale(crit, loss):
    """Data parallel with a gradient-AVERAGING trainer (DDP): world_size x this rank's share."""
    if not crit.distributed or crit.grad_reduction == 'sum':
        return loss
    if crit.grad_reduction != 'mean':
        raise ValueError("grad_reduction must be 'mean' or 'sum', got %r" % (crit.grad_reduction,))
    import torch.distributed as dist
    world = dist.get_world_size(crit.process_group)
    return loss * world if world > 1 else loss


class MultiBoxLoss512(_AnchorCriterion):
    """``models/SSD512.py:477-626``: SmoothL1 (beta 1/9) or DIoU box loss; unnormalised softmax
    focal over positives + negatives, or CE with per-image mining over all non-positives."""
    KIND = 'ssd512'


class MultiBoxLoss300(_AnchorCriterion):
    """``models/SSD300.py:446-594``: nn.L1Loss (mean over elements) or DIoU; CE mining over the
    negatives of the whole batch (global top sum(3 n_pos))."""
    KIND = 'ssd300'


class RetinaFocalLoss(_AnchorCriterion):
    """``models/RetinaNet.py:353-506``: focal divided by the batch positives; CE mining over the
    negatives (IoU < threshold - 0.1) of each image."""
    KIND = 'retina'


class RefineDetLoss(nn.Module):
    """``models/RefineDet512.py:698-956``."""

    def __init__(self, priors_cxcy, config, threshold=0.5, neg_pos_ratio=3, theta=0.01):
        super().__init__()
        self.priors_cxcy = priors_cxcy
        self.priors_xy = cxcy_to_xy(priors_cxcy)
        self.threshold = threshold
        self.neg_pos_ratio = neg_pos_ratio
        self.alpha = _cfg(config, 'reg_weights', 1.0)
        self.device = _cfg(config, 'device')
        self.n_classes = _cfg(config, 'n_classes')
        self.config = config
        self.theta = theta
        self.distributed = False
        self.process_group = None
        self.grad_reduction = 'mean'
        self.force_collectives = False
        self.last_components = None

    def increase_threshold(self, increment=0.05):
        if self.threshold + increment >= 0.7:
            self.threshold = 0.7
        else:
            self.threshold += increment

    def _tot(self, npos, B):
        return (core.allreduce_npos(npos, self.process_group, self.force_collectives)
                if self.distributed else npos[B:])

    def compute_arm_loss(self, arm_locs, arm_scores, boxes, labels):
        """Binary anchor-refinement loss vs the fixed priors (RefineDet512.py:730-820)."""
        if not self.distributed and on_host(arm_locs, arm_scores):
            return hostpath.refinedet_arm(self.priors_cxcy.cpu(), self.priors_xy.cpu(), arm_locs, arm_scores,
                                          boxes, labels, self.threshold, self.neg_pos_ratio, self.alpha)
        L.require_device(arm_locs, arm_scores, what='RefineDetLoss')
        B, P, _ = arm_scores.shape
        gt = core.pack_gt(boxes, labels)
        obj, ovl, npos = core.match(gt, self.priors_xy, P, self.threshold, flags=L.MATCH_BINARY)
        spec = core.CriterionSpec(L.REG['smoothl1'], L.CLS['ce'], L.MATCH_BINARY | L.POOL['nonpos'],
                                  self.neg_pos_ratio, float(self.alpha))
        loss, comps = core.fused_criterion(arm_locs, arm_scores, gt, obj, ovl, npos,
                                           self._tot(npos, B), self.priors_cxcy, spec, self.threshold,
                                           self.threshold - 0.1)
        self.last_components = comps
        return loss

    def compute_odm_loss(self, arm_locs, arm_scores, odm_locs, odm_scores, boxes, labels):
        """Refined-detection loss vs the per-image decoded ARM boxes with easy negatives
        (softmax(ARM)[...,1] < theta) removed (RefineDet512.py:822-939)."""
        if not self.distributed and on_host(arm_locs, arm_scores, odm_locs, odm_scores):
            return hostpath.refinedet_odm(self.priors_cxcy.cpu(), arm_locs, arm_scores, odm_locs, odm_scores,
                                          boxes, labels, self.threshold, self.neg_pos_ratio, self.alpha,
                                          self.theta)
        L.require_device(arm_locs, arm_scores, odm_locs, odm_scores, what='RefineDetLoss')
        B, P, _ = odm_scores.shape
        assert P == self.priors_cxcy.size(0) == odm_locs.size(1)
        al = arm_locs.detach().contiguous().float()
        asc = arm_scores.detach().contiguous().float()
        gt = core.pack_gt(boxes, labels)
        obj, ovl, npos = core.match(gt, al, P, self.threshold, flags=L.MATCH_ODM,
                                    priors_cxcy=self.priors_cxcy, arm_scores=asc, theta=self.theta)
        spec = core.CriterionSpec(L.REG['smoothl1'], L.CLS['ce'],
                                  L.MATCH_ODM | L.POOL['nonpos_not_easy'], self.neg_pos_ratio,
                                  float(self.alpha))
        loss, comps = core.fused_criterion(odm_locs, odm_scores, gt, obj, ovl, npos, self._tot(npos, B),
                                           self.priors_cxcy, spec, self.threshold, self.threshold - 0.1,
                                           theta=self.theta, arm_locs=al, arm_scores=asc)
        self.last_components = comps
        return loss

    def forward(self, arm_locs, arm_scores, odm_locs, odm_scores, boxes, labels):
        arm = self.compute_arm_loss(arm_locs, arm_scores, boxes, labels)
        odm = self.compute_odm_loss(arm_locs.detach(), arm_scores.detach(), odm_locs, odm_scores,
                                    boxes, labels)
        return _dp_scale(self, arm + odm)


def criterion_entry(arch):
    """The criterion half of ``models/__init__.py:model_entry`` (networks are out of scope)."""
    a = arch.upper()
    table = {'SSD300': MultiBoxLoss300, 'SSD512': MultiBoxLoss512, 'RETINA50': RetinaFocalLoss,
             'RETINA101': RetinaFocalLoss, 'REFINEDET': RefineDetLoss}
    if a not in table:
        raise NotImplementedError('criterion for %s is not part of the sbod hot path' % arch)
    return table[a]
