"""Host-side orchestration of the HIP hot path (device memory, workspaces, ragged GT packing).

Everything here runs on ROCm device tensors; inputs on the CPU are rejected.  No call in this
module synchronises with the host unless its docstring says so.
"""
import numpy as np
import torch

from . import _lib as L


class GtPack:
    """Ragged ground truth packed once per step (dataset/Datasets.py:58-86 list-of-tensors).

    boxes [sum G, 4] f32 xyxy, labels [sum G] int64, offsets [B+1] int32 on the device;
    ``counts`` / ``gmax`` are host ints (taken from tensor shapes: no device sync).  A pack
    staged into fixed-capacity buffers (``GtStaging``) reports ``gmax`` = its per-image capacity,
    so every launch that reads it has the same shape from step to step (hipGraph replay)."""

    __slots__ = ('boxes', 'labels', 'offsets', 'counts', 'gmax', 'batch')

    def __init__(self, boxes, labels, offsets, counts, gmax=None):
        self.boxes, self.labels, self.offsets, self.counts = boxes, labels, offsets, counts
        self.gmax = gmax if gmax is not None else (max(counts) if counts else 0)
        self.batch = len(counts)


_PTR_TABLES = {}


def _ptr_tables(B):
    """Host arrays (box pointers, label pointers, counts) handed to sbod_gt_pack, cached per B.
    The C call reads them before it returns, so one set per batch size is enough."""
    t = _PTR_TABLES.get(B)
    if t is None:
        bp, lp, cn = np.zeros(B, np.uint64), np.zeros(B, np.uint64), np.zeros(B, np.int32)
        t = (bp, lp, cn, bp.ctypes.data, lp.ctypes.data, cn.ctypes.data)
        _PTR_TABLES[B] = t
    return t


def _check_counts(counts, allow_empty):
    if not allow_empty and 0 in counts:
        raise RuntimeError('max(): Expected reduction dim 0 to have non-zero size (an image has no '
                           'ground-truth objects, as in the reference criterion)')


def _as_rows(boxes, labels):
    """Per-image [G,4] f32 / [G] int64 contiguous device tensors (converted only when needed)."""
    bx, lb = [], []
    dev = None
    for b, l in zip(boxes, labels):
        if not (b.is_cuda and l.is_cuda):
            L.require_device(b, l, what='pack_gt')
        if dev is None:
            dev = b.device
        elif b.device != dev or l.device != dev:
            raise RuntimeError('pack_gt: ground truth of one batch spans several devices')
        if b.dtype != torch.float32 or not b.is_contiguous() or b.dim() != 2:
            b = b.reshape(-1, 4).float().contiguous()
        if l.dtype != torch.int64 or not l.is_contiguous() or l.dim() != 1:
            l = l.reshape(-1).long().contiguous()
        bx.append(b)
        lb.append(l)
    return bx, lb, dev


def _launch_pack(bx, lb, counts, capacity, out_b, out_l, out_off):
    B = len(counts)
    bp, lp, cn, bpa, lpa, cna = _ptr_tables(B)
    bp[:] = [b.data_ptr() for b in bx]
    lp[:] = [l.data_ptr() for l in lb]
    cn[:] = counts
    L.call('sbod_gt_pack', bpa, lpa, cna, B, capacity, L.ptr(out_b), L.ptr(out_l), L.ptr(out_off),
           L.stream_of(out_off))


def _pack_fast(boxes, labels, capacity, per_image, dev_index, out_b, out_l, out_off, allow_empty):
    """The whole list check + sbod_gt_pack launch in C++ (_sbodhost, csrc/hostpack.cpp).
    Counts on success; None when the batch needs the Python path (conversions, errors)."""
    ext = L.host_ext
    if ext is None or type(boxes) is not list or type(labels) is not list:
        return None
    r = ext.pack_device_lists(boxes, labels, capacity, per_image, dev_index, out_b.data_ptr(),
                              out_l.data_ptr(), out_off.data_ptr(), L.stream_of(out_off), allow_empty)
    if type(r) is int:
        raise L.SbodError('sbod_gt_pack failed (%d): %s'
                          % (r, L.lib().sbod_last_error().decode(errors='replace')))
    return r


# pack_gt's output buffers for regular device batches, cached per (device, stream, batch size)
# and grown on demand: every consumer of a pack runs in stream order on the stream that packed
# it, so the next pack on that stream may overwrite the buffers (as the per-stream workspaces).
_PACK_CACHE = {}
_PACK_CAP = {}    # rows to allocate next time for a key whose batch overflowed its buffers
_PACK_CAPTURED = set()   # data_ptr of cached pack buffers handed out under hipGraph capture
_PACK_RETIRED = []       # grown-out-of pack buffers a captured graph may still address (kept alive)


def _pack_cached(boxes, labels, allow_empty):
    """The C++ list check + sbod_gt_pack launch into the stream's cached buffers (no Python loop
    over the images, no allocation).  None when the batch needs the Python path."""
    ext = L.host_ext
    if ext is None or type(boxes) is not list or type(labels) is not list or not boxes:
        return None
    b0 = boxes[0]
    if not b0.is_cuda:
        return None
    dev = b0.device
    B = len(boxes)
    stream = L._raw_stream(dev.index)
    key = (dev.index, stream, B)
    buf = _PACK_CACHE.get(key)
    if buf is None:
        if torch.cuda.is_current_stream_capturing():
            return None   # nothing is allocated under capture: the Python path's own tensors
        cap = max(_PACK_CAP.get(key, 0), 256 * B)
        buf = _PACK_CACHE[key] = (torch.empty(cap, 4, dtype=torch.float32, device=dev),
                                  torch.empty(cap, dtype=torch.int64, device=dev),
                                  torch.empty(B + 1, dtype=torch.int32, device=dev), cap)
    gb, gl, off, cap = buf
    r = ext.pack_device_lists(boxes, labels, cap, -1, dev.index, gb.data_ptr(), gl.data_ptr(), off.data_ptr(),
                              stream, allow_empty)
    if r is None:
        return None
    if type(r) is int:
        raise L.SbodError('sbod_gt_pack failed (%d): %s' % (r, L.lib().sbod_last_error().decode(errors='replace')))
    if torch.cuda.is_current_stream_capturing():
        _PACK_CAPTURED.add(gb.data_ptr())   # the graph writes these rows on every replay
    n = sum(r)
    return GtPack(gb[:n], gl[:n], off, r)


def pack_gt(boxes, labels, device=None, allow_empty=False, reuse=False):
    """Pack per-image lists into a GtPack with ONE device launch (sbod_gt_pack: the pointers
    and offsets travel in the kernel arguments).  An image with no objects raises like the
    reference does (``overlap.max(dim=0)`` of an empty matrix, models/SSD512.py:538).  A GtPack
    (e.g. from ``GtStaging.stage``) is returned as is.  ``reuse=True`` (a caller that consumes
    the pack at once on the current stream, e.g. the criterion classes): a regular device batch
    (lists of [G,4] float32 / [G] int64 contiguous device tensors) is checked and packed in C++
    into buffers cached per stream, which the NEXT reuse-pack on that stream overwrites; anything
    else (conversions, errors) takes the Python path with buffers of its own."""
    if isinstance(boxes, GtPack):
        return boxes
    if len(boxes) != len(labels):
        raise ValueError('boxes and labels must have the same length')
    if reuse:
        fast = _pack_cached(boxes, labels, allow_empty)
        if fast is not None:
            return fast
    counts = [b.shape[0] for b in boxes]
    _check_counts(counts, allow_empty)
    bx, lb, dev = _as_rows(boxes, labels)
    n = sum(counts)
    key = (dev.index, L._raw_stream(dev.index), len(counts))
    if key in _PACK_CACHE and n > _PACK_CACHE[key][3] and not torch.cuda.is_current_stream_capturing():
        _PACK_CAP[key] = 2 * n    # the stream's buffers grow on its next regular call
        old = _PACK_CACHE.pop(key)
        if old[0].data_ptr() in _PACK_CAPTURED:
            # a captured graph still packs GT into these buffers on replay: never hand them back
            # to the allocator (as workspace() retires captured workspaces)
            _PACK_CAPTURED.discard(old[0].data_ptr())
            _PACK_RETIRED.append(old)
    gb = torch.empty(max(n, 1), 4, dtype=torch.float32, device=dev)
    gl = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    off = torch.empty(len(counts) + 1, dtype=torch.int32, device=dev)
    _launch_pack(bx, lb, counts, max(n, 1), gb, gl, off)
    return GtPack(gb[:n], gl[:n], off, counts)


class GtStaging:
    """Fixed-capacity device ground truth for batches of ``batch`` images with at most
    ``capacity`` objects each.

    ``stage(boxes, labels)`` packs a collate_fn batch into the SAME device buffers every step
    and returns a GtPack whose ``gmax`` is the capacity, so a hipGraph captured over a criterion
    call keeps reading valid ground truth when it is replayed with the next batch:
      * device lists (train_anchor.py:266-268 already moved them): one sbod_gt_pack launch;
      * host (CPU) lists, straight from the DataLoader: packed into a pinned host buffer and sent
        with ONE host->device copy (double-buffered, so the host never overwrites a buffer whose
        copy is still in flight) — replacing the training loop's per-image ``.to(device)``."""

    def __init__(self, batch, capacity, device):
        self.batch, self.capacity = int(batch), int(capacity)
        self.device = torch.device(device)
        if self.device.type == 'cuda' and self.device.index is None:
            self.device = torch.device('cuda', torch.cuda.current_device())
        rows = self.batch * self.capacity
        # one device region, boxes | labels | offsets, so the host path is a single copy
        self._nb = (rows * 16, rows * 8, (self.batch + 1) * 4)
        region = torch.zeros(sum(self._nb), dtype=torch.uint8, device=self.device)
        self.boxes, self.labels, self.offsets = self._views(region)
        self._region = region
        self._host = []
        self._host_next = 0
        self._fixed = None

    def _views(self, region):
        nb_b, nb_l, _ = self._nb
        return (region[:nb_b].view(torch.float32).view(-1, 4),
                region[nb_b:nb_b + nb_l].view(torch.int64),
                region[nb_b + nb_l:].view(torch.int32))

    def _pinned(self):
        if not self._host:
            n = sum(self._nb)
            self._host = [(torch.empty(n, dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
                          for _ in range(2)]
        buf, ev = self._host[self._host_next]
        self._host_next ^= 1
        ev.synchronize()   # the copy that last used this buffer has finished
        return buf, ev

    def stage(self, boxes, labels, allow_empty=False):
        if len(boxes) != self.batch or len(labels) != self.batch:
            raise ValueError('GtStaging: batch of %d images, staging holds %d'
                             % (len(boxes), self.batch))
        if boxes[0].is_cuda:
            counts = _pack_fast(boxes, labels, self.boxes.shape[0], self.capacity, self.device.index or 0,
                                self.boxes, self.labels, self.offsets, allow_empty)
            if counts is not None:
                return GtPack(self.boxes, self.labels, self.offsets, counts, gmax=self.capacity)
        counts = [b.shape[0] for b in boxes]
        _check_counts(counts, allow_empty)
        if max(counts) > self.capacity:
            raise ValueError('GtStaging: an image has %d objects, capacity is %d'
                             % (max(counts), self.capacity))
        if boxes[0].is_cuda:
            bx, lb, dev = _as_rows(boxes, labels)
            if dev != self.device:
                raise RuntimeError('GtStaging: ground truth on %s, staging on %s' % (dev, self.device))
            _launch_pack(bx, lb, counts, self.boxes.shape[0], self.boxes, self.labels, self.offsets)
        else:
            self._stage_host(boxes, labels, counts)
        return GtPack(self.boxes, self.labels, self.offsets, counts, gmax=self.capacity)

    def stage_and_replay(self, boxes, labels, launches, event=0, event_stream=0, allow_empty=False,
                         pack_stream=None, src_stream=None):
        """One-call submit of a captured step: ``stage`` of device lists on ``pack_stream`` (a raw
        hipStream_t; default the first launch's stream — the graph that reads the GT must be on
        it), then every (graph exec, stream) of ``launches`` (from ``graph_launches``), then
        ``event`` (a raw hipEvent_t, 0 for none) recorded on ``event_stream`` — all in C++
        (_sbodhost.stage_and_replay).  Returns the GtPack, or None when the batch or the build
        needs the Python path (nothing was launched then).

        Ordering: the lists may have been produced on the CURRENT stream (e.g. a non_blocking
        ``.to(device)``).  The packing stream waits for it first, and the current stream waits
        for the packing launch afterwards (not for the graphs), so the pack never reads a copy
        in flight and the caching allocator cannot recycle the lists' memory under it.
        ``src_stream`` (a raw hipStream_t) names the stream the lists were produced on when it is
        not the current one; passing the packing stream itself says they are ready (no wait)."""
        ext = L.host_ext
        if (ext is None or type(boxes) is not list or type(labels) is not list or not launches
                or len(boxes) != self.batch or not boxes[0].is_cuda):
            return None
        fixed = self._fixed
        if fixed is None:   # the staging buffers' constants, computed once (per-step host time)
            dev = self.device.index or 0
            fixed = self._fixed = (self.boxes.shape[0], self.capacity, dev, self.boxes.data_ptr(),
                                   self.labels.data_ptr(), self.offsets.data_ptr())
        r = ext.stage_and_replay(boxes, labels, fixed[0], fixed[1], fixed[2], fixed[3], fixed[4], fixed[5],
                                 pack_stream if pack_stream is not None else launches[0][1], allow_empty,
                                 launches, event or None, event_stream or None,
                                 (src_stream if src_stream is not None else L._raw_stream(fixed[2])) or None)
        if r is None:
            return None
        if type(r) is int:
            raise L.SbodError('stage_and_replay failed (%d): %s'
                              % (r, L.lib().sbod_last_error().decode(errors='replace')))
        return GtPack(self.boxes, self.labels, self.offsets, r, gmax=self.capacity)

    def _stage_host(self, boxes, labels, counts):
        buf, ev = self._pinned()
        hb, hl, ho = self._views(buf)
        n = sum(counts)
        if n:
            torch.cat([b.reshape(-1, 4).float() for b in boxes], out=hb[:n])
            torch.cat([l.reshape(-1).long() for l in labels], out=hl[:n])
        ho.copy_(torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)))
        self._region.copy_(buf, non_blocking=True)
        ev.record(torch.cuda.current_stream(self.device))


def graph_launches(pairs):
    """((graph exec, stream) raw handles) for ``GtStaging.stage_and_replay`` from
    ((torch.cuda.CUDAGraph, torch.cuda.Stream), ...), computed once per captured step."""
    return tuple((int(g.raw_cuda_graph_exec()), int(st.cuda_stream)) for g, st in pairs)


_WS = {}
_WS_CAPTURED = set()   # data_ptr of workspaces handed out under hipGraph capture
_WS_RETIRED = []       # grown-out-of workspaces a captured graph may still address (kept alive)


def workspace(nbytes, device, slot='default'):
    """Device scratch, cached per (device, current stream, slot) and grown on demand.  Reuse is
    safe because every user of a slot runs in stream order on that stream.  A buffer handed out
    under hipGraph capture is never returned to the allocator when the slot grows later (the
    graph keeps its address and writes it on every replay): it is retired and kept alive."""
    dev = device if isinstance(device, torch.device) else torch.device(device)
    key = (dev, L._raw_stream(dev.index if dev.index is not None else torch.cuda.current_device())
           if dev.type == 'cuda' else 0, slot)
    buf = _WS.get(key)
    n = max(int(nbytes), 1)
    capturing = dev.type == 'cuda' and torch.cuda.is_current_stream_capturing()
    if buf is None or buf.numel() < n:
        if capturing:
            # a workspace first allocated under hipGraph capture has faulted replays on this
            # runtime: the caller warms up on the capture stream so it exists beforehand
            raise L.SbodError('sbod workspace %r (%d bytes) would be allocated under hipGraph capture: '
                              'run the same calls once on the capture stream before capturing'
                              % (slot, n))
        if buf is not None:
            _CLEAN.pop(buf.data_ptr(), None)
            if buf.data_ptr() in _WS_CAPTURED:
                _WS_RETIRED.append(buf)        # a captured graph still writes it on replay
            # else its memory returns to the allocator
        buf = torch.empty(max(n, 1 << 20), dtype=torch.uint8, device=dev)
        _CLEAN.pop(buf.data_ptr(), None)
        _WS[key] = buf
    if capturing:
        _WS_CAPTURED.add(buf.data_ptr())
    return buf


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
    nb = L.lib().sbod_match_workspace_bytes_p(B, gt.gmax, P)
    ws = workspace(nb, dev, 'match')
    # the keys / counts are left zero by every successful call (SBOD_MATCH_WS_ZEROED)
    zflag = _zeroed_flag(ws, nb, L.MATCH_WS_ZEROED, 'match')
    _CLEAN.pop(ws.data_ptr(), None)
    L.call('sbod_match_f32', L.ptr(gt.boxes), L.ptr(gt.labels), L.ptr(gt.offsets), B, gt.gmax,
           L.ptr(anchors.contiguous()), L.ptr(priors_cxcy), L.ptr(arm_scores), P, float(threshold),
           float(theta), int(flags) | zflag, L.ptr(obj), L.ptr(ovl), L.ptr(npos), L.ptr(ws), nb,
           L.stream_of(anchors))
    _CLEAN[ws.data_ptr()] = (nb, None)
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


# ----------------------------------------------------------------------------- fused criterion
class CriterionSpec:
    """Static description of one criterion (which losses, pools and normalisers)."""

    __slots__ = ('reg', 'cls', 'flags', 'neg_pos_ratio', 'reg_weight', 'alpha', 'gamma')

    def __init__(self, reg, cls, flags=0, neg_pos_ratio=3, reg_weight=1.0, alpha=0.25, gamma=2.0):
        self.reg, self.cls, self.flags = reg, cls, flags
        self.neg_pos_ratio, self.reg_weight = neg_pos_ratio, reg_weight
        self.alpha, self.gamma = alpha, gamma


_UNIT = {}


def unit_grad(device):
    """The read-only upstream gradient 1.0 (a cached 0-d float32 device tensor).  A criterion loss
    back-propagated with it — ``loss.backward(core.unit_grad(loss.device))`` — skips the
    upstream-gradient launch entirely (the fused forward already wrote the gradients at scale
    1), and autograd needs no ones-fill kernel either: two launches fewer per captured train
    step.  Any other gradient (AMP scaling, a weighted sum of losses) takes the scale launch."""
    dev = torch.device(device)
    if dev.type == 'cuda' and dev.index is None:
        dev = torch.device('cuda', torch.cuda.current_device())
    t = _UNIT.get(dev)
    if t is None:
        t = _UNIT[dev] = torch.ones((), dtype=torch.float32, device=dev)
    return t


class _FusedLoss(torch.autograd.Function):
    """Forward computes the loss AND the gradients w.r.t. locs/scores in one pass (read once,
    write once); backward applies the upstream scalar on the device (no host sync, no pass at
    all when it is 1)."""

    @staticmethod
    def forward(ctx, locs, scores, run, want):
        out, gl, gs = run(want)
        # kept as plain attributes (not save_for_backward) and released in backward, so the
        # returned gradients are the only references and AccumulateGrad adopts them as .grad
        # instead of cloning 4(4+C)BP bytes every step
        ctx.grads = (gl, gs)
        ctx.set_materialize_grads(False)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        if ctx.grads is None:
            raise RuntimeError('sbod fused criterion: backward through the same graph twice is not '
                               'supported (its gradients are produced in forward)')
        gl, gs = ctx.grads
        ctx.grads = None
        if g is None or gl is None:
            return None, None, None, None
        u = _UNIT.get(g.device)
        if u is not None and g.data_ptr() == u.data_ptr():   # unit_grad(): nothing to apply
            return gl, gs, None, None
        if g.dtype != torch.float32 or not g.is_contiguous():
            g = g.detach().to(torch.float32).contiguous()
        L.call('sbod_scale2_inplace', L.ptr(gl), gl.numel(), L.ptr(gs), gs.numel(),
               L.DT_F32 if gl.dtype == torch.float32 else L.DT_BF16, L.ptr(g), L.stream_of(gl))
        return gl, gs, None, None


def fused_criterion(locs, scores, gt, obj, ovl, n_pos, npos_total, priors_cxcy, spec, threshold,
                    neg_threshold, theta=0.01, arm_locs=None, arm_scores=None, exchange=None):
    """Scalar loss (autograd-enabled) of one criterion pass; also returns the device vector
    {total, conf, loc, n_pos_total} (no sync).

    ``exchange`` (CE with the global pool only): ``f(pool [B*P] f32) -> (pool_all, local_off)``,
    the data-parallel exchange step — every rank's pool gathered rank-major (``allgather_pool``).
    Mining then selects over the whole gathered batch (sbod_multibox_mine_global)."""
    locs = locs.contiguous()
    scores = scores.contiguous()
    if locs.dtype not in (torch.float32, torch.bfloat16) or scores.dtype != locs.dtype:
        raise TypeError('sbod criterion: locs/scores must both be float32 or bfloat16')
    dt = L.DT_F32 if locs.dtype == torch.float32 else L.DT_BF16
    B, P, C = scores.shape
    if locs.shape != (B, P, 4) or priors_cxcy.shape[0] != P:
        raise AssertionError('n_priors mismatch: priors %d, locs %s, scores %s'
                             % (priors_cxcy.shape[0], tuple(locs.shape), tuple(scores.shape)))
    dev = locs.device
    stream = L.stream_of(locs)

    holder = []

    def run(want_grad):
        out = torch.empty(4, dtype=torch.float32, device=dev)
        holder.append(out)
        gl = torch.empty_like(locs) if want_grad else None
        gs = torch.empty_like(scores) if want_grad else None
        nb = L.lib().sbod_loss_workspace_bytes(B, P)
        ws = workspace(nb, dev, 'loss')
        flags = spec.flags | (L.LOSS_DEFER_MINING if exchange is not None else 0)
        # the fused finish's accumulators are left zero by every successful call
        zprefix = _loss_zero_bytes(B, P)
        zflag = _zeroed_flag(ws, zprefix, L.LOSS_WS_ZEROED, 'criterion')
        _CLEAN.pop(ws.data_ptr(), None)
        L.call('sbod_multibox_loss', L.ptr(locs), L.ptr(scores), dt, B, P, C, L.ptr(priors_cxcy),
               L.ptr(arm_locs), L.ptr(arm_scores), L.ptr(gt.boxes), L.ptr(gt.labels),
               L.ptr(gt.offsets), L.ptr(obj), L.ptr(ovl), L.ptr(n_pos), L.ptr(npos_total),
               float(threshold), float(neg_threshold), float(theta), spec.reg, spec.cls, flags | zflag,
               int(spec.neg_pos_ratio), float(spec.reg_weight), float(spec.alpha), float(spec.gamma),
               L.ptr(gl), L.ptr(gs), L.ptr(out), L.ptr(ws), nb, stream)
        _CLEAN[ws.data_ptr()] = (zprefix, None)   # (only the finish's state is known clean)
        if exchange is not None:
            off = L.lib().sbod_loss_pool_offset(B, P)
            pool = ws.narrow(0, off, 4 * B * P).view(torch.float32)
            pool_all, local_off = exchange(pool)
            pool_all = pool_all.contiguous()
            L.call('sbod_multibox_mine_global', L.ptr(scores), dt, B, P, C, L.ptr(npos_total), spec.reg,
                   spec.cls, flags, int(spec.neg_pos_ratio), float(spec.reg_weight), L.ptr(pool_all),
                   pool_all.numel(), int(local_off), L.ptr(gs), L.ptr(out), L.ptr(ws), nb, stream)
        return out, gl, gs

    want = torch.is_grad_enabled() and (locs.requires_grad or scores.requires_grad)
    loss = _FusedLoss.apply(locs, scores, run, want)
    return loss, holder[0]


_VARIANTS = []        # sbod_build_variants(), queried once
_CRIT_SIZES = {}      # (B, Gmax, P) -> (workspace bytes, zero-on-entry bytes)
_MATCH_OUT = {}       # (device, stream, B, P) -> (obj, ovl, npos) reused by criterion classes
_CRIT_SHAPE = {}      # criterion workspace data_ptr -> (B, Gmax, P) of its last call


def _variants():
    if not _VARIANTS:
        _VARIANTS.append(L.lib().sbod_build_variants())
    return _VARIANTS[0]


def criterion_focal(locs, scores, gt, priors_cxcy, priors_xy, spec, threshold, neg_threshold,
                    two_launch=None, fresh_match=True):
    """A focal criterion on one device in ONE launch (sbod_criterion_focal): the matcher and the
    fused loss + gradient pass, the normaliser produced inside the launch.  Returns (scalar loss
    with autograd, device vector {total, conf, loc, n_pos_total}, (obj, ovl, n_pos)).
    ``two_launch`` (default None = True) runs the same call as the matcher and loss launches — the
    only form the product library has; ``two_launch=False`` asks for the one-launch form, which is
    a variant build (sbod_build_variants()): asked of the product library it raises instead of
    silently running two launches.
    ``fresh_match=False`` (the criterion classes, which do not keep the matcher outputs): obj /
    ovl / n_pos live in buffers reused by the next call on the same stream."""
    if two_launch is None:
        two_launch = True
    if not two_launch and not (_variants() & L.VARIANT_ONE_LAUNCH_CRITERION):
        raise L.SbodError('the one-launch criterion is built into the variant library only '
                          '(EXTRA=-DSBOD_VARIANT_ONE_LAUNCH scripts/build_lib_variant.sh); this library runs the '
                          'matcher and the loss pass as two launches (criterion.one_launch = False)')
    if not locs.is_contiguous():
        locs = locs.contiguous()
    if not scores.is_contiguous():
        scores = scores.contiguous()
    ldt = locs.dtype
    if (ldt is not torch.float32 and ldt is not torch.bfloat16) or scores.dtype is not ldt:
        raise TypeError('sbod criterion: locs/scores must both be float32 or bfloat16')
    dt = L.DT_F32 if ldt is torch.float32 else L.DT_BF16
    B, P, C = scores.shape
    if locs.shape != (B, P, 4) or priors_cxcy.shape[0] != P:
        raise AssertionError('n_priors mismatch: priors %d, locs %s, scores %s'
                             % (priors_cxcy.shape[0], tuple(locs.shape), tuple(scores.shape)))
    if gt.batch != B:
        raise ValueError('criterion: %d images of ground truth for a batch of %d' % (gt.batch, B))
    dev = locs.device
    stream = L._raw_stream(dev.index)
    mkey = (dev.index, stream, B, P)
    mo = None if fresh_match else _MATCH_OUT.get(mkey)
    if mo is None:
        mo = (torch.empty(B, P, dtype=torch.int32, device=dev), torch.empty(B, P, dtype=torch.float32, device=dev),
              torch.empty(B + 1, dtype=torch.int32, device=dev))
        if not fresh_match and not torch.cuda.is_current_stream_capturing():
            _MATCH_OUT[mkey] = mo
    obj, ovl, npos = mo
    gmax = max(int(gt.gmax), 1)
    pxy = priors_xy if priors_xy.is_contiguous() else priors_xy.contiguous()
    sizes = _CRIT_SIZES.get((B, gmax, P))
    if sizes is None:
        lib = L.lib()
        sizes = _CRIT_SIZES[(B, gmax, P)] = (lib.sbod_criterion_workspace_bytes(B, gmax, P),
                                             lib.sbod_criterion_zero_bytes(B, gmax, P))
    nb, zb = sizes
    holder = []

    def run(want_grad):
        out = torch.empty(4, dtype=torch.float32, device=dev)
        holder.append(out)
        gl = torch.empty_like(locs) if want_grad else None
        gs = torch.empty_like(scores) if want_grad else None
        ws = workspace(nb, dev, 'criterion')
        wp = ws.data_ptr()
        _CRIT_SHAPE[wp] = (B, gmax, P)
        zflag = _zeroed_flag(ws, zb, L.CRIT_WS_ZEROED, 'criterion')
        _CLEAN.pop(wp, None)
        flags = ((spec.flags & (L.LOSS_FOCAL_NORM | L.LOSS_UNFUSED_FINISH)) | zflag |
                 (L.CRIT_TWO_LAUNCH if two_launch else 0))
        L.call('sbod_criterion_focal', locs.data_ptr(), scores.data_ptr(), dt, B, P, C, priors_cxcy.data_ptr(),
               pxy.data_ptr(), gt.boxes.data_ptr(), gt.labels.data_ptr(), gt.offsets.data_ptr(), gmax,
               float(threshold), float(neg_threshold), spec.reg, flags, float(spec.reg_weight), float(spec.alpha),
               float(spec.gamma), obj.data_ptr(), ovl.data_ptr(), npos.data_ptr(), L.ptr(gl), L.ptr(gs),
               out.data_ptr(), wp, nb, stream)
        _CLEAN[wp] = (zb, None)   # (only the zero-on-entry prefix is known clean)
        return out, gl, gs

    want = torch.is_grad_enabled() and (locs.requires_grad or scores.requires_grad)
    loss = _FusedLoss.apply(locs, scores, run, want)
    return loss, holder[0], (obj, ovl, npos)


def criterion_focal_fast(locs, scores, boxes, labels, priors_cxcy, priors_xy, spec, threshold, neg_threshold):
    """The criterion classes' focal call in ONE native call (_sbodhost.criterion_focal_fast): GT
    list checks + packing into the stream's cached buffers, sbod_criterion_focal (two launches,
    ``fresh_match=False`` buffers), and the loss tensor's C++ autograd node — the same launches,
    buffers and gradients as ``pack_gt(reuse=True)`` + ``criterion_focal``.  Returns
    (loss, components) or None when the call needs that Python path (first call on a stream,
    growing buffers, conversions, capture, any irregular argument: it re-checks and raises the
    errors)."""
    ext = L.host_ext
    if (ext is None or L._recorder or type(boxes) is not list or type(labels) is not list or not locs.is_cuda
            or torch.cuda.is_current_stream_capturing()):
        return None   # (a recording caller needs the sbod_* calls to pass through L.call)
    dev = locs.device
    B, P = locs.shape[0], locs.shape[1]
    stream = L._raw_stream(dev.index)
    pk = _PACK_CACHE.get((dev.index, stream, B))
    mo = _MATCH_OUT.get((dev.index, stream, B, P))
    ws = _WS.get((dev, stream, 'criterion'))
    if (pk is None or mo is None or ws is None or priors_cxcy.shape[0] != P or not priors_cxcy.is_contiguous()
            or not priors_xy.is_contiguous()):
        return None
    gb, gl, off, cap = pk
    obj, ovl, npos = mo
    wp = ws.data_ptr()
    ent = _CLEAN.pop(wp, None)
    u = _UNIT.get(dev)
    flags = (spec.flags & (L.LOSS_FOCAL_NORM | L.LOSS_UNFUSED_FINISH)) | L.CRIT_TWO_LAUNCH
    r = ext.criterion_focal_fast(locs, scores, boxes, labels, priors_cxcy.data_ptr(), priors_xy.data_ptr(),
                                 gb.data_ptr(), gl.data_ptr(), off.data_ptr(), cap, spec.reg, flags, float(threshold),
                                 float(neg_threshold), float(spec.reg_weight), float(spec.alpha), float(spec.gamma),
                                 obj.data_ptr(), ovl.data_ptr(), npos.data_ptr(), wp, ws.numel(),
                                 ent[0] if ent is not None else 0, stream, u.data_ptr() if u is not None else None)
    if r is None:
        if ent is not None:
            _CLEAN[wp] = ent   # nothing ran on the workspace
        return None
    if type(r) is int:
        raise L.SbodError('sbod_criterion_focal failed (%d): %s'
                          % (r, L.lib().sbod_last_error().decode(errors='replace')))
    loss, comps, zb, gmax = r
    _CLEAN[wp] = (zb, None)
    _CRIT_SHAPE[wp] = (B, gmax, P)
    return loss, comps


def criterion_status(device=None):
    """The one-launch criterion's in-launch wait status on ``device`` (current stream's cached
    workspace): 0 = every wait completed.  Synchronises the stream (diagnostics, tests)."""
    dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
    key = (dev if dev.index is not None else torch.device('cuda', torch.cuda.current_device()),
           L._raw_stream(dev.index if dev.index is not None else torch.cuda.current_device()), 'criterion')
    ws = _WS.get(key)
    if ws is None:
        return 0
    return L.lib().sbod_criterion_status(L.ptr(ws), L._raw_stream(key[0].index))


def loss_finish_status(device=None, reset=True):
    """The fused loss finish's sticky word on the current stream's cached loss and criterion
    workspaces (sbod_loss_finish_status): 1 if a bounded gather wait ever gave up there — every
    later loss from that workspace is NaN until its zero-on-entry prefix is zeroed again.  With
    ``reset`` such a workspace is marked not clean, so the next call zeroes it (one memset, outside
    any capture) and computes again.  Synchronises the stream (diagnostics: call it when a fused-
    finish loss reads NaN)."""
    dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
    if dev.index is None:
        dev = torch.device('cuda', torch.cuda.current_device())
    stream = L._raw_stream(dev.index)
    st = 0
    for slot in ('loss', 'criterion'):
        ws = _WS.get((dev, stream, slot))
        if ws is None:
            continue
        if slot == 'loss':
            B, G, P = 1, 0, 1
        else:
            sh = _CRIT_SHAPE.get(ws.data_ptr())
            if sh is None:
                continue
            B, G, P = sh
        r = L.lib().sbod_loss_finish_status(L.ptr(ws), B, G, P, stream)
        if r < 0:
            raise L.SbodError('sbod_loss_finish_status failed (%d): %s'
                              % (r, L.lib().sbod_last_error().decode(errors='replace')))
        if r and reset:
            _CLEAN.pop(ws.data_ptr(), None)
        st |= r
    return st


_POOL_SIZES_OK = set()   # (group, world, B*P) whose equality over the ranks was verified


def allgather_pool(group=None):
    """The data-parallel exchange of MultiBoxLoss300's global mining pool (SSD300.py:580-588):
    every rank's [B*P] pool gathered rank-major over RCCL (B*P*4 bytes per rank; equal B on every
    rank, as a DistributedSampler with drop_last gives).  Returns ``f(pool) -> (pool_all,
    local_off)`` for ``fused_criterion(exchange=...)``.

    The first eager call at a given pool size checks that every rank holds the same B*P (one
    tiny MAX all-reduce of (n, -n) and a host read), so unequal shards fail loudly on every rank
    instead of desynchronising the gather.  Later calls at a verified size — and calls under
    hipGraph capture, whose replays keep the captured shapes — enqueue the gather alone, so a
    data-parallel SSD300 step is capturable (an unverified size under capture raises: run the
    step eagerly once first, as any capture warm-up does)."""
    import torch.distributed as dist

    def exchange(pool):
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        n = pool.numel()
        key = (id(group) if group is not None else None, world, n)
        if key not in _POOL_SIZES_OK:
            if pool.is_cuda and torch.cuda.is_current_stream_capturing():
                raise L.SbodError('sbod global mining under hipGraph capture: the per-rank pool size '
                                  '%d was never verified; run the criterion eagerly once first' % n)
            chk = torch.tensor([n, -n], dtype=torch.int64, device=pool.device)
            dist.all_reduce(chk, op=dist.ReduceOp.MAX, group=group)
            hi, lo = chk.tolist()
            if hi != -lo:
                raise RuntimeError('sbod global mining: ranks hold unequal batches (B*P between %d and %d); '
                                   'use equal per-rank batches (drop_last=True)' % (-lo, hi))
            _POOL_SIZES_OK.add(key)
        out = torch.empty(world * n, dtype=pool.dtype, device=pool.device)
        if dist.get_backend(group) == 'gloo':     # gloo has no all_gather_into_tensor
            parts = [torch.empty_like(pool) for _ in range(world)]
            dist.all_gather(parts, pool, group=group)
            out = torch.cat(parts)
        else:
            dist.all_gather_into_tensor(out, pool, group=group)
        return out, rank * n
    return exchange


def allreduce_npos(n_pos, group=None, force=False):
    """Data parallel: the global positive count (one 4-byte SUM all-reduce over RCCL, enqueued on
    the current stream — no host sync; bench.DPGraph issues it eagerly between the criterion's
    two captured graphs, and tests also capture it whole on one GPU with ``force``).
    Every rank then normalises by the global count, so the per-rank gradients are exactly the
    global-batch gradient's slices.  A one-rank group skips the collective unless
    ``force`` (tests exercise the captured collective on one GPU that way)."""
    import torch.distributed as dist
    tot = n_pos[-1:].clone()
    if dist.is_available() and dist.is_initialized() and (force or dist.get_world_size(group) > 1):
        dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    return tot


# ----------------------------------------------------------------------------- detection
class DetectHandle:
    """An in-flight ``detect``: the kernels are queued on the stream and the per-image counts are
    copied to pinned host memory behind an event.  ``wait()`` blocks on that event only (work
    queued after the detect — e.g. a training backward — keeps running) and returns the lists
    ``detect`` returns.  The inputs must stay alive and unmodified until ``wait()``.

    A handle made under hipGraph capture (``detect(..., capture=True)``) is persistent: its
    outputs and pinned count buffer are the graph's, and after each replay ``replayed()`` arms
    it again (event behind the replay, fresh result lists)."""

    __slots__ = ('_args', '_out', '_cnt_host', '_event', '_full', '_res', '_window', '_launch',
                 '_slot_key', '_persistent', '_stream')

    def __init__(self, args, out, cnt_host, event, full, window, persistent=False):
        self._args, self._out, self._cnt_host, self._event = args, out, cnt_host, event
        self._full, self._res, self._window = full, None, window
        self._persistent = persistent

    def replayed(self, stream=None):
        """After a replay of the graph this handle was captured in: record its event behind the
        replay (on ``stream``, default the current stream) so ``wait()`` returns this replay's
        detections."""
        self._event.record(stream if stream is not None else torch.cuda.current_stream())
        self._res = None
        return self

    def rearmed(self):
        """As ``replayed`` when the event was already recorded behind the replay elsewhere
        (``GtStaging.stage_and_replay``)."""
        self._res = None
        return self

    def wait(self):
        if self._res is not None:
            return self._res
        lc, locs, sc, B, top_k, in_place, debug = self._args
        out_b, out_l, out_s, cnt, dbg_p, dbg_b = self._out
        self._event.synchronize()
        counts = self._cnt_host.tolist()
        if not self._persistent:
            _COUNT_SLOTS.setdefault(self._slot_key, []).append((self._cnt_host, self._event))
        if L.DETECT_CORRUPT in counts:
            raise L.SbodError('detect: a candidate key of image(s) %s decodes to a prior index >= P (corrupted '
                              'or stale detect workspace; its zero-on-entry contract was broken)'
                              % [i for i, n in enumerate(counts) if n == L.DETECT_CORRUPT])
        if min(counts) < 0:   # rare: some image needs a wider candidate window (exactness)
            # The retry reuses the launch's workspace (cached per launch stream), so it runs on
            # THAT stream: a later detect already queued there (pipelined graph replays share
            # the workspace) finishes first and leaves the counters zero, and the retry cannot
            # overlap it.  cnt.cpu() then waits for the retry in that stream's order.
            # (ExternalStream on the launch's device, whatever device is current here)
            with torch.cuda.stream(torch.cuda.ExternalStream(self._stream, device=self._slot_key[0])):
                _detect_launch(*self._launch_args(4096))
                counts = cnt.cpu().tolist()
                if min(counts) < 0:
                    # a class whose survivors a 4,096-candidate window cannot bound (thousands of
                    # near-duplicates): chunked greedy NMS over all of its candidates
                    _detect_launch(*self._launch_args(-1))
                    counts = cnt.cpu().tolist()
            if min(counts) < 0:
                raise L.SbodError('detect: internal error, the exhaustive pass left an image undecided')
        if in_place and lc is not locs:
            locs.copy_(lc)          # models/utils.py:224 clamps the caller's tensor in place
        if min(counts) == top_k:     # every image full (the usual eval case)
            if self._full is None:
                self._full = (list(out_b.unbind(0)), list(out_l.unbind(0)), list(out_s.unbind(0)))
            res = self._full
        else:
            sizes = []
            for n in counts:
                sizes += [n, top_k - n]
            res = (list(out_b.view(B * top_k, 4).split(sizes)[0::2]),
                   list(out_l.view(-1).split(sizes)[0::2]), list(out_s.view(-1).split(sizes)[0::2]))
        self._res = (res, dbg_p, dbg_b) if debug else res
        return self._res

    def _launch_args(self, window):
        return self._launch + (window,)


_COUNT_SLOTS = {}


def _count_slot(dev, B):
    """A free (pinned count buffer, event) pair for a detect of batch B on ``dev``; returned to
    the pool by DetectHandle.wait().  Several handles in flight get separate pairs."""
    free = _COUNT_SLOTS.get((dev, B))
    if free:
        return free.pop()
    return torch.empty(B, dtype=torch.int32, pin_memory=True), torch.cuda.Event()


# Workspaces whose leading counters are known to be zero: data_ptr -> bytes.  sbod_detect_f32
# leaves its candidate counters zero, so after the first call on a workspace no memset is
# needed — none in a captured graph (SBOD_DETECT_COUNTERS_ZEROED).
_CLEAN = {}
_LOSS_ZERO = {}     # (B, P) -> sbod_loss_zero_bytes: the fused finish's words and records


def _loss_zero_bytes(B, P):
    z = _LOSS_ZERO.get((B, P))
    if z is None:
        z = _LOSS_ZERO[(B, P)] = int(L.lib().sbod_loss_zero_bytes(B, P))
    return z


def _zeroed_flag(ws, need, flag, what):
    """``flag`` when the first ``need`` bytes of ``ws`` are known clean (every successful call
    leaves its zero-on-entry prefix zero), else 0 (the call zeroes them itself: a memset, which
    must not be captured)."""
    ent = _CLEAN.get(ws.data_ptr())
    if ent is not None and ent[0] >= need:
        return flag
    if torch.cuda.is_current_stream_capturing():
        raise L.SbodError('%s under hipGraph capture: run it once on the capture stream with this '
                          'shape first (its workspace counters are not known to be zero)' % what)
    return 0


def reserve_count_slots(dev, B, n):
    """Make ``n`` (pinned count buffer, event) pairs available for detects of batch B on ``dev``
    — e.g. before capturing ``n`` graphs, since pinned memory cannot be allocated under capture."""
    free = _COUNT_SLOTS.setdefault((dev, B), [])
    while len(free) < n:
        free.append((torch.empty(B, dtype=torch.int32, pin_memory=True), torch.cuda.Event()))


_DET_SIZES = {}   # (B, P, C) -> (workspace bytes, counter bytes)


def _det_sizes(B, P, C):
    v = _DET_SIZES.get((B, P, C))
    if v is None:
        lib = L.lib()
        v = _DET_SIZES[(B, P, C)] = (lib.sbod_detect_workspace_bytes(B, P, C), lib.sbod_detect_counter_bytes(B, C))
    return v


def _detect_launch(lc, sc, B, P, C, pri, pm, box_type, act, min_score, max_overlap, top_k, fn, out,
                   dbg, ws, nb, cnt_host, in_flags, window):
    out_b, out_l, out_s, cnt = out
    need = _det_sizes(B, P, C)[1]
    flags = _zeroed_flag(ws, need, L.DETECT_COUNTERS_ZEROED, 'detect') | in_flags
    # a call that fails part-way can leave its counters non-zero (k_det_prepare has added to
    # them, k_det_merge never ran): the workspace counts as clean again only after a success
    _CLEAN.pop(ws.data_ptr(), None)
    L.call('sbod_detect_f32', L.ptr(lc), L.ptr(sc), B, P, C, L.ptr(pri), L.ptr(pm), L.BOX[box_type],
           L.ACT[act], float(min_score), float(max_overlap), int(top_k), fn, int(window), flags,
           L.ptr(out_b), L.ptr(out_l), L.ptr(out_s), L.ptr(cnt), L.ptr(cnt_host), L.ptr(dbg[0]),
           L.ptr(dbg[1]), L.ptr(ws), nb, L.stream_of(sc))
    # only this call's prefix is known clean: a call with a smaller B * C writes other regions
    # over the rest of a larger one's counters
    _CLEAN[ws.data_ptr()] = (need, None)


# The per-class NMS and the per-image merge as two launches (k_det_segment_w4, k_det_merge with
# its inline second window) or as one (k_det_nms, the image's last class merges): the default of
# ``detect(two_pass=None)``, chosen by the same-box A/B in DESIGN.md round 4.
DETECT_TWO_PASS = True


def detect(locs, scores, min_score, max_overlap, top_k, priors_cxcy, box_type='offset',
           act='softmax', pos_mask=None, final_nms=None, debug=False, window=0, async_=False,
           capture=False, two_pass=None):
    """Batched decode + per-class NMS + top-k.  Returns (boxes, labels, scores) lists of per-image
    tensors (views of batched device outputs).  ONE host sync: the per-image counts (waited on
    through an event).  ``async_=True`` returns a ``DetectHandle`` instead (``.wait()`` gives the
    lists), so a caller can overlap the detect kernels with later host work.  ``capture=True``
    (inside hipGraph capture) returns a persistent handle: call ``.replayed()`` after each replay,
    then ``.wait()``.  ``two_pass`` (None: the module default
    ``DETECT_TWO_PASS``) runs the per-class NMS and the per-image merge as two launches (with the
    inline second window) or, False, as one (k_det_nms)."""
    L.require_device(locs, scores, what='detect')
    B, P, C = scores.shape
    if top_k <= 0:
        raise ValueError('top_k must be positive')
    dev = scores.device
    in_place = box_type not in ('offset', 'center')
    if scores.dtype == torch.bfloat16 and locs.dtype == torch.bfloat16 and C <= 32:
        # bf16 activations read as they are (widened exactly in the kernel, SBOD_DETECT_INPUT_BF16):
        # the results of detect on their fp32 values, without widened copies
        sc, lc, in_flags = scores.contiguous(), locs.contiguous(), L.DETECT_INPUT_BF16
    else:
        sc = scores.contiguous().float()
        lc = locs if (locs.is_contiguous() and locs.dtype == torch.float32) else locs.contiguous().float()
        in_flags = 0
    if not (DETECT_TWO_PASS if two_pass is None else two_pass):
        in_flags |= L.DETECT_FUSED
    pri = priors_cxcy.contiguous().float() if priors_cxcy is not None else None
    pm = pos_mask.contiguous().to(torch.uint8) if pos_mask is not None else None
    out_b = torch.empty(B, top_k, 4, dtype=torch.float32, device=dev)
    out_l = torch.empty(B, top_k, dtype=torch.int64, device=dev)
    out_s = torch.empty(B, top_k, dtype=torch.float32, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    dbg_p = torch.empty(B, P, C, dtype=torch.float32, device=dev) if debug else None
    dbg_b = torch.empty(B, P, 4, dtype=torch.float32, device=dev) if debug else None
    nb = _det_sizes(B, P, C)[0]
    ws = workspace(nb, dev, 'detect')
    fn = -1.0 if final_nms is None else float(final_nms)
    # counts -> pinned host memory (written by the last detect kernel itself) behind an event,
    # both cached per (device, B): a pinned allocation per call goes through hipHostMalloc / the
    # host allocator's event bookkeeping and stalls the launching thread for the whole queue
    if capture:
        # owned by the graph from now on (its last kernel writes this buffer on every replay);
        # pinned memory cannot be allocated under capture, so it comes from the pool an eager
        # warm-up call filled
        free = _COUNT_SLOTS.get((dev, B))
        if not free:
            raise L.SbodError('detect(capture=True): run detect eagerly once with this batch size '
                              'before capturing (warm-up), so its pinned count buffer exists')
        cnt_host, ev = free.pop()
    else:
        cnt_host, ev = _count_slot(dev, B)
    launch = (lc, sc, B, P, C, pri, pm, box_type, act, min_score, max_overlap, top_k, fn,
              (out_b, out_l, out_s, cnt), (dbg_p, dbg_b), ws, nb, cnt_host, in_flags)
    _detect_launch(*launch, window)
    raw = L._raw_stream(dev.index)   # the stream whose workspace the launch used
    if not capture:
        ce = ev.cuda_event   # 0 until torch creates the event at its first record
        if ce:
            L.call('sbod_event_record', ce, raw)
        else:
            ev.record(torch.cuda.current_stream(dev))
    # the per-image views for the usual all-full case: built while the kernels run when the call
    # waits for them itself, else by wait() (a pipelined caller collects them later anyway)
    full = (list(out_b.unbind(0)), list(out_l.unbind(0)), list(out_s.unbind(0))) if not async_ else None
    h = DetectHandle((lc, locs, sc, B, top_k, in_place, debug), (out_b, out_l, out_s, cnt, dbg_p, dbg_b),
                     cnt_host, ev, full, window, persistent=capture)
    h._launch = launch
    h._slot_key = (dev, B)
    h._stream = raw
    return h if (async_ or capture) else h.wait()


def nms(boxes, scores, overlap, top_k=0, variant='tv', beta1=1.0):
    """Single-segment greedy NMS on the device. Returns (keep [n] int64 zero-padded, count tensor)."""
    L.require_device(boxes, scores, what='nms')
    n = boxes.shape[0]
    b = boxes.contiguous().float()
    s = scores.contiguous().float()
    keep = torch.empty(n, dtype=torch.int64, device=boxes.device)
    count = torch.empty(1, dtype=torch.int32, device=boxes.device)
    nb = L.lib().sbod_nms_workspace_bytes(n)
    ws = workspace(nb, boxes.device, 'nms')
    L.call('sbod_nms_f32', L.ptr(b), L.ptr(s), n, float(overlap), int(top_k), L.NMS[variant],
           float(beta1), L.ptr(keep), L.ptr(count), L.ptr(ws), nb, L.stream_of(b))
    return keep, count


# ----------------------------------------------------------------------------- standalone losses
class _RowOp(torch.autograd.Function):
    """Per-row values + per-row local derivative from one kernel; backward = grad_out * local."""

    @staticmethod
    def forward(ctx, x, run, want):
        val, local = run(want)
        ctx.save_for_backward(local)
        return val

    @staticmethod
    def backward(ctx, g):
        (local,) = ctx.saved_tensors
        if local is None:
            return None, None, None
        while g.dim() < local.dim():
            g = g.unsqueeze(-1)
        return g * local, None, None


class _Overlap(torch.autograd.Function):
    """Row-wise overlap [n] of two box sets; the kernel writes the local derivatives w.r.t. both
    (iou_utils.py:6-164 lets autograd reach both), backward scales them by the upstream grad."""

    @staticmethod
    def forward(ctx, x1, x2, run, want1, want2):
        val, g1, g2 = run(want1, want2)
        ctx.save_for_backward(g1, g2)
        return val

    @staticmethod
    def backward(ctx, g):
        g1, g2 = ctx.saved_tensors
        g = g.unsqueeze(-1)
        return (g * g1 if g1 is not None else None), (g * g2 if g2 is not None else None), None, None, None


def aligned_overlap(kind, b1, b2):
    """Row-wise IoU / GIoU / DIoU / CIoU [n] with autograd w.r.t. both box sets."""
    L.require_device(b1, b2, what='bbox_overlaps')
    n = b1.shape[0]
    x1, x2 = b1.contiguous().float(), b2.contiguous().float()

    def run(want1, want2):
        ov = torch.empty(n, dtype=torch.float32, device=b1.device)
        g1 = torch.empty(n, 4, dtype=torch.float32, device=b1.device) if want1 else None
        g2 = torch.empty(n, 4, dtype=torch.float32, device=b1.device) if want2 else None
        L.call('sbod_aligned_overlap_f32', L.OV[kind], L.ptr(x1), L.ptr(x2), n, L.ptr(ov), L.ptr(g1),
               L.ptr(g2), L.stream_of(x1))
        return ov, g1, g2

    grad_on = torch.is_grad_enabled()
    return _Overlap.apply(x1, x2, run, grad_on and b1.requires_grad, grad_on and b2.requires_grad)


def smooth_l1_elementwise(pred, target, beta):
    L.require_device(pred, target, what='SmoothL1Loss')
    p, t = pred.contiguous().float(), target.contiguous().float()
    if p.shape != t.shape:
        p, t = torch.broadcast_tensors(p, t)
        p, t = p.contiguous(), t.contiguous()
    n = p.numel()

    def run(want):
        loss = torch.empty_like(p)
        g = torch.empty_like(p) if want else None
        L.call('sbod_smooth_l1_f32', L.ptr(p), L.ptr(t), n, float(beta), L.ptr(loss), L.ptr(g),
               L.stream_of(p))
        return loss, g

    grad_on = torch.is_grad_enabled()
    return _SmoothL1.apply(p, t, run, grad_on and pred.requires_grad, grad_on and target.requires_grad)


class _SmoothL1(torch.autograd.Function):
    """Element-wise smooth-L1 of (pred - target): one kernel gives the loss and d/dpred; the
    target's derivative is its negation (nn.SmoothL1Loss propagates to both inputs)."""

    @staticmethod
    def forward(ctx, p, t, run, want_p, want_t):
        val, local = run(want_p or want_t)
        ctx.want = (want_p, want_t)
        ctx.save_for_backward(local)
        return val

    @staticmethod
    def backward(ctx, g):
        (local,) = ctx.saved_tensors
        if local is None:
            return None, None, None, None, None
        gl = g * local
        return (gl if ctx.want[0] else None), (-gl if ctx.want[1] else None), None, None, None


def focal_rows(kind, logits, target, alpha_fg, alpha_bg, gamma):
    """Per-row focal loss [rows] (softmax / sigmoid / bce forms) with autograd w.r.t. logits."""
    L.require_device(logits, target, what='focal')
    z = logits.contiguous().float()
    y = target.contiguous().to(torch.int64)
    rows, C = z.shape

    def run(want):
        loss = torch.empty(rows, dtype=torch.float32, device=z.device)
        g = torch.empty_like(z) if want else None
        L.call('sbod_focal_f32', L.FOCAL[kind], L.ptr(z), L.ptr(y), rows, C, float(alpha_fg),
               float(alpha_bg), float(gamma), L.ptr(loss), L.ptr(g), L.stream_of(z))
        return loss, g

    want = torch.is_grad_enabled() and logits.requires_grad
    return _RowOp.apply(z, run, want)


# ----------------------------------------------------------------------------- a14: DeformConv2d
class _DeformConv(torch.autograd.Function):
    """out = DCN(x, offset, sigmoid(mask_logits), weight) on the HIP path.

    A training forward (any input needs a gradient) runs ``sbod_dcn_fwd_train_f32`` into a
    per-call STATE buffer that autograd keeps until the backward: the coefficients, channels-last
    x, both weight layouts and the per-input-pixel sample counts, so ``sbod_dcn_bwd_state_f32``
    re-derives none of them (six launches for all four gradients; the state is read-only there,
    so a retained graph's second backward sees the same state).  An inference forward takes the
    forward-only workspace (no state kept)."""

    @staticmethod
    def forward(ctx, x, offset, mask_logits, weight, ks, padding, stride):
        B, C, H, W = x.shape
        O = weight.shape[0]
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        if tuple(offset.shape) != (B, 2 * ks * ks, Ho, Wo):
            raise ValueError('DeformConv2d: offset shape %s, expected %s'
                             % (tuple(offset.shape), (B, 2 * ks * ks, Ho, Wo)))
        if mask_logits is not None and tuple(mask_logits.shape) != (B, ks * ks, Ho, Wo):
            raise ValueError('DeformConv2d: mask shape %s' % (tuple(mask_logits.shape),))
        if tuple(weight.shape) != (O, C, ks, ks):
            raise ValueError('DeformConv2d: weight shape %s' % (tuple(weight.shape),))
        out = torch.empty(B, O, Ho, Wo, dtype=torch.float32, device=x.device)
        dims = (B, C, H, W, O, ks, stride, padding)
        ctx.cfg = dims
        ctx.modulated = mask_logits is not None
        if any(ctx.needs_input_grad[:4]):
            nb = L.lib().sbod_dcn_state_bytes(*dims)
            state = torch.empty(nb, dtype=torch.uint8, device=x.device)
            L.call('sbod_dcn_fwd_train_f32', L.ptr(x), L.ptr(offset), L.ptr(mask_logits), L.ptr(weight), *dims,
                   L.ptr(out), L.ptr(state), nb, L.stream_of(x))
            ctx.save_for_backward(state)
        else:
            nb = L.lib().sbod_dcn_fwd_workspace_bytes(*dims)
            ws = workspace(nb, x.device, 'dcn')
            L.call('sbod_dcn_fwd_f32', L.ptr(x), L.ptr(offset), L.ptr(mask_logits), L.ptr(weight), *dims,
                   L.ptr(out), L.ptr(ws), nb, L.stream_of(x))
        return out

    @staticmethod
    def backward(ctx, gout):
        state, = ctx.saved_tensors
        B, C, H, W, O, ks, stride, padding = dims = ctx.cfg
        g = gout.contiguous().float()
        if g.data_ptr() % 16:          # the weight-gradient kernel reads grad_out as float4
            g = g.clone()
        need = ctx.needs_input_grad
        dev = state.device
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        gx = torch.empty(B, C, H, W, dtype=torch.float32, device=dev) if need[0] else None
        goff = torch.empty(B, 2 * ks * ks, Ho, Wo, dtype=torch.float32, device=dev) if need[1] else None
        gm = (torch.empty(B, ks * ks, Ho, Wo, dtype=torch.float32, device=dev)
              if (ctx.modulated and need[2]) else None)
        gw = torch.empty(O, C, ks, ks, dtype=torch.float32, device=dev) if need[3] else None
        nb = L.lib().sbod_dcn_scratch_bytes(*dims)
        ws = workspace(nb, dev, 'dcn_scratch')
        L.call('sbod_dcn_bwd_state_f32', L.ptr(g), *dims, L.ptr(gx), L.ptr(goff), L.ptr(gm), L.ptr(gw),
               L.ptr(state), state.numel(), L.ptr(ws), nb, L.stream_of(g))
        return gx, goff, gm, gw, None, None, None


def deform_conv2d(x, offset, mask_logits, weight, ks=3, padding=1, stride=1):
    """Modulated deformable conv (Deformable_convolution.py:33-91) given the p_conv output
    ``offset`` [B,2k²,Ho,Wo] and the m_conv output BEFORE sigmoid ``mask_logits`` [B,k²,Ho,Wo]
    (None: modulation=False).  fp32 in, fp32 out."""
    L.require_device(x, offset, weight, what='DeformConv2d')
    c = lambda t: None if t is None else t.contiguous().float()
    return _DeformConv.apply(c(x), c(offset), c(mask_logits), c(weight), int(ks), int(padding),
                             int(stride))
