"""Data-parallel sharding on CPU (gloo, world_size 2): each rank owns half the images, the batch
positive count is SUM-all-reduced through ``core.allreduce_npos`` (the same call the criteria use
over RCCL), and every rank normalises by it.  Then the sum of the shard losses equals the
single-process loss and every rank's gradients equal its slice of the full-batch gradients
(SURVEY §8(e)).  The loss arithmetic is the oracle's (the HIP kernels are covered by -m gpu)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import loss_ref as LR
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models.priors import prior_table

B, C = 4, 21


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, reg, cls, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        P = torch.from_numpy(prior_table('SSD300')[::3].copy())
        boxes, labels = synth.make_gt(B, seed=77)
        locs, scores = synth.make_preds(B, P.shape[0], C, seed=77)
        sl = slice(rank * B // world, (rank + 1) * B // world)
        my_boxes, my_labels = boxes[sl], labels[sl]
        n_local = LR.local_npos(P, my_boxes, my_labels)
        npos = torch.tensor([0, n_local], dtype=torch.int32)   # [per-image..., total] layout
        tot = core.allreduce_npos(npos)                          # the criteria's exchange step
        lo = locs[sl].clone().requires_grad_(True)
        sc = scores[sl].clone().requires_grad_(True)
        loss = LR.criterion(kind, P, lo, sc, my_boxes, my_labels, reg, cls, npos_total=int(tot.item()))
        loss.backward()
        total = loss.detach().clone()
        dist.all_reduce(total)
        out_q.put((rank, float(total), int(tot.item()), lo.grad.numpy(), sc.grad.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('kind,reg,cls', [('ssd512', 'diou', 'focal'), ('retina', 'smoothl1', 'ce'),
                                          ('ssd512', 'smoothl1', 'ce')])
def test_dp_shards_match_single_process(kind, reg, cls):
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, reg, cls, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    P = torch.from_numpy(prior_table('SSD300')[::3].copy())
    boxes, labels = synth.make_gt(B, seed=77)
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=77)
    lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    ref = LR.criterion(kind, P, lo, sc, boxes, labels, reg, cls)
    ref.backward()
    assert res[0][2] == res[1][2] == LR.local_npos(P, boxes, labels)
    np.testing.assert_allclose(res[0][1], ref.item(), rtol=1e-5)
    np.testing.assert_allclose(np.concatenate([r[3] for r in res]), lo.grad.numpy(), rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(np.concatenate([r[4] for r in res]), sc.grad.numpy(), rtol=1e-5, atol=1e-9)


def _worker_global_pool(rank, world, port, out_q):
    """MultiBoxLoss300 CE: hard negatives are mined over the WHOLE batch (SSD300.py:580-588), so
    the ranks exchange their pools through ``core.allgather_pool`` (the criteria's exchange
    step) and each mines its rows of the global top-k."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        P = torch.from_numpy(prior_table('SSD300')[::3].copy())
        boxes, labels = synth.make_gt(B, seed=78)
        locs, scores = synth.make_preds(B, P.shape[0], C, seed=78)
        sl = slice(rank * B // world, (rank + 1) * B // world)
        my_boxes, my_labels = boxes[sl], labels[sl]
        npos = torch.tensor([0, LR.local_npos(P, my_boxes, my_labels)], dtype=torch.int32)
        tot = int(core.allreduce_npos(npos).item())
        pool = LR.ssd300_pool(P, scores[sl], my_boxes, my_labels)
        pool_all, off = core.allgather_pool()(pool)
        lo = locs[sl].clone().requires_grad_(True)
        sc = scores[sl].clone().requires_grad_(True)
        loss = LR.criterion('ssd300', P, lo, sc, my_boxes, my_labels, 'l1', 'ce', npos_total=tot,
                            pool_all=pool_all, local_off=off)
        loss.backward()
        total = loss.detach().clone()
        dist.all_reduce(total)
        out_q.put((rank, float(total), off, lo.grad.numpy(), sc.grad.numpy()))
    finally:
        dist.destroy_process_group()


def test_dp_ssd300_global_mining_exchange():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_global_pool, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    P = torch.from_numpy(prior_table('SSD300')[::3].copy())
    boxes, labels = synth.make_gt(B, seed=78)
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=78)
    lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    ref = LR.criterion('ssd300', P, lo, sc, boxes, labels, 'l1', 'ce')
    ref.backward()
    assert [r[2] for r in res] == [0, (B // world) * P.shape[0]]
    np.testing.assert_allclose(res[0][1], ref.item(), rtol=1e-5)
    np.testing.assert_allclose(np.concatenate([r[3] for r in res]), lo.grad.numpy(), rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(np.concatenate([r[4] for r in res]), sc.grad.numpy(), rtol=1e-5, atol=1e-9)


def _worker_criterion_class(rank, world, port, kind, reg, cls, out_q):
    """The drop-in criterion CLASS with ``distributed = True`` over gloo, through a CPU seam: its
    orchestration runs unchanged, only the device entry points it calls (pack_gt, match,
    fused_criterion) are oracle-backed CPU stand-ins.  Shared 'network' parameters theta feed
    every rank's predictions, and their gradients are AVERAGED over ranks as DDP does."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from shape_based_object_detection_amd import _lib as L
        from shape_based_object_detection_amd.models import criteria as CR
        P = torch.from_numpy(prior_table('SSD300')[::3].copy())
        calls = []
        reg_name = {v: k for k, v in L.REG.items()}
        cls_name = {v: k for k, v in L.CLS.items()}
        L.require_device = lambda *a, **k: None
        core.pack_gt = lambda boxes, labels, **k: (list(boxes), list(labels))

        def match(gt, anchors, n_priors, threshold=0.5, flags=0, **k):
            calls.append('match')
            n = LR.local_npos(P, gt[0], gt[1], threshold)
            return None, None, torch.tensor([0] * len(gt[0]) + [n], dtype=torch.int32)

        real_ar, real_ag = core.allreduce_npos, core.allgather_pool

        def allreduce_npos(npos, group=None, force=False):
            calls.append('allreduce_npos')
            return real_ar(npos, group, force)

        def allgather_pool(group=None):
            calls.append('allgather_pool')
            return real_ag(group)

        def fused(locs, scores, gt, obj, ovl, n_pos, npos_total, priors_cxcy, spec, thr, nthr,
                  exchange=None, **k):
            boxes, labels = gt
            kw = {}
            if exchange is not None:
                pool = LR.ssd300_pool(P, scores.detach(), boxes, labels, thr)
                kw['pool_all'], kw['local_off'] = exchange(pool)
            loss = LR.criterion(kind, P, locs, scores, boxes, labels, reg_name[spec.reg], cls_name[spec.cls],
                                threshold=thr, npos_total=int(npos_total.item()), **kw)
            return loss, None

        core.match, core.fused_criterion = match, fused
        core.allreduce_npos, core.allgather_pool = allreduce_npos, allgather_pool
        cls_of = {'ssd512': CR.MultiBoxLoss512, 'ssd300': CR.MultiBoxLoss300, 'retina': CR.RetinaFocalLoss}
        crit = cls_of[kind](priors_cxcy=P, config=dict(reg_weights=1.0, device='cpu', n_classes=C,
                                                       reg_loss=reg, cls_loss=cls))
        crit.distributed = True
        boxes, labels = synth.make_gt(B, seed=79)
        locs, scores = synth.make_preds(B, P.shape[0], C, seed=79)
        sl = slice(rank * B // world, (rank + 1) * B // world)
        th_l = torch.zeros(4, requires_grad=True)
        th_s = torch.zeros(C, requires_grad=True)
        loss = crit(locs[sl] + th_l, scores[sl] + th_s, boxes[sl], labels[sl])
        loss.backward()
        gl, gs = th_l.grad.clone(), th_s.grad.clone()
        for g in (gl, gs):           # DDP: gradient all-reduce, averaged over ranks
            dist.all_reduce(g)
            g /= world
        mean_loss = loss.detach().clone()
        dist.all_reduce(mean_loss)
        mean_loss /= world
        out_q.put((rank, calls, float(mean_loss), gl.numpy(), gs.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('kind,reg,cls', [('ssd512', 'diou', 'focal'), ('ssd300', 'smoothl1', 'ce'),
                                          ('retina', 'smoothl1', 'ce')])
def test_dp_criterion_class_ddp_mean(kind, reg, cls):
    """criterion.distributed = True: the class makes the exchange calls (positive-count all-reduce;
    SSD300 CE also the pool all-gather), and with DDP's gradient AVERAGING the shared parameters'
    gradient and the mean loss equal the single-process batch's."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_criterion_class, args=(r, world, port, kind, reg, cls, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = ['match', 'allreduce_npos'] + (['allgather_pool'] if kind == 'ssd300' else [])
    assert all(r[1] == want for r in res), [r[1] for r in res]
    P = torch.from_numpy(prior_table('SSD300')[::3].copy())
    boxes, labels = synth.make_gt(B, seed=79)
    locs, scores = synth.make_preds(B, P.shape[0], C, seed=79)
    th_l = torch.zeros(4, requires_grad=True)
    th_s = torch.zeros(C, requires_grad=True)
    oreg = 'l1' if (kind == 'ssd300' and reg == 'smoothl1') else reg
    ref = LR.criterion(kind, P, locs + th_l, scores + th_s, boxes, labels, oreg, cls)
    ref.backward()
    np.testing.assert_allclose(res[0][2], ref.item(), rtol=1e-5)
    np.testing.assert_allclose(res[0][3], th_l.grad.numpy(), rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(res[0][4], th_s.grad.numpy(), rtol=1e-4, atol=1e-7)
