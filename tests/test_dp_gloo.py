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
