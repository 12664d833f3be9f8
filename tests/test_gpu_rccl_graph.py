"""RCCL collectives of the data-parallel criteria, captured into a hipGraph, on one GPU.

A one-rank ``nccl`` (= RCCL) process group with ``force_collectives`` makes the criteria run the
same collectives a multi-GPU rank runs (the n_pos SUM all-reduce, core.allreduce_npos; for
MultiBoxLoss300's CE the pool all-gather of the global mining exchange, core.allgather_pool,
SSD300.py:580-588).  The criterion forward+backward is then captured into a hipGraph on a side
stream and replayed: the replay's loss and gradients must equal the eager call's bit for bit
(same kernels, deterministic reductions), and equal the non-distributed criterion's (a one-rank
sum is the identity).
"""
import socket

import numpy as np
import pytest
import torch

from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


class Cfg(dict):
    __getattr__ = dict.__getitem__


@pytest.fixture(scope='module')
def nccl_group():
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip('a process group is already initialised in this process')
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(DEV)
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1,
                            device_id=DEV)
    yield dist.group.WORLD
    dist.destroy_process_group()


def _run(crit, locs, scores, gt, one):
    locs.grad = None
    scores.grad = None
    loss = crit(locs, scores, gt, None)
    loss.backward(one)
    return loss


@pytest.mark.parametrize('arch,reg,cls', [('SSD512', 'diou', 'focal'), ('SSD300', 'l1', 'ce')])
def test_criterion_with_rccl_collectives_captured(nccl_group, arch, reg, cls):
    B, C = 8, 21
    pri = torch.from_numpy(prior_table(arch)).to(DEV)
    P = pri.shape[0]
    boxes, labels = synth.make_gt(B, seed=31, n_classes=C)
    l0, s0 = synth.make_preds(B, P, C, seed=31)
    cfg = Cfg(reg_weights=1.0, device=DEV, n_classes=C, reg_loss=reg, cls_loss=cls)
    kls = CR.MultiBoxLoss512 if arch == 'SSD512' else CR.MultiBoxLoss300
    plain = kls(priors_cxcy=pri, config=cfg)
    crit = kls(priors_cxcy=pri, config=cfg)
    crit.distributed = True
    crit.force_collectives = True
    locs = l0.to(DEV).requires_grad_(True)
    scores = s0.to(DEV).requires_grad_(True)
    one = core.unit_grad(DEV)
    stage = core.GtStaging(B, 16, DEV)
    dev_boxes = [b.to(DEV) for b in boxes]
    dev_labels = [l.to(DEV) for l in labels]

    gt = stage.stage(dev_boxes, dev_labels)
    ref = _run(plain, locs, scores, gt, one).item()
    ref_gl, ref_gs = locs.grad.clone(), scores.grad.clone()

    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        for _ in range(2):     # warm-up: workspaces, the communicator, the pool-size check
            gt = stage.stage(dev_boxes, dev_labels)
            eager = _run(crit, locs, scores, gt, one)
    torch.cuda.current_stream(DEV).wait_stream(side)
    torch.cuda.synchronize()
    eager_v = eager.item()
    eager_gl, eager_gs = locs.grad.clone(), scores.grad.clone()
    assert eager_v == ref
    assert torch.equal(eager_gl, ref_gl) and torch.equal(eager_gs, ref_gs)

    locs.grad = None
    scores.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        loss = crit(locs, scores, gt, None)
        loss.backward(one)
    for _ in range(3):
        stage.stage(dev_boxes, dev_labels)
        g.replay()
    torch.cuda.synchronize()
    assert loss.item() == eager_v
    assert torch.equal(locs.grad, eager_gl)
    assert torch.equal(scores.grad, eager_gs)
    np.testing.assert_allclose(loss.item(), ref, rtol=0)
