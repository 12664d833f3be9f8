"""Host-time breakdown of one bench step on the GPU box, without profiler overhead: each piece
is timed over many iterations with perf_counter (GPU work runs asynchronously behind it; a
synchronize between pieces isolates host cost from queueing effects)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import core  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR, utils as MU  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402

dev = torch.device('cuda')
Pn = prior_table('SSD512')
P = Pn.shape[0]
pri = torch.from_numpy(Pn).to(dev)
cfg = bench.Cfg(reg_weights=1.0, device=dev, n_classes=21, reg_loss='diou', cls_loss='focal',
                focal_type='softmax', model={'box_type': 'offset'})
crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
boxes, labels, locs0, scores0, det = bench.make_batch(32, 0, dev)
locs = locs0.clone().requires_grad_(True)
scores = scores0.clone().requires_grad_(True)
N = 300


def host_time(fn, n=N):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(n):
        t = time.perf_counter()
        fn()
        tot += time.perf_counter() - t
        torch.cuda.synchronize()
    return round(tot / n * 1e6, 2)


res = {}
res['pack_gt'] = host_time(lambda: core.pack_gt(boxes, labels))
gt = core.pack_gt(boxes, labels)
res['match'] = host_time(lambda: core.match(gt, crit.priors_xy, P, 0.5))
obj, ovl, npos = core.match(gt, crit.priors_xy, P, 0.5)
spec = crit._spec()


def fused():
    locs.grad = None
    scores.grad = None
    return core.fused_criterion(locs, scores, gt, obj, ovl, npos, npos[32:], pri, spec, 0.5, 0.4)[0]


res['fused_fwd'] = host_time(fused)


def fwd():
    locs.grad = None
    scores.grad = None
    return crit(locs, scores, boxes, labels)


res['criterion_fwd'] = host_time(fwd)
holder = []


def mk():
    holder.append(fwd())


def bwd():
    holder.pop().backward()


for _ in range(10):
    mk()
    bwd()
torch.cuda.synchronize()
tb = 0.0
for _ in range(N):
    mk()
    torch.cuda.synchronize()
    t = time.perf_counter()
    bwd()
    tb += time.perf_counter() - t
    torch.cuda.synchronize()
res['backward'] = round(tb / N * 1e6, 2)
res['detect_api_incl_sync'] = host_time(lambda: MU.detect(locs.detach(), det, 0.01, 0.45, 200, pri, cfg))
res['empty_x4'] = host_time(lambda: [torch.empty(32, P, dtype=torch.int32, device=dev) for _ in range(4)])
print(json.dumps(res))


# autograd floor: a Python Function whose backward just hands back a preallocated gradient
class _Trivial(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.g = torch.empty_like(x)
        return x.new_zeros(())

    @staticmethod
    def backward(ctx, g):
        r = ctx.g
        ctx.g = None
        return r


xs = locs0.clone().requires_grad_(True)
tt = 0.0
for it in range(N + 10):
    xs.grad = None
    y = _Trivial.apply(xs)
    torch.cuda.synchronize()
    t = time.perf_counter()
    y.backward()
    if it >= 10:
        tt += time.perf_counter() - t
    torch.cuda.synchronize()
res2 = {'trivial_function_backward': round(tt / N * 1e6, 2)}
print(json.dumps(res2))
