#!/usr/bin/env python3
"""Throughput of the sbod hot path on MI355X (contract: one JSON line on rank 0).

One step = one pass of the hot path over one batch of SSD512 synthetic input resident in HBM
(SURVEY §8(d) recipe; BASELINE.json metric "images/sec train step SSD512 batch=32"):
  1. MultiBoxLoss512 (DIoU box loss + softmax focal, the configs[1] losses) forward AND
     backward through the drop-in criterion: ground-truth packing, the HIP matcher, the fused
     loss+gradient pass, and the upstream-gradient application;
  2. detect on the same batch (softmax, offset decode + clamp, per-class NMS at IoU 0.45,
     min_score 0.01, top_k 200 — models.utils.detect's work), whose per-image lists need one
     device->host sync.  Its kernels are queued between the criterion's forward and backward
     (core.detect(async_=True)) so they run under the backward's host work; the lists are
     collected at the end of the step.  --sync-detect: models.utils.detect after the backward.
Per-GPU batch is fixed (weak scaling); with N > 1 every rank owns its images and the loss
normaliser (batch positives) is SUM-all-reduced over RCCL each step, as data-parallel training
needs for exact single-device parity.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from shape_based_object_detection_amd import _lib as L  # noqa: E402
from shape_based_object_detection_amd import core, synth  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402
from shape_based_object_detection_amd.models import utils as MU  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
N_CLASSES = 21
ARCH = 'SSD512'


class Cfg(dict):
    __getattr__ = dict.__getitem__


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-sample-images', type=int, default=2)
    ap.add_argument('--sync-detect', action='store_true',
                    help='run detect after the backward, synchronously (no overlap of its kernels '
                         'with the backward host work)')
    return ap.parse_args()


def make_batch(B, seed, dev):
    P = prior_table(ARCH).shape[0]
    boxes, labels = synth.make_gt(B, seed=seed, n_classes=N_CLASSES)
    locs, scores = synth.make_preds(B, P, N_CLASSES, seed=seed)
    det_scores = scores.clone()
    det_scores[:, :, 0] += 6.0            # detection workload: +6 background logit (§8(d))
    return ([b.to(dev) for b in boxes], [l.to(dev) for l in labels], locs.to(dev), scores.to(dev),
            det_scores.to(dev))


def bytes_per_step(B, P, C):
    """Algorithmic HBM bytes of the fused loss pass: read locs+scores once,
    write their gradients once, priors once per batch."""
    return B * P * 2 * (4 + C) * 4 + 16 * P


# Algorithmic HBM bytes per launch of the streaming (HBM-bound) kernels of one step (DESIGN.md
# "Kernels"): every input read once, every output written once.  w = workload constants.
ALGO_BYTES = {
    # scores [B,P,C] + locs [B,P,4] + priors [P,4] read; decoded boxes [B,P,4] and the
    # candidate keys (8 B each) + per-(image, class) counts written
    'k_det_prepare': lambda w: w['B'] * w['P'] * (4 * w['C'] + 16 + 16) + 16 * w['P']
                               + 8 * w['n_cand'] + 4 * w['B'] * w['C'],
    # locs + scores read, their gradients written, matcher obj (i32) + overlap (f32) read,
    # the hard-negative pool (f32) written, priors read once
    'k_multibox': lambda w: w['B'] * w['P'] * (2 * (16 + 4 * w['C']) + 12) + 16 * w['P'],
    # priors read per image tile, obj + overlap written, per-tile per-object partial keys (u64)
    'k_match_tile': lambda w: w['B'] * w['P'] * (16 + 8) + w['B'] * ((w['P'] + 255) // 256) * w['Gmax'] * 8,
}
HBM_KERNELS = tuple(ALGO_BYTES)
ALL_KERNELS = HBM_KERNELS + ('k_det_segment', 'k_det_merge', 'k_match_final', 'k_hnm')
TIMING_EVERY = 10
PMC_FILE = os.path.join(HERE, 'profiles', 'pmc_traffic.json')


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (FETCH_SIZE and
    WRITE_SIZE collected in separate passes; FETCH doubled on gfx950, KB -> bytes), or None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        return d['kernels'][kernel]['traffic_bytes_per_launch']
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(B_sample, threads):
    """The oracle (CPU restatement of the reference, pinned by tests/golden) on host cores:
    criterion fwd+bwd on B_sample images + detect on B_sample images.  kind = 'port'."""
    import numpy as np
    from oracle import loss_ref as LR
    from oracle import match_ref as M
    torch.set_num_threads(threads)
    Pn = prior_table(ARCH)
    P = torch.from_numpy(Pn)
    boxes, labels = synth.make_gt(B_sample, seed=0, n_classes=N_CLASSES)
    locs, scores = synth.make_preds(B_sample, Pn.shape[0], N_CLASSES, seed=0)
    det = scores.clone()
    det[:, :, 0] += 6.0
    t0 = time.perf_counter()
    lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
    loss = LR.criterion('ssd512', P, lo, sc, boxes, labels, 'diou', 'focal')
    loss.backward()
    t1 = time.perf_counter()
    probs = torch.softmax(det, 2).numpy()
    bx = M.decode_boxes(locs.numpy(), Pn, 'offset')
    M.detect(probs, bx, 0.01, 0.45, 200)
    t2 = time.perf_counter()
    per_img = (t2 - t0) / B_sample
    return {'value': round(1.0 / per_img, 4), 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': '%d SSD512 images: oracle MultiBoxLoss512 (DIoU+focal) fwd+bwd %.2f s + oracle '
                      'detect (numpy greedy NMS, torchvision semantics) %.2f s, torch/numpy on %d host '
                      'threads' % (B_sample, t1 - t0, t2 - t1, threads)}


def main():
    a = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    L.lib()
    B = a.batch
    Pn = prior_table(ARCH)
    P = Pn.shape[0]
    priors = torch.from_numpy(Pn).to(dev)
    cfg = Cfg(reg_weights=1.0, device=dev, n_classes=N_CLASSES, reg_loss='diou', cls_loss='focal',
              focal_type='softmax', model={'box_type': 'offset'})
    crit = CR.MultiBoxLoss512(priors_cxcy=priors, config=cfg)
    crit.distributed = world > 1
    boxes, labels, locs0, scores0, det_scores = make_batch(B, 1000 * rank, dev)
    locs = locs0.clone().requires_grad_(True)
    scores = scores0.clone().requires_grad_(True)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    loss_ms = []

    def step(record=False):
        # criterion forward; detect's kernels queued (core.detect async: the same work as
        # models.utils.detect, whose lists are collected at the end of the step); backward —
        # its host work overlaps the detect kernels; then the per-image detection lists
        locs.grad = None
        scores.grad = None
        if record:
            ev[0].record()
        loss = crit(locs, scores, boxes, labels)
        if record:
            ev[1].record()
        if a.sync_detect:
            if record:
                ev[2].record()
            loss.backward()
            if record:
                ev[3].record()
            return loss, MU.detect(locs.detach(), det_scores, 0.01, 0.45, 200, priors, cfg)
        h = core.detect(locs.detach(), det_scores, 0.01, 0.45, 200, priors, box_type='offset',
                        act='softmax', async_=True)
        if record:
            ev[2].record()
        loss.backward()
        if record:
            ev[3].record()
        return loss, h.wait()

    # workload constants for the algorithmic byte counts (computed before any timing)
    with torch.no_grad():
        n_cand = int((torch.softmax(det_scores, 2)[:, :, 1:] > 0.01).sum().item())
    wl = {'B': B, 'P': P, 'C': N_CLASSES, 'n_cand': n_cand, 'Gmax': max(int(b.shape[0]) for b in boxes)}

    for _ in range(max(a.warmup - 1, 0)):
        step()
    # one more untimed step with every instrumented kernel bracketed by HIP events: the
    # per-kernel table, and the dominant HBM-bound kernel that is timed live below
    torch.cuda.synchronize()
    L.timing_enable('*')
    step()
    torch.cuda.synchronize()
    kernel_us = {}
    for k in ALL_KERNELS:
        n, ms = L.timing_query(k)
        if n:
            kernel_us[k] = round(ms * 1e3, 1)
    dominant = max(HBM_KERNELS, key=lambda k: kernel_us.get(k, 0.0))
    # live timing of the dominant kernel over the timed region, one launch in TIMING_EVERY: a timed
    # launch carries its events on the dispatch (exact kernel time, agrees with rocprofv3) but
    # costs host time, so only a sample of the steps pays it
    L.call('sbod_timing_every', TIMING_EVERY)
    L.timing_enable(dominant)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dom_n, dom_ms = L.timing_query(dominant)
    L.timing_enable(None)
    L.call('sbod_timing_every', 1)
    # criterion fwd+bwd GPU time, from event-bracketed steps AFTER the timed region (the per-step
    # event records would otherwise add host work to the steps being timed)
    for _ in range(min(a.steps, 20)):
        step(record=True)
        loss_ms.append(tuple(ev))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    torch.cuda.synchronize()
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    crit_ms = sorted(e0.elapsed_time(e1) + e2.elapsed_time(e3) for e0, e1, e2, e3 in loss_ms)
    crit_ms_med = crit_ms[len(crit_ms) // 2]
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    imgs = world * B * a.steps
    value = imgs / elapsed
    ms_step = elapsed / a.steps * 1e3
    nbytes = bytes_per_step(B, P, N_CLASSES)
    line = {
        'metric': 'images/sec train step SSD512 batch=32 @1/2/4/8 GPU; IoU+NMS Manchors/sec',
        'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': a.steps,
        'warmup': a.warmup, 'ms_per_step': round(ms_step, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
        'config': {'workload': 'SSD512 per-GPU batch %d: MultiBoxLoss512(DIoU+focal) fwd+bwd + '
                               'detect(min_score 0.01, iou 0.45, top_k 200)%s'
                               % (B, '' if a.sync_detect else ', detect kernels overlapped with the backward'),
                   'global_batch': world * B, 'n_priors': P, 'n_classes': N_CLASSES,
                   'parallelism': 'dp%d' % world},
        'manchors_per_sec': round(world * B * P * a.steps / elapsed / 1e6, 3),
        'criterion_fwd_bwd_ms_median': round(crit_ms_med, 4),
        'criterion_GBps_algorithmic': round(nbytes / (crit_ms_med * 1e-3) / 1e9, 1),
    }
    avg_s = dom_ms / max(dom_n, 1) * 1e-3
    algo = ALGO_BYTES[dominant](wl)
    achieved = algo / avg_s / 1e9
    traffic = pmc_traffic(dominant)
    line['roofline'] = {
        'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
        'kernel': dominant, 'launches': dom_n, 'timed_every': TIMING_EVERY, 'avg_us': round(avg_s * 1e6, 2),
        'algorithmic_bytes_per_launch': algo,
    }
    line['kernel_us_per_step'] = kernel_us
    if not a.no_cpu_baseline:
        threads = min(os.cpu_count() or 1, 16)
        line['cpu_baseline'] = cpu_baseline(a.cpu_sample_images, threads)
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
