#!/usr/bin/env python3
"""Throughput of the sbod hot path on MI355X (contract: one JSON line on rank 0).

One step = one pass of the hot path over one batch of SSD512 synthetic input resident in HBM
(SURVEY §8(d) recipe; BASELINE.json metric "images/sec train step SSD512 batch=32"):
  1. ground-truth packing of the per-image lists into fixed-capacity device buffers (one
     sbod_gt_pack launch);
  2. MultiBoxLoss512 (DIoU box loss + softmax focal, the configs[1] losses) forward AND
     backward through the drop-in criterion: the HIP matcher, the fused loss+gradient pass and
     the upstream-gradient application;
  3. detect on the same batch (softmax, offset decode + clamp, per-class NMS at IoU 0.45,
     min_score 0.01, top_k 200 — models.utils.detect's work) up to its per-image lists, which
     need one device->host sync.
Every kernel runs every step.  By default (``--submit direct``) the step's entry-point calls are
recorded once per resident batch (its own outputs, the streams' warm workspaces) and issued
again each step from the fast C wrappers; ``--submit graph`` captures them into hipGraphs
(criterion and detect) and replays those instead (a hipGraphLaunch costs ~8 us of host time, two
per step, more than the launches it replaces).  Criterion and detect each alternate over two
streams, and ``--depth`` (default 4) steps are in flight: step k is submitted before step
k-3's per-image lists are collected.  ``--eager`` runs the Python API calls every step; the line
also carries the eager step time.  Data-parallel runs always replay graphs (the RCCL exchange of
the loss normaliser is a torch.distributed call the recorder does not see).

Inputs come from HBM, not from the 256 MiB Infinity Cache (MI355X_MICROARCH.md, "Infinity
Cache": FETCH_SIZE and kernel time both count its hits): the bench holds ``--batches`` (default
6) distinct seeded SSD512 batches — each with its own ground truth, locs/scores and detect
scores, and its own captured graphs and gradient buffers — and step k runs batch k mod 6.  One
step touches ~100 MB, a full rotation ~600 MB, so every replay reads lines last touched 5 steps
(~500 MB) earlier.

Data parallel (``--gpus N``): one process per GPU.  Without WORLD_SIZE in the environment this
script starts the N rank processes itself (subprocesses, before any GPU call); under
torch.distributed.run it is one of them.  Per-GPU batch is fixed (weak scaling).  The hot path's
exchange is the SUM all-reduce of the batch positive count (the loss normaliser), inside the
graph.  Reported beside the hot-path value: the same step with the SSD512-sized gradient
all-reduce of data-parallel training (26,450,959 fp32 values), bucketed on its own
RCCL communicator and overlapped with the step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--eager]
                    [--no-cpu-baseline] [--no-dcn]
"""
import argparse
import collections
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
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
F32_MFMA_PEAK_TFS = 157.3  # dense fp32 MFMA (MI355X_MICROARCH.md)
N_CLASSES = 21
ARCH = 'SSD512'
SSD512_PARAMS = 26450959   # SSD512 parameter count -> fp32 gradient elements
BUCKET_MB = 25             # DDP's default bucket size


class Cfg(dict):
    __getattr__ = dict.__getitem__


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--eager', action='store_true', help='no hipGraph: launch every call each step')
    ap.add_argument('--one-stream', action='store_true',
                    help='graph mode: one graph per step (criterion and detect in stream order)')
    ap.add_argument('--priority', choices=('none', 'detect', 'criterion'), default='detect',
                    help='graph mode: which of the two streams gets the high HIP stream priority')
    ap.add_argument('--order', choices=('criterion_first', 'detect_first', 'detect_early'), default='criterion_first',
                    help='graph mode: which graph of a step is submitted first')
    ap.add_argument('--crit-form', choices=('two', 'one'), default='two',
                    help='focal criterion: matcher + loss launches (two) or the one-launch form (one)')
    ap.add_argument('--finish', choices=('fused', 'separate'), default='separate',
                    help='focal loss finish: in the loss pass\'s last-arriving workgroup (fused) or a separate '
                         'one-block launch after it (same exact sum)')
    ap.add_argument('--det-form', choices=('two', 'one'), default='two',
                    help='detect: per-class NMS and per-image merge as two launches or one (k_det_nms)')
    ap.add_argument('--hw-queues', type=int, default=None,
                    help='HIP hardware queues per process (GPU_MAX_HW_QUEUES, <= 32; the runtime default is 4): '
                         'more streams than queues share a queue and serialise')
    ap.add_argument('--submit', choices=('graph', 'direct', 'fork'), default='direct',
                    help='graph: replay captured hipGraphs (criterion and detect, two launches); fork: one '
                         'graph per step with detect forked onto its stream inside it; direct: issue the '
                         'recorded entry-point calls')
    ap.add_argument('--gt-fold', type=int, choices=(0, 1), default=1,
                    help='direct submit: 1 = the GT packing folded into the matcher\'s first launch '
                         '(sbod_criterion_focal_lists: one launch fewer per step), 0 = a separate sbod_gt_pack '
                         'launch.  Same-box A/B at the driver\'s 20 steps, six rounds: 0.0367-0.0401 vs '
                         '0.0379-0.0426 ms (fold faster in 5 of 6; host submit 25-27 vs 28-31 us); at 300 '
                         'GPU-bound steps 0.0331 vs 0.0325 (profiles/r6_fold20_ab_a.jsonl)')
    ap.add_argument('--depth', type=int, default=4,
                    help='graph mode: steps in flight (submit step k, then collect step k - depth + 1)')
    ap.add_argument('--crit-streams', type=int, default=2,
                    help='graph mode: streams the criterion graphs alternate over (1 = one criterion stream)')
    ap.add_argument('--det-streams', type=int, default=2,
                    help='graph mode: streams the detect graphs alternate over (1 = one detect stream)')
    ap.add_argument('--sync', choices=('auto', 'spin', 'yield'), default='auto',
                    help='how the host waits for the GPU (hipSetDeviceFlags schedule, set before the '
                         'device is initialised): auto = the runtime default (yield with one context)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-dcn', action='store_true')
    ap.add_argument('--batches', type=int, default=6,
                    help='distinct resident batches rotated step by step (HBM, not cache, reads)')
    ap.add_argument('--timing-steps', type=int, default=12,
                    help='eager steps whose every kernel dispatch carries HIP events')
    ap.add_argument('--no-c2', action='store_true', help='skip the config C2 bf16 B=16 figure')
    ap.add_argument('--c2-finish', choices=('fused', 'separate'), default='fused',
                    help='C2 figure\'s loss finish: C2 is host-bound, so the form with one launch fewer per '
                         'step (fused) wins there: 0.0301-0.0311 vs 0.0351-0.0389 ms, three rounds on one box '
                         '(profiles/r5_c2_finish_ab_a1.jsonl)')
    ap.add_argument('--c2-det-form', choices=('two', 'one'), default='one',
                    help='C2 figure: detect as two launches (segment, merge) or one (k_det_nms); the C2 step '
                         'is host-bound, so one launch fewer wins there (same-box A/B 0.0327-0.0363 vs '
                         '0.0346-0.0375 ms) while the GPU-bound headline keeps two')
    return ap.parse_args(argv)


class Batch:
    """One resident synthetic batch (SURVEY §8(d) recipe): per-image GT lists on the device,
    locs/scores leaves (grad-enabled) in ``dtype``, and the detection workload's scores."""

    def __init__(self, B, seed, dev, dtype=torch.float32):
        P = prior_table(ARCH).shape[0]
        boxes, labels = synth.make_gt(B, seed=seed, n_classes=N_CLASSES)
        locs, scores = synth.make_preds(B, P, N_CLASSES, seed=seed)
        det_scores = scores.clone()
        det_scores[:, :, 0] += 6.0            # detection workload: +6 background logit (§8(d))
        self.boxes = [b.to(dev) for b in boxes]
        self.labels = [l.to(dev) for l in labels]
        self.locs = locs.to(dev, dtype).requires_grad_(True)
        self.scores = scores.to(dev, dtype).requires_grad_(True)
        self.det_scores = det_scores.to(dev, dtype)


def criterion_bytes(B, P, C):
    """Algorithmic HBM bytes of the fused loss pass: read locs+scores once,
    write their gradients once, priors once per batch."""
    return B * P * 2 * (4 + C) * 4 + 16 * P


def detect_bytes(w):
    """scores [B,P,C] read; candidate keys (8 B each) and per-(image, class) counts written
    (k_det_prepare; since round 6 the boxes are decoded by the NMS kernels after it, for the
    candidates they read only — those kernels are latency-bound and not counted)."""
    return w['B'] * w['P'] * 4 * w['C'] + 8 * w['n_cand'] + 4 * w['B'] * w['C']


# Algorithmic HBM bytes per launch of the streaming (HBM-bound) kernels of one step (DESIGN.md
# "Kernels"): every input read once, every output written once.  w = workload constants.
ALGO_BYTES = {
    'k_det_prepare': detect_bytes,
    # locs + scores read, their gradients written, matcher obj (i32) + overlap (f32) read,
    # priors read once
    'k_multibox': lambda w: w['B'] * w['P'] * (2 * (16 + 4 * w['C']) + 8) + 16 * w['P'],
    # priors read per image tile, obj + overlap written
    'k_match_tile': lambda w: w['B'] * w['P'] * (16 + 8),
    # the one-launch focal criterion (matcher + loss pass): locs + scores read, their gradients
    # written, obj + overlap written, priors (xyxy and cxcy) read once
    'k_criterion': lambda w: w['B'] * w['P'] * (2 * (16 + 4 * w['C']) + 8) + 32 * w['P'],
}
HBM_KERNELS = tuple(ALGO_BYTES)
ALL_KERNELS = HBM_KERNELS + ('k_det_nms', 'k_det_segment', 'k_det_merge', 'k_match_final', 'k_hnm', 'k_loss_final')
PMC_FILE = os.path.join(HERE, 'profiles', 'pmc_traffic.json')
DIST_BACKEND = os.environ.get('SBOD_BENCH_DIST_BACKEND', 'nccl')   # 'gloo': one-GPU rehearsal only
# The step's captures restrict unsafe HIP calls in the capturing thread only: with ranks, the
# process group's watchdog thread queries events while the main thread captures, which a global
# capture would count against the graph (torch.cuda.graph's capture_error_mode)
CAPTURE_MODE = 'thread_local'


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (FETCH_SIZE and
    WRITE_SIZE collected in separate passes; FETCH doubled on gfx950, KB -> bytes), or None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        return d['kernels'][kernel]['traffic_bytes_per_launch']
    except (OSError, KeyError, ValueError):
        return None


# ----------------------------------------------------------------------------- CPU baseline
def cpu_baseline(B, threads_all, det_images_one=8):
    """The oracle (CPU restatement of the reference, pinned by tests/golden) on host cores, over
    the SAME B-image workload as the GPU step: warm median of MultiBoxLoss512 (DIoU+focal)
    fwd+bwd on the whole batch, plus detect (softmax, offset decode, numpy greedy NMS with
    torchvision semantics, top-k) on every one of the B images, at all host threads (capped at
    16, the box's CPU share).  The 1-thread figure times the criterion the same way and detect on
    ``det_images_one`` images (the NMS is single-threaded numpy either way: images spread over 8
    Python threads took 35.8 s vs 6.3 s in turn for 8 images, the greedy loop holds the GIL).
    kind = 'port'."""
    from oracle import loss_ref as LR
    from oracle import match_ref as M
    Pn = prior_table(ARCH)
    P = torch.from_numpy(Pn)
    boxes, labels = synth.make_gt(B, seed=0, n_classes=N_CLASSES)
    locs, scores = synth.make_preds(B, Pn.shape[0], N_CLASSES, seed=0)
    det = scores.clone()
    det[:, :, 0] += 6.0
    out = {}
    for threads, n_det in ((threads_all, B), (1, min(det_images_one, B))):
        torch.set_num_threads(threads)
        crit = []
        for _ in range(3):      # first run warms the allocator / thread pool; median of the rest
            lo, sc = locs.clone().requires_grad_(True), scores.clone().requires_grad_(True)
            t0 = time.perf_counter()
            LR.criterion('ssd512', P, lo, sc, boxes, labels, 'diou', 'focal').backward()
            crit.append(time.perf_counter() - t0)
        t_crit = sorted(crit[1:])[len(crit[1:]) // 2]
        t0 = time.perf_counter()
        probs = torch.softmax(det[:n_det], 2).numpy()
        bx = M.decode_boxes(locs[:n_det].numpy(), Pn, 'offset')
        M.detect(probs, bx, 0.01, 0.45, 200)
        t_det = time.perf_counter() - t0
        per_img = t_crit / B + t_det / n_det
        out[threads] = (1.0 / per_img, t_crit, t_det, n_det)
    torch.set_num_threads(threads_all)
    v_all, c_all, d_all, n_all = out[threads_all]
    v_one, c_one, d_one, n_one = out[1]
    return {'value': round(v_all, 3), 'unit': 'images/s', 'cores': threads_all, 'kind': 'port',
            'sample': ('oracle MultiBoxLoss512 (DIoU+focal) fwd+bwd on the %d-image batch, warm median '
                       'of 2: %.3f s; oracle detect on all %d images of it: %.2f s (%.3f s/image); '
                       'images/s = 1 / (criterion s/img + detect s/img), %d host threads'
                       % (B, c_all, n_all, d_all, d_all / n_all, threads_all)),
            'one_thread': {'value': round(v_one, 3), 'cores': 1, 'criterion_s': round(c_one, 4),
                           'detect_s': round(d_one, 3), 'detect_images': n_one}}


def dcn_cpu_baseline(threads, H=64, B=4, C=256, O=256):
    """The DCN leg of the CPU baseline (BASELINE.md's timed CPU path includes DeformConv2d): the
    oracle (oracle/dcn_ref.py, the reference's forward restated in torch-CPU, autograd backward)
    forward + the four input gradients on a bounded C4 sample (B images at HxH, 256 -> 256, 3x3,
    modulated) on host cores; TF/s of the same three contractions the GPU figure counts.  Second
    of two runs (the first warms the allocator / thread pool).  kind = 'port'."""
    from oracle import dcn_ref as DR
    g = torch.Generator().manual_seed(H)
    x = torch.randn(B, C, H, H, generator=g).requires_grad_(True)
    off = torch.randn(B, 18, H, H, generator=g).requires_grad_(True)
    ml = torch.randn(B, 9, H, H, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, 3, 3, generator=g) / 48).requires_grad_(True)
    gout = torch.randn(B, O, H, H, generator=g)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    ts = []
    for _ in range(2):
        t0 = time.perf_counter()
        out = DR.deform_conv2d(x, off, torch.sigmoid(ml), w, 3, 1, 1)
        torch.autograd.grad(out, (x, off, ml, w), gout)
        ts.append(time.perf_counter() - t0)
    torch.set_num_threads(prev)
    fl = 3 * 2.0 * B * H * H * O * C * 9
    return {'tflops': round(fl / ts[-1] / 1e12, 4), 'unit': 'TF/s', 'cores': threads, 'kind': 'port',
            'sample': 'oracle DeformConv2d fwd + 4 input gradients, B=%d %dx%d 256->256 3x3 modulated: %.3f s '
                      '(second of two runs)' % (B, H, H, ts[-1])}


# ----------------------------------------------------------------------------- DCN (config C4)
def dcn_figure(dev, H=64, B=16, C=256, O=256, iters=5):
    """DeformConv2d (a14) forward+backward at one of config C4's maps: TF/s of the three
    contractions (fwd, d-cols, d-weight: 3 x 2*M*O*C*9) against the fp32 MFMA peak.  The step is
    out = deform_conv2d(...) and the four input gradients by torch.autograd.grad (as after a
    zero_grad(set_to_none=True): no accumulation kernels); timed replayed from one hipGraph
    (``ms``, the primary figure) and launched eagerly through autograd (``eager_ms``: the
    per-call host cost shows at the small maps)."""
    g = torch.Generator(device=dev).manual_seed(H)
    x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(True)
    off = torch.randn(B, 18, H, H, device=dev, generator=g).requires_grad_(True)
    ml = torch.randn(B, 9, H, H, device=dev, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, 3, 3, device=dev, generator=g) / 48).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=dev, generator=g)
    params = (x, off, ml, w)

    def step():
        return torch.autograd.grad(core.deform_conv2d(x, off, ml, w), params, gout)

    def clock(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    # captured on the warm-up stream: the cached workspaces are per stream
    with torch.cuda.graph(graph, stream=side):
        step()
    graph.replay()
    ms = clock(graph.replay)
    eager = clock(step)
    fl = 3 * 2.0 * B * H * H * O * C * 9
    tf = fl / ms / 1e9
    return {'config': 'C4 DeformConv2d B=%d %d->%d 3x3 %dx%d fwd+bwd fp32' % (B, C, O, H, H),
            'ms': round(ms, 4), 'tflops': round(tf, 2), 'peak_tflops': F32_MFMA_PEAK_TFS,
            'mfma_frac': round(tf / F32_MFMA_PEAK_TFS, 4), 'timing': 'hipGraph replay',
            'eager_ms': round(eager, 4), 'eager_mfma_frac': round(fl / eager / 1e9 / F32_MFMA_PEAK_TFS, 4)}


# ----------------------------------------------------------------------------- the step
class DPGraph:
    """A data-parallel step's criterion as two captured graphs around an EAGER all-reduce of the
    positive count: the matcher (and the count's copy into `tot`) | torch.distributed.all_reduce
    (asynchronous: RCCL runs it on its own stream behind the matcher, no host sync) | the loss
    pass and its backward.  No collective is captured, so the step does not depend on capturing
    RCCL (or on a capture of it surviving the process group's watchdog thread), and a one-GPU gloo
    rehearsal replays the same graphs.

    ``front()`` issues the matcher and the all-reduce, ``back()`` makes the current stream wait for
    the all-reduce and replays the loss pass.  The matcher needs only the ground truth and the
    priors (models/SSD512.py:535-563), so ``Step`` issues step k+1's front before step k's back:
    the loss pass of step k then waits on a collective issued one step earlier (long complete),
    never on one in flight.  Both run on the current stream."""

    def __init__(self, ga1, tot, ga2, group=None):
        self.ga1, self.tot, self.ga2, self.group = ga1, tot, ga2, group
        self.work = None

    def front(self):
        import torch.distributed as dist
        if self.work is not None:
            raise RuntimeError('DPGraph.front: the previous front of this batch was never consumed')
        self.ga1.replay()
        self.work = dist.all_reduce(self.tot, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def back(self):
        if self.work is None:
            self.front()
        w, self.work = self.work, None
        w.wait()          # the current stream waits for the all-reduce (no host sync under RCCL)
        self.ga2.replay()

    def replay(self):
        self.front()
        self.back()


def capture_dp_criterion(crit, locs, scores, gt, one, stream):
    """Capture `crit(locs, scores, gt, None).backward(one)` (a distributed criterion) as a DPGraph:
    core.allreduce_npos is swapped, for the capture only, for a split point that ends the first
    graph after the count's copy and begins the second on the same stream and memory pool."""
    ga1, ga2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    tot = torch.zeros(1, dtype=torch.int32, device=locs.device)
    orig = core.allreduce_npos
    split = {'done': False}

    def split_point(n_pos, group=None, force=False):
        if split['done']:
            raise RuntimeError('capture_dp_criterion: more than one collective in the criterion')
        tot.copy_(n_pos[-1:])
        ga1.capture_end()
        ga2.capture_begin(pool=ga1.pool(), capture_error_mode=CAPTURE_MODE)
        split['done'] = True
        split['group'] = group
        return tot

    core.allreduce_npos = split_point
    try:
        with torch.cuda.stream(stream):
            ga1.capture_begin(capture_error_mode=CAPTURE_MODE)
            loss = crit(locs, scores, gt, None)
            loss.backward(one)
            if not split['done']:
                raise RuntimeError('capture_dp_criterion: the criterion issued no all-reduce')
            ga2.capture_end()
    finally:
        core.allreduce_npos = orig
    return DPGraph(ga1, tot, ga2, split.get('group')), loss


class Step:
    """Criterion forward+backward and detect on one batch; eager or captured in hipGraphs.

    ``n_batches`` resident batches are rotated (step k uses batch k mod n): in graph mode each
    batch has its own pair of graphs (criterion on criterion stream k mod ``crit_streams``, detect
    on detect stream k mod ``det_streams``) and its own GT staging buffers, and the graphs own its
    gradients and detections, so consecutive steps never share an input, output or workspace and
    the two-deep pipeline (submit step k, then collect step k-1) needs no copies."""

    def __init__(self, dev, B, rank, world, graph, two_streams=True, priority='none', n_batches=6,
                 dtype=torch.float32, order='criterion_first', det_streams=2, crit_form='two', det_form='two',
                 crit_streams=2, depth=4, submit='direct', gt_fold=True, finish='separate'):
        self.dev, self.B = dev, B
        self.world = world
        self.gt_fold = bool(gt_fold)
        Pn = prior_table(ARCH)
        self.P = Pn.shape[0]
        self.priors = torch.from_numpy(Pn).to(dev)
        self.cfg = Cfg(reg_weights=1.0, device=dev, n_classes=N_CLASSES, reg_loss='diou',
                       cls_loss='focal', focal_type='softmax', model={'box_type': 'offset'})
        self.crit = CR.MultiBoxLoss512(priors_cxcy=self.priors, config=self.cfg)
        self.crit.distributed = world > 1
        self.crit.one_launch = crit_form == 'one'
        self.crit.separate_finish = finish == 'separate'
        self.det_two_pass = det_form == 'two'
        self.batches = [Batch(B, 1000 * rank + 100 * i, dev, dtype) for i in range(max(1, n_batches))]
        cap = max(int(b.shape[0]) for bt in self.batches for b in bt.boxes)
        self.capacity = max(16, (cap + 15) // 16 * 16)
        # GT staging per resident batch: step k's packing never overwrites buffers that step k-1's
        # criterion (possibly on the other criterion stream) is still reading
        for bt in self.batches:
            bt.stage = core.GtStaging(B, self.capacity, dev)
        # the warm-up runs on the capture streams, so every workspace the captured calls use
        # (cached per stream in core.workspace) already exists: nothing large is allocated
        # under capture.  Graph mode: the criterion and detect are two graphs replayed on two
        # streams, so their kernels (several latency-bound, few workgroups) run concurrently;
        # a fork/join INSIDE one graph costs ~30 us per edge on this runtime
        # (scripts/probe_graph_launch.py), two graphs on two streams need no edge at all.
        # criterion graphs alternate over `crit_streams` streams the same way (each stream has its
        # own cached workspaces): step k's matcher need not wait for step k-1's loss pass
        # with ranks every criterion graph holds the normaliser's RCCL all-reduce: collectives on
        # one communicator must run in the order they were issued on every rank, which two
        # criterion streams replaying concurrently would not guarantee (step k+1's all-reduce
        # could start before step k's on one rank and after it on another: a cross-rank deadlock).
        # Data-parallel steps therefore keep ONE criterion stream; detect has no collective.
        if world > 1:
            crit_streams = 1
        self.cap_streams = [torch.cuda.Stream(dev, priority=-1 if priority == 'criterion' else 0)
                            for _ in range(max(1, crit_streams))]
        self.cap_stream = self.cap_streams[0]
        self._cap_warm = set()
        # detect graphs alternate over `det_streams` streams (batch i on stream i mod n): step k's
        # prepare need not wait for step k-1's segment / merge (latency-bound, few workgroups),
        # so the two overlap instead of the detect chain setting the step period
        self.det_streams = [torch.cuda.Stream(dev, priority=-1 if priority == 'detect' else 0)
                            for _ in range(max(1, det_streams))]
        self.det_stream = self.det_streams[0]
        self._det_warm = set()
        self.two = two_streams
        self.detect_first = order == 'detect_first'
        self.detect_early = order == 'detect_early'   # detect graph launched before the GT packing
        self.graph = None
        self.use_graph = graph
        self.capture_error = None
        self.fast = None
        self.k = 0
        self.pending = collections.deque()
        self.trace = None   # per-step host stamps of the timed run: (submit start, submit end, collect end)
        self.depth = max(2, int(depth))
        # the recorder sees sbod entry points only: with ranks, the normaliser's RCCL all-reduce
        # (torch.distributed) must be in the replayed work, so data-parallel steps replay graphs
        self.submit = submit if world == 1 or submit == 'fork' else 'graph'
        self.host_submit = self.host_collect = 0.0
        # the read-only unit upstream gradient: no ones-fill and no scale launch in the step
        self.one = core.unit_grad(dev)

    def fresh_streams(self):
        """New criterion / detect streams (same count and priorities) with their warm-up state
        reset: the eager fallback after a failed capture, whose streams may stay capturing."""
        self.cap_streams = [torch.cuda.Stream(self.dev, priority=s.priority) for s in self.cap_streams]
        self.cap_stream = self.cap_streams[0]
        self.det_streams = [torch.cuda.Stream(self.dev, priority=s.priority) for s in self.det_streams]
        self.det_stream = self.det_streams[0]
        self._cap_warm.clear()
        self._det_warm.clear()

    def _next_batch(self):
        bt = self.batches[self.k % len(self.batches)]
        self.k += 1
        return bt

    def cs_of(self, i):
        return self.cap_streams[i % len(self.batches) % len(self.cap_streams)]

    def ds_of(self, i):
        return self.det_streams[i % len(self.batches) % len(self.det_streams)]

    def detect(self, bt, capture):
        return core.detect(bt.locs.detach(), bt.det_scores, 0.01, 0.45, 200, self.priors,
                           box_type='offset', act='softmax', async_=True, capture=capture,
                           two_pass=self.det_two_pass)

    def body(self, bt, gt):
        """One stream, in stream order: criterion forward, detect (lists collected later),
        backward."""
        loss = self.crit(bt.locs, bt.scores, gt, None)
        h = self.detect(bt, False)
        loss.backward(self.one)
        return loss, h

    def launch_eager(self):
        bt = self._next_batch()
        bt.locs.grad = None
        bt.scores.grad = None
        gt = bt.stage.stage(bt.boxes, bt.labels)
        return self.body(bt, gt)

    def eager(self):
        loss, h = self.launch_eager()
        return loss, h.wait()

    def eager_split(self):
        """The two-stream form eagerly (also warms both capture streams' workspaces): GT
        packing, criterion forward and backward on the batch's criterion stream, detect on its
        detect stream."""
        bt = self._next_batch()
        bt.locs.grad = None
        bt.scores.grad = None
        cs, ds = self.cs_of(self.k - 1), self.ds_of(self.k - 1)
        cs.wait_stream(torch.cuda.current_stream(self.dev))
        ds.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(cs):
            gt = bt.stage.stage(bt.boxes, bt.labels)
            loss = self.crit(bt.locs, bt.scores, gt, None)
        with torch.cuda.stream(ds):
            h = self.detect(bt, False)
        self._det_warm.add(ds.cuda_stream)
        with torch.cuda.stream(cs):
            loss.backward(self.one)
        self._cap_warm.add(cs.cuda_stream)
        out = loss, h.wait()
        torch.cuda.current_stream(self.dev).wait_stream(cs)
        return out

    def eager_half(self, part):
        """One half of the two-stream step alone, eagerly, on its own stream: 'criterion' (GT
        packing, forward, backward) or 'detect' — the roofline's kernel timed without the other
        half's kernels running beside it."""
        bt = self._next_batch()
        bt.locs.grad = None
        bt.scores.grad = None
        if part == 'detect':
            ds = self.det_streams[0]
            ds.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(ds):
                self.detect(bt, False).wait()
            torch.cuda.current_stream(self.dev).wait_stream(ds)
            return
        cs = self.cs_of(self.k - 1)
        cs.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(cs):
            gt = bt.stage.stage(bt.boxes, bt.labels)
            loss = self.crit(bt.locs, bt.scores, gt, None)
            loss.backward(self.one)
        torch.cuda.current_stream(self.dev).wait_stream(cs)

    def capture(self, after_first=None):
        """Capture one graph pair per resident batch (the usual torch pattern: warm-up already
        done on the capture streams; gradients set to None so the captured backward owns
        them).  ``after_first`` runs after the first batch's capture."""
        n = len(self.batches)
        for cs in self.cap_streams:   # every criterion stream's workspaces exist before capture
            if cs.cuda_stream not in self._cap_warm:
                bt = self.batches[0]
                cs.wait_stream(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(cs):
                    self.crit(bt.locs, bt.scores, bt.stage.stage(bt.boxes, bt.labels), None).backward(self.one)
                torch.cuda.current_stream(self.dev).wait_stream(cs)
                self._cap_warm.add(cs.cuda_stream)
        # every detect stream's workspace exists before capture (one graph per step: detect runs
        # on the criterion streams)
        for ds in (self.det_streams if self.two else self.cap_streams):
            if ds.cuda_stream not in self._det_warm:
                ds.wait_stream(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(ds):
                    self.detect(self.batches[0], False).wait()
                self._det_warm.add(ds.cuda_stream)
        core.reserve_count_slots(self.dev, self.B, n)
        torch.cuda.synchronize()
        self.slots = []
        for bi, bt in enumerate(self.batches):
            bt.locs.grad = None
            bt.scores.grad = None
            gt = bt.stage.stage(bt.boxes, bt.labels)   # the batch's own staging buffers
            torch.cuda.synchronize()
            if self.submit == 'direct':
                # native submit: the step's entry-point calls recorded once (each with its own
                # outputs, the streams' warm workspaces and zero-on-entry flags set), then issued
                # again every step from the fast wrappers — the same launches a graph would replay,
                # without the graph launch (scripts/submit_probe.py: hipGraphLaunch ~8 us each)
                cs, ds = self.cs_of(bi), self.ds_of(bi)
                crit_calls, det_calls = [], []
                cs.wait_stream(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(cs), L.record_calls(crit_calls):
                    loss = self.crit(bt.locs, bt.scores, gt, None)
                    loss.backward(self.one)
                ds.wait_stream(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(ds), L.record_calls(det_calls):
                    h = self.detect(bt, True)     # persistent handle: its outputs are the slot's
                torch.cuda.synchronize()
                if any(n == 'sbod_gt_pack' for n, _ in crit_calls + det_calls) or not crit_calls or not det_calls:
                    raise RuntimeError('direct submit: unexpected recorded calls %s'
                                       % [n for n, _ in crit_calls + det_calls])
                self.slots.append((crit_calls, det_calls, loss, h))
                continue
            if self.submit == 'fork':
                # ONE graph per step: detect forked onto the detect stream inside the capture and
                # joined back, so one hipGraphLaunch submits both chains (which stay concurrent)
                g = torch.cuda.CUDAGraph()
                cs, ds = self.cs_of(bi), self.ds_of(bi)
                with torch.cuda.graph(g, stream=cs, capture_error_mode=CAPTURE_MODE):
                    ds.wait_stream(cs)
                    with torch.cuda.stream(ds):
                        h = self.detect(bt, True)
                    loss = self.crit(bt.locs, bt.scores, gt, None)
                    loss.backward(self.one)
                    cs.wait_stream(ds)
                self.slots.append((g, None, loss, h))
                if after_first is not None and len(self.slots) == 1:
                    after_first()
                continue
            if self.two:
                gb = torch.cuda.CUDAGraph()
                if self.world > 1:   # two graphs around the eager all-reduce (DPGraph)
                    ga, loss = capture_dp_criterion(self.crit, bt.locs, bt.scores, gt, self.one, self.cs_of(bi))
                else:
                    ga = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(ga, stream=self.cs_of(bi), capture_error_mode=CAPTURE_MODE):
                        loss = self.crit(bt.locs, bt.scores, gt, None)
                        loss.backward(self.one)
                with torch.cuda.graph(gb, stream=self.ds_of(bi), capture_error_mode=CAPTURE_MODE):
                    h = self.detect(bt, True)
                self.slots.append((ga, gb, loss, h))
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.cs_of(bi), capture_error_mode=CAPTURE_MODE):
                    loss = self.crit(bt.locs, bt.scores, gt, None)
                    h = self.detect(bt, True)
                    loss.backward(self.one)
                self.slots.append((g, None, loss, h))
            if after_first is not None and len(self.slots) == 1:
                after_first()
        torch.cuda.synchronize()
        self.graph = self.slots[0][0]
        # raw handles for the one-call submit (C++: GT packing + both replays + detect event)
        self.fast = None
        if self.submit == 'direct':
            if L.host_ext is None:
                raise RuntimeError('direct submit needs the _sbodhost extension')
            self.programs = []
            for bi, (crit_calls, det_calls, _, h) in enumerate(self.slots):
                ds, cs = self.ds_of(bi), self.cs_of(bi)
                h.replayed(ds)   # creates the event (recorded once here)
                prog = None
                if (hasattr(L.host_ext, 'make_step_program') and len(crit_calls) == 1 and len(det_calls) == 1
                        and crit_calls[0][0] == 'sbod_criterion_focal' and det_calls[0][0] == 'sbod_detect_f32'):
                    # the whole submit in one native call (list checks + packing, the two recorded
                    # entry points, the event)
                    stg = self.batches[bi].stage
                    prog = L.host_ext.make_step_program(
                        (stg.boxes.shape[0], stg.capacity, self.dev.index or 0, stg.boxes.data_ptr(),
                         stg.labels.data_ptr(), stg.offsets.data_ptr(), cs.cuda_stream),
                        tuple(crit_calls[0][1]), tuple(det_calls[0][1]), h._event.cuda_event, ds.cuda_stream,
                        self.gt_fold)
                self.programs.append(prog)
            torch.cuda.synchronize()
        elif L.host_ext is not None and self.world == 1:   # (DP: DPGraph replays from Python)
            self.fast = []
            for bi, (ga, gb, _, h) in enumerate(self.slots):
                ds, cs = self.ds_of(bi), self.cs_of(bi)
                if gb is None:          # one graph per step: criterion then detect on one stream
                    h.replayed(cs)
                    self.fast.append((core.graph_launches([(ga, cs)]), h._event.cuda_event, cs.cuda_stream, None))
                    continue
                h.replayed(ds)          # creates the event (recorded once here)
                pairs = [(ga, cs), (gb, ds)]
                if self.detect_first:
                    pairs.reverse()
                early = None
                if self.detect_early:   # the detect graph alone first, then packing + criterion
                    early = core.graph_launches([(gb, ds)])[0]
                    pairs = [(ga, cs)]
                self.fast.append((core.graph_launches(pairs), h._event.cuda_event, ds.cuda_stream, early))
            torch.cuda.synchronize()
        self.k = 0
        self.pending.clear()
        self.host_submit = self.host_collect = 0.0

    def launch_replay(self):
        i = self.k % len(self.slots)
        bt = self._next_batch()
        ga, gb, loss, h = self.slots[i]
        if self.submit == 'direct':
            prog = self.programs[i]
            if prog is not None:
                r = L.host_ext.submit_step_program(prog, bt.boxes, bt.labels)
                if r is not True:
                    raise RuntimeError('direct submit failed (%r): %s' % (
                        r, L.lib().sbod_last_error().decode(errors='replace') if type(r) is int else 'lists'))
                return loss, h.rearmed()
            # GT packing (C++ list checks + one launch) on the criterion stream, the recorded
            # criterion and detect calls on their streams, the detect event
            cs, ds = self.cs_of(i).cuda_stream, self.ds_of(i).cuda_stream
            stg = bt.stage
            r = L.host_ext.pack_device_lists(bt.boxes, bt.labels, stg.boxes.shape[0], stg.capacity,
                                             self.dev.index or 0, stg.boxes.data_ptr(), stg.labels.data_ptr(),
                                             stg.offsets.data_ptr(), cs, False)
            if type(r) is not list:
                raise RuntimeError('direct submit: GT packing failed (%r)' % (r,))
            L.replay_calls(ga)
            L.replay_calls(gb)
            L.call('sbod_event_record', h._event.cuda_event, ds)
            return loss, h.rearmed()
        if self.fast is not None:
            launches, ev, ev_stream, early = self.fast[i]
            if early is not None:
                L.call('sbod_graph_launch', early[0], early[1])
            # GT packing on the criterion's stream, whichever graph is submitted first.  The
            # lists are resident device tensors written (and synchronised) before any step, so
            # the packing needs no wait on the stream that made them (src_stream = its own)
            cs = self.cs_of(i).cuda_stream
            if bt.stage.stage_and_replay(bt.boxes, bt.labels, launches, ev, ev_stream, pack_stream=cs,
                                         src_stream=cs) is not None:
                return loss, h.rearmed()
        cs = self.cs_of(i)
        if isinstance(ga, DPGraph):
            with torch.cuda.stream(cs):
                if ga.work is None:       # not issued by the previous step (the first one)
                    bt.stage.stage(bt.boxes, bt.labels)
                    ga.front()
                if len(self.slots) > 1:
                    # step k+1's GT packing, matcher and count all-reduce go out BEFORE this step's
                    # loss pass (its own staging buffers and graphs: nothing of step k is touched)
                    j = self.k % len(self.slots)
                    nbt, nga = self.batches[self.k % len(self.batches)], self.slots[j][0]
                    if nga.work is None:
                        nbt.stage.stage(nbt.boxes, nbt.labels)
                        nga.front()
                ga.back()
            ds = self.ds_of(i)
            with torch.cuda.stream(ds):
                gb.replay()
                return loss, h.replayed(ds)
        if gb is None:
            with torch.cuda.stream(cs):
                bt.stage.stage(bt.boxes, bt.labels)
                ga.replay()
                return loss, h.replayed(cs)
        with torch.cuda.stream(cs):
            bt.stage.stage(bt.boxes, bt.labels)
            ga.replay()
        ds = self.ds_of(i)
        with torch.cuda.stream(ds):
            gb.replay()
            return loss, h.replayed(ds)

    def replay(self):
        loss, h = self.launch_replay()
        return loss, h.wait()

    def pipelined(self):
        """One step, pipelined ``depth`` deep: launch step k (GT packing + graph replays), then
        collect step k-depth+1's per-image detection lists (its host sync overlaps the steps
        still on the GPU).  Returns that step's (loss, lists), or None while the pipe fills."""
        t0 = time.perf_counter()
        nxt = self.launch_replay()
        t1 = time.perf_counter()
        self.host_submit += t1 - t0
        self.pending.append(nxt)
        out = None
        if len(self.pending) >= self.depth:
            prev = self.pending.popleft()
            out = prev[0], prev[1].wait()
            self.host_collect += time.perf_counter() - t1
        if self.trace is not None:
            self.trace.append((t0, t1, time.perf_counter()))
        return out

    def drain(self):
        """Collect every launched step not collected yet (oldest first)."""
        out = []
        while self.pending:
            prev = self.pending.popleft()
            out.append((prev[0], prev[1].wait()))
        return out

    def __call__(self):
        return self.replay() if self.graph is not None else self.eager()


def c2_figure(dev, steps, warmup, B=16, n_batches=12, det_form='two', finish='separate'):
    """Config C2 (SSD512 batch=16 bf16 on 1 GPU): the same captured step with bf16 locs / scores
    (and bf16 gradients) for the criterion, and the detect reading the bf16 activations directly
    (SBOD_DETECT_INPUT_BF16: widened exactly on load, no fp32 copies).  ``n_batches`` resident batches
    (~23 MB touched per step) keep the rotation above the Infinity Cache.  Algorithmic bytes of
    the criterion at 2 B/element: SURVEY §8(d) (16.56 MB at B=16)."""
    st = Step(dev, B, 0, 1, graph=True, n_batches=n_batches, dtype=torch.bfloat16, priority='detect',
              det_form=det_form, finish=finish)
    for _ in range(max(warmup - 1, 1)):
        st.eager_split()
    torch.cuda.synchronize()
    # the bf16 criterion's loss-pass kernel, event-timed over eager criterion halves alone (as the
    # headline roofline): locs + scores read and their gradients written at 2 B/element, the
    # matcher's obj + overlap (8 B) read per anchor-image, the priors (16 B) once
    st.eager_half('criterion')
    torch.cuda.synchronize()
    L.timing_enable('k_multibox')
    for _ in range(12):
        st.eager_half('criterion')
    torch.cuda.synchronize()
    n_mb, ms_mb = L.timing_query('k_multibox')
    L.timing_enable(None)
    mb_bytes = B * st.P * (2 * 2 * (4 + N_CLASSES) + 8) + 16 * st.P
    mb_us = ms_mb * 1e3 / n_mb if n_mb else float('nan')
    st.capture()
    for _ in range(len(st.slots) + 1):
        st.replay()
    # three timed runs, the median reported: at B=16 the step is short enough (~40 us) that one
    # host stall inside a 50-step run moved a single figure 0.04 -> 0.12 ms between boxes
    runs = []
    for _ in range(3):
        with torch.cuda.stream(st.cap_stream):
            runs.append(timed(st.pipelined, steps, None, dev, finish=st.drain) / steps * 1e3)
    ms = sorted(runs)[1]
    crit_b = B * st.P * 2 * (4 + N_CLASSES) * 2 + 16 * st.P
    del st
    torch.cuda.synchronize()
    return {'config': 'C2 SSD512 batch=%d bf16: MultiBoxLoss512(DIoU+focal) fwd+bwd in bf16 + detect '
                      '(bf16 activations read in place), captured, %d resident batches' % (B, n_batches),
            'detect_form': det_form, 'loss_finish': finish,
            'ms_per_step': round(ms, 4), 'images_per_s': round(B / (ms * 1e-3), 1),
            'criterion_algorithmic_bytes': crit_b, 'steps': steps,
            'runs_ms_per_step': [round(r, 4) for r in runs],
            'roofline': {'bound': 'hbm', 'kernel': 'k_multibox<bf16>', 'avg_us': round(mb_us, 2),
                         'launches_timed': n_mb, 'algorithmic_bytes_per_launch': mb_bytes,
                         'achieved': round(mb_bytes / (mb_us * 1e-6) / 1e9, 1), 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': round(mb_bytes / (mb_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                         'timing': 'HIP events attached to each dispatch, 12 eager criterion halves alone'}}


def api_figure(st, steps, dist, dev, depth=4):
    """The drop-in API path as a caller issues it (train_anchor.py:271-284 and :342-363): the
    reference-named criterion class on the per-image GT lists, ``loss.backward()`` (autograd's own
    upstream gradient), and ``models.utils.detect(...)`` — with ``async_=True`` so the step is
    pipelined ``depth`` deep like the headline (step k issued before step k-depth+1's lists are
    collected; no other host sync).  Every call does its full per-call host work (argument checks,
    GT packing, allocations, autograd).  Returns ms per step and the host time per call."""
    from shape_based_object_detection_amd.models import utils as MU
    crit = CR.MultiBoxLoss512(priors_cxcy=st.priors, config=st.cfg)
    host = [0.0, 0.0, 0.0, 0.0]

    def one(k):
        bt = st.batches[k % len(st.batches)]
        bt.locs.grad = None
        bt.scores.grad = None
        t0 = time.perf_counter()
        loss = crit(bt.locs, bt.scores, bt.boxes, bt.labels)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        h = MU.detect(bt.locs.detach(), bt.det_scores, 0.01, 0.45, 200, st.priors, st.cfg, async_=True)
        t3 = time.perf_counter()
        host[0] += t1 - t0
        host[1] += t2 - t1
        host[2] += t3 - t2
        return h

    def loop(n):
        pend = collections.deque()
        for k in range(n):
            pend.append(one(k))
            if len(pend) >= depth:
                t = time.perf_counter()
                pend.popleft().wait()
                host[3] += time.perf_counter() - t
        while pend:
            pend.popleft().wait()

    loop(2 * depth)
    torch.cuda.synchronize()
    host[:] = [0.0, 0.0, 0.0, 0.0]
    n = max(steps, 50)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop(n)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {'ms_per_step': round(el / n * 1e3, 4), 'steps': n, 'pipeline_depth': depth,
            'host_us_per_call': {'criterion': round(host[0] / n * 1e6, 1), 'backward': round(host[1] / n * 1e6, 1),
                                 'detect': round(host[2] / n * 1e6, 1),
                                 'collect_incl_wait': round(host[3] / n * 1e6, 1)},
            'calls': 'MultiBoxLoss512(...)(locs, scores, boxes, labels); loss.backward(); '
                     'models.utils.detect(..., async_=True) collected %d steps later' % (depth - 1)}


def timed(fn, steps, dist, dev, per_step=None, finish=None):
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        fn()
        if per_step is not None:
            per_step(i)
    if finish is not None:
        finish()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def grad_allreduce_figure(step, a, dist, dev, world):
    """The data-parallel train step's gradient exchange: an SSD512-sized fp32
    gradient buffer SUM-all-reduced in DDP-sized buckets on its own RCCL communicator and stream,
    overlapped with the hot-path step (as DDP overlaps it with the backward).  Returns the
    all-reduce alone and the overlapped step."""
    grad = torch.ones(SSD512_PARAMS, dtype=torch.float32, device=dev)
    per = BUCKET_MB * (1 << 20) // 4
    buckets = list(grad.split(per))
    group = dist.new_group(backend=DIST_BACKEND)
    comm = torch.cuda.Stream(dev)

    def allreduce():
        for b in buckets:
            dist.all_reduce(b, group=group)

    for _ in range(3):
        allreduce()
    torch.cuda.synchronize()
    n_ar = max(5, a.steps // 5)
    t_ar = timed(allreduce, n_ar, dist, dev) / n_ar
    cur = torch.cuda.current_stream(dev)

    def overlapped():
        comm.wait_stream(cur)
        with torch.cuda.stream(comm):
            allreduce()
        step()
        cur.wait_stream(comm)

    for _ in range(3):
        overlapped()
    t_step = timed(overlapped, a.steps, dist, dev) / a.steps
    nbytes = SSD512_PARAMS * 4
    return {'grad_elems': SSD512_PARAMS, 'grad_bytes': nbytes, 'bucket_mb': BUCKET_MB,
            'n_buckets': len(buckets), 'allreduce_ms': round(t_ar * 1e3, 4),
            'allreduce_busbw_GBps': round(2 * (world - 1) / world * nbytes / t_ar / 1e9, 1),
            'step_ms': round(t_step * 1e3, 4),
            'images_per_s': round(world * a.batch / t_step, 1)}


def main():
    a = parse()
    if a.hw_queues is not None:   # before the first HIP call (torch initialises HIP lazily)
        os.environ['GPU_MAX_HW_QUEUES'] = str(max(1, min(32, a.hw_queues)))
    if 'WORLD_SIZE' not in os.environ and a.gpus > 1:
        # one process per GPU: start the ranks now, before anything touches the GPU
        from shape_based_object_detection_amd.launch import spawn_ranks
        sys.exit(spawn_ranks(a.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    if a.sync != 'auto':   # before torch creates the device's context
        import ctypes
        hip = ctypes.CDLL('libamdhip64.so')
        hip.hipSetDeviceFlags(ctypes.c_uint(1 if a.sync == 'spin' else 2))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != a.gpus:
        raise SystemExit('bench.py: --gpus %d but WORLD_SIZE=%d' % (a.gpus, world))
    dist = None
    # rehearsal of the data-parallel path on a one-GPU box (diagnostic only): every rank on cuda:0
    # and the gloo backend (RCCL refuses two ranks on one device); the driver's runs set neither
    if os.environ.get('SBOD_BENCH_SAME_DEVICE') == '1':
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if DIST_BACKEND == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(DIST_BACKEND)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    L.lib()
    B = a.batch
    st = Step(dev, B, rank, world, graph=not a.eager, two_streams=not a.one_stream, priority=a.priority,
              n_batches=a.batches, order=a.order, det_streams=a.det_streams, crit_form=a.crit_form,
              det_form=a.det_form, crit_streams=a.crit_streams, depth=a.depth, submit=a.submit,
              gt_fold=a.gt_fold, finish=a.finish)
    P = st.P
    # workload constants for the algorithmic byte counts (computed before any timing; the
    # candidate count is averaged over the resident batches)
    with torch.no_grad():
        n_cand = sum(int((torch.softmax(bt.det_scores, 2)[:, :, 1:] > 0.01).sum().item())
                     for bt in st.batches) // len(st.batches)
    wl = {'B': B, 'P': P, 'C': N_CLASSES, 'n_cand': n_cand}

    # warm-up on the capture streams (lazy init of autograd / allocator state, and the
    # per-stream workspaces the captured calls will use)
    for _ in range(max(a.warmup - 1, 1)):
        st.eager_split()
    torch.cuda.synchronize()

    # Kernel durations: eager two-stream steps over the rotating batches with HIP events attached
    # to EVERY instrumented dispatch on its own launch stream (hipExtLaunchKernel start/stop
    # events: the runtime stamps the dispatch's begin and end, as rocprofv3's kernel trace does).
    # The longest HBM-bound kernel here is the roofline's kernel (timed alone below).
    L.timing_enable('*')
    for _ in range(max(a.timing_steps, 10)):
        st.eager_split()
    torch.cuda.synchronize()
    kernel_us, kernel_n = {}, {}
    for k in ALL_KERNELS:
        n, ms = L.timing_query(k)
        if n:
            kernel_us[k] = round(ms * 1e3 / n * (n / max(a.timing_steps, 10)), 2)   # per step
            kernel_n[k] = n
    L.timing_enable(None)
    dominant = max(HBM_KERNELS, key=lambda k: kernel_us.get(k, 0.0))
    # the roofline's duration: the dominant kernel's half of the step (criterion or detect)
    # alone, so no kernel of the other half shares the CUs and HBM with it (the in-step figure
    # is kernel_us_per_step above; the concurrent step is step_hbm_frac)
    def alone(kern):
        """``kern`` timed in its half of the step (criterion or detect) alone: (launches, mean s,
        host window)"""
        hf = 'detect' if kern.startswith('k_det') else 'criterion'
        st.eager_half(hf)
        torch.cuda.synchronize()
        L.timing_enable(kern)
        w0 = time.monotonic_ns()    # the pass's host window: a kernel trace of this run selects
        for _ in range(max(a.timing_steps, 10)):   # the same dispatches (scripts/roofline_check.py)
            st.eager_half(hf)
        torch.cuda.synchronize()
        w1 = time.monotonic_ns()
        nk, msk = L.timing_query(kern)
        L.timing_enable(None)
        return hf, nk, (msk / nk * 1e-3 if nk else float('nan')), w0, w1

    half, n_dom, dom_avg_s, t_win0, t_win1 = alone(dominant)
    # the other half's main HBM kernel, timed the same way (both halves' rooflines in the line)
    others = {}
    for k in ('k_multibox', 'k_det_prepare'):
        if k != dominant and k in kernel_us:
            _, nk, sk, w0, w1 = alone(k)
            others[k] = (nk, sk, w0, w1)

    eager_ms = None
    api = None
    if st.use_graph:        # the same step without the graph, for the host-overhead comparison
        n_e = min(a.steps, 20)
        eager_ms = timed(st.eager, n_e, dist, dev) / n_e * 1e3
        if world == 1:      # the drop-in API path a caller drives
            api = api_figure(st, min(a.steps, 200), dist, dev)

    spans = []
    if st.use_graph:
        # every batch's graph carries a device span record for the dominant kernel (first
        # workgroup start -> last workgroup end, s_memrealtime), read after the timed region
        L.timing_enable(dominant)
        try:
            st.capture()
        except Exception as ex:   # noqa: BLE001 — fall back to eager launches, say so in the line
            st.graph = None
            st.use_graph = False
            st.capture_error = repr(ex)[:300]
            # a capture that failed part-way leaves its stream capturing and torch's current stream
            # set to it; on this runtime an invalidated capture cannot be ended, so the eager
            # fallback leaves those streams for fresh ones (scripts/probe_capture_abort.py)
            torch.cuda.set_stream(torch.cuda.default_stream(dev))
            for s in st.cap_streams + st.det_streams:
                try:
                    L.call('sbod_stream_abort_capture', s.cuda_stream)
                except L.SbodError:
                    pass
            st.fresh_streams()
            torch.cuda.synchronize()
        L.timing_enable(None)
    if st.use_graph:
        for _ in range(len(st.slots) + 1):
            st.replay()
        # the W warm-up steps of the timed kind: pipelined submits and collects, drained before the
        # timed region (which starts from an empty pipeline, after its barrier + synchronize)
        with torch.cuda.stream(st.cap_stream):
            for _ in range(max(a.warmup, 1)):
                st.pipelined()
            st.drain()
        torch.cuda.synchronize()
        st.host_submit = st.host_collect = 0.0
        # the training loop's current stream is the criterion's: the GT lists it hands over
        # are ordered on the stream that packs them (no cross-stream event pair per step)
        st.trace = []
        prof = getattr(L.host_ext, 'submit_profile', None) if L.host_ext is not None else None
        if prof is not None:
            prof(True)
        with torch.cuda.stream(st.cap_stream):
            m_before = time.monotonic_ns()   # host CLOCK_MONOTONIC (rocprofv3's clock): the timed
            t_before = time.perf_counter()   # region in a kernel trace (scripts/timed_trace.py)
            elapsed = timed(st.pipelined, a.steps, dist, dev, finish=st.drain)
            t_after = time.perf_counter()
            m_after = time.monotonic_ns()
        host_submit, host_collect = st.host_submit, st.host_collect
        tr, st.trace = st.trace, None
        sub_phases = prof(True) if prof is not None else None
        # where a short run's time goes: until the first submit starts (barrier + synchronize),
        # the submits and collects of the K steps, and the drain after the last submit
        if tr:
            sub = [(b - a_) * 1e6 for a_, b, _ in tr]
            run_detail = {'before_first_submit_us': round((tr[0][0] - t_before) * 1e6, 1),
                          'submit_us_first4': [round(x, 1) for x in sub[:4]],
                          'submit_us_median': round(sorted(sub)[len(sub) // 2], 1),
                          'last_submit_to_end_us': round((t_after - tr[-1][1]) * 1e6, 1),
                          'steps_span_us': round((tr[-1][2] - tr[0][0]) * 1e6, 1),
                          'timed_window_ns': [m_before, m_after],
                          # per step (first 40): submit start (us from the first), submit and collect us
                          'steps_us': [[round((x0 - tr[0][0]) * 1e6, 1), round((x1 - x0) * 1e6, 1),
                                        round((x2 - x1) * 1e6, 1)] for x0, x1, x2 in tr[:40]]}
            if sub_phases and sub_phases.get('calls'):
                nc = sub_phases.pop('calls')
                first = sub_phases.pop('first_calls_us', None)
                run_detail['native_submit_us_per_step'] = {k: round(v / nc, 2) for k, v in sub_phases.items()}
                if first:   # the fill: [pack, criterion, detect, event] us of the first submits
                    run_detail['native_submit_first_us'] = [[round(x, 1) for x in c] for c in first]
        else:
            run_detail = None
        # the in-graph span of the dominant kernel (a host-synchronous read, so outside the
        # timed region): each batch's graph keeps the record of its latest replay, so after
        # every full rotation the query returns len(slots) distinct launches
        for _ in range(max(2, -(-12 // len(st.slots)))):
            for _ in range(len(st.slots)):
                st.replay()
            torch.cuda.synchronize()
            n, ms = L.timing_query(dominant)
            spans += [ms / n] * n if n else []
    else:
        elapsed = timed(st, a.steps, dist, dev)
    ms_step = elapsed / a.steps * 1e3

    dp = grad_allreduce_figure(st.replay if st.use_graph else st.eager, a, dist, dev, world) if dist else None

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    value = world * B * a.steps / elapsed
    step_bytes = criterion_bytes(B, P, N_CLASSES) + detect_bytes(wl)
    line = {
        'metric': 'images/sec train step SSD512 batch=32 @1/2/4/8 GPU; IoU+NMS Manchors/sec',
        'value': round(value, 2), 'unit': 'images/s', 'n_gpus': world, 'steps': a.steps,
        'warmup': a.warmup, 'ms_per_step': round(ms_step, 4), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32', 'data': 'synthetic',
        'config': {'workload': 'SSD512 per-GPU batch %d: GT packing + MultiBoxLoss512(DIoU+focal) '
                               'fwd+bwd + detect(min_score 0.01, iou 0.45, top_k 200)%s'
                               % (B, ((', the recorded criterion and detect entry-point calls issued natively '
                                       'per step (criterion and detect streams, %d steps in flight)' % st.depth)
                                      if st.submit == 'direct' else
                                      (', one hipGraph per step (detect forked onto its own stream inside it)'
                                       if st.submit == 'fork' else None) or
                                      (', criterion and detect hipGraphs replayed on two streams per step'
                                       if st.two else ', one hipGraph replay per step'))
                                  if st.use_graph else ', eager launches'),
                   'global_batch': world * B, 'n_priors': P, 'n_classes': N_CLASSES,
                   'parallelism': 'dp%d' % world},
        'manchors_per_sec': round(world * B * P * a.steps / elapsed / 1e6, 3),
        'step_algorithmic_bytes': step_bytes,
        'step_GBps_algorithmic': round(step_bytes / (ms_step * 1e-3) / 1e9, 1),
        'step_hbm_frac': round(step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        'graph': st.use_graph, 'stream_priority': a.priority, 'submit_order': a.order,
        'detect_streams': len(st.det_streams), 'criterion_streams': len(st.cap_streams),
        'pipeline_depth': st.depth, 'submit': st.submit,
        'gt_fold': st.gt_fold if st.submit == 'direct' else None,
        'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES'), 'host_sync': a.sync, 'criterion_form': a.crit_form, 'loss_finish': a.finish, 'detect_form': a.det_form,
        'capture_error': st.capture_error,
        'eager_ms_per_step': round(eager_ms, 4) if eager_ms is not None else None,
        'api_ms_per_step': api['ms_per_step'] if api else None,
        'api': api,
    }
    algo = ALGO_BYTES[dominant](wl)
    achieved = algo / dom_avg_s / 1e9
    line['roofline'] = {
        'bound': 'hbm', 'achieved': round(achieved, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
        'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': pmc_traffic(dominant),
        'kernel': dominant, 'launches_timed': n_dom, 'avg_us': round(dom_avg_s * 1e6, 2),
        'timing': ('HIP start/stop events attached to each dispatch (hipExtLaunchKernel) on its '
                   'launch stream, %d eager %s halves of the step alone, rotating %d HBM-resident '
                   'batches' % (max(a.timing_steps, 10), half, len(st.batches))),
        'in_step_avg_us': kernel_us.get(dominant),
        'algorithmic_bytes_per_launch': algo,
        'trace_window_ns': [t_win0, t_win1],
    }
    if spans:
        sp = sum(spans) / len(spans)
        line['roofline']['graph_span'] = {
            'avg_us': round(sp * 1e3, 2), 'samples': len(spans),
            'frac': round(algo / (sp * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            'timing': 'in the replayed graph: first workgroup start to last workgroup end '
                      '(s_memrealtime), excludes the dispatch ramp and the end-of-kernel release',
            'clock_hz': L.lib().sbod_timing_clock_hz()}
    line['roofline_other'] = {
        k: {'avg_us': round(sk * 1e6, 2), 'launches_timed': nk, 'in_step_avg_us': kernel_us.get(k),
            'algorithmic_bytes_per_launch': ALGO_BYTES[k](wl),
            'frac': round(ALGO_BYTES[k](wl) / sk / 1e9 / HBM_PEAK_GBS, 4), 'trace_window_ns': [w0, w1]}
        for k, (nk, sk, w0, w1) in others.items()}
    line['kernel_us_per_step'] = kernel_us
    line['kernel_launches_timed'] = kernel_n
    line['resident_batches'] = len(st.batches)
    if st.use_graph:   # host time per step: GT packing + replays, and collecting the lists
        line['timed_run_detail'] = run_detail
        line['host_us_per_step'] = {'submit': round(host_submit / a.steps * 1e6, 1),
                                    'collect_incl_wait': round(host_collect / a.steps * 1e6, 1)}
    if dp is not None:
        line['dp_train_step_with_grad_allreduce'] = dp
    if not a.no_c2 and world == 1:
        line['c2_bf16'] = c2_figure(dev, a.steps, a.warmup, det_form=a.c2_det_form, finish=a.c2_finish)
    if not a.no_dcn:
        maps = [dcn_figure(dev, H=h, iters=5 if h >= 32 else 20) for h in (64, 32, 16, 8)]
        tot_ms = sum(m['ms'] for m in maps)
        tot_tf = sum(3 * 2.0 * 16 * h * h * 256 * 256 * 9 for h in (64, 32, 16, 8)) / tot_ms / 1e9
        line['dcn'] = dict(maps[0], maps={str(h): m for h, m in zip((64, 32, 16, 8), maps)},
                           c4_all_maps={'ms': round(tot_ms, 3), 'tflops': round(tot_tf, 2),
                                        'mfma_frac': round(tot_tf / F32_MFMA_PEAK_TFS, 4)})
    if not a.no_cpu_baseline:
        line['cpu_baseline'] = cpu_baseline(B, min(os.cpu_count() or 1, 16))
        if not a.no_dcn:   # the DCN leg: TF/s of the oracle beside the GPU figure in line['dcn']
            line['cpu_baseline']['dcn'] = dcn_cpu_baseline(min(os.cpu_count() or 1, 16))
            if 'dcn' in line:
                line['dcn']['cpu_baseline_tflops'] = line['cpu_baseline']['dcn']['tflops']
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
