"""Device-side ground-truth packing and the hipGraph-captured step.

  * sbod_gt_pack (one launch, pointers in the kernel arguments) == torch.cat of the lists, and
    GtStaging's device-list and host-list paths fill identical fixed-capacity buffers;
  * a criterion forward+backward + detect captured with torch.cuda.graph and replayed gives the
    eager results bit for bit, also after the staged ground truth changes between replays (the
    graph reads the fixed-capacity buffers, not the capture-time lists);
  * a timed kernel inside the capture overwrites its own span record on every replay.
"""
import numpy as np
import pytest
import torch

from shape_based_object_detection_amd import _lib as L
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


class Cfg(dict):
    __getattr__ = dict.__getitem__


def test_gt_pack_matches_cat():
    boxes, labels = synth.make_gt(37, seed=4)           # > 1 chunk? no: 37 < 64; still ragged
    boxes += [torch.zeros(0, 4)]                         # an empty image is packed as 0 rows
    labels += [torch.zeros(0, dtype=torch.int64)]
    bx = [b.to(DEV) for b in boxes]
    lb = [l.to(DEV) for l in labels]
    gt = core.pack_gt(bx, lb, allow_empty=True)
    torch.testing.assert_close(gt.boxes, torch.cat(bx), rtol=0, atol=0)
    assert torch.equal(gt.labels, torch.cat(lb))
    offs = np.concatenate([[0], np.cumsum([b.shape[0] for b in boxes])]).astype(np.int32)
    np.testing.assert_array_equal(gt.offsets.cpu().numpy(), offs)


def test_gt_pack_many_images_chunks():
    boxes, labels = synth.make_gt(150, seed=8)          # 3 launches of <= 64 images
    bx = [b.to(DEV) for b in boxes]
    lb = [l.to(DEV) for l in labels]
    gt = core.pack_gt(bx, lb)
    assert torch.equal(gt.boxes, torch.cat(bx)) and torch.equal(gt.labels, torch.cat(lb))
    offs = np.concatenate([[0], np.cumsum([b.shape[0] for b in boxes])]).astype(np.int32)
    np.testing.assert_array_equal(gt.offsets.cpu().numpy(), offs)


def test_staging_device_and_host_paths_agree():
    boxes, labels = synth.make_gt(16, seed=21)
    st_d = core.GtStaging(16, 16, DEV)
    st_h = core.GtStaging(16, 16, DEV)
    gd = st_d.stage([b.to(DEV) for b in boxes], [l.to(DEV) for l in labels])
    gh = st_h.stage(boxes, labels)                      # CPU lists: pinned pack + one copy
    n = sum(b.shape[0] for b in boxes)
    torch.cuda.synchronize()
    assert gd.gmax == gh.gmax == 16
    assert torch.equal(gd.boxes[:n], gh.boxes[:n]) and torch.equal(gd.labels[:n], gh.labels[:n])
    assert torch.equal(gd.offsets, gh.offsets)
    assert torch.equal(gd.boxes[:n].cpu(), torch.cat(boxes))
    with pytest.raises(ValueError):
        big, bl = synth.make_gt(16, seed=1, max_objects=40)
        st_d.stage([b.to(DEV) for b in big] * 1, [l.to(DEV) for l in bl])


def _setup(B=8, seed=31):
    P = torch.from_numpy(prior_table('SSD512')).to(DEV)
    cfg = Cfg(reg_weights=1.0, device=DEV, n_classes=21, reg_loss='diou', cls_loss='focal')
    crit = CR.MultiBoxLoss512(priors_cxcy=P, config=cfg)
    locs, scores = synth.make_preds(B, P.shape[0], 21, seed=seed)
    det = scores.clone()
    det[:, :, 0] += 6.0
    return P, crit, locs.to(DEV).requires_grad_(True), scores.to(DEV).requires_grad_(True), det.to(DEV)


def _gt(B, seed):
    boxes, labels = synth.make_gt(B, seed=seed)
    return [b.to(DEV) for b in boxes], [l.to(DEV) for l in labels]


def _eager(P, crit, locs, scores, det, gt):
    locs.grad = None
    scores.grad = None
    loss = crit(locs, scores, gt[0], gt[1])
    res = core.detect(locs.detach(), det, 0.01, 0.45, 200, P)
    loss.backward()
    return loss.item(), locs.grad.clone(), scores.grad.clone(), res


def _same_det(a, b):
    for x, y in zip(a, b):
        assert len(x) == len(y)
        for u, v in zip(x, y):
            assert torch.equal(u, v)


def test_graph_replay_equals_eager():
    B = 8
    P, crit, locs, scores, det = _setup(B)
    stage = core.GtStaging(B, 16, DEV)
    side = torch.cuda.Stream()
    ds = torch.cuda.Stream()

    def body(gt, capture):
        loss = crit(locs, scores, gt, None)
        cur = torch.cuda.current_stream()
        ds.wait_stream(cur)
        with torch.cuda.stream(ds):
            h = core.detect(locs.detach(), det, 0.01, 0.45, 200, P, async_=True, capture=capture)
        loss.backward()
        cur.wait_stream(ds)
        return loss, h

    gt1 = _gt(B, 100)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):                      # warm-up (lazy state) off the capture stream
        for _ in range(2):
            locs.grad = None
            scores.grad = None
            _, h = body(stage.stage(*gt1), False)
            h.wait()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    locs.grad = None
    scores.grad = None
    g = torch.cuda.CUDAGraph()
    pack = stage.stage(*gt1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=side):            # capture on the warmed-up stream
        g_loss, g_h = body(pack, True)
    g_gl, g_gs = locs.grad, scores.grad
    for seed in (100, 200, 300):                         # new ground truth every replay
        gt = _gt(B, seed)
        stage.stage(*gt)
        g.replay()
        res = g_h.replayed().wait()
        gl, gs = g_gl.clone(), g_gs.clone()
        lv = g_loss.item()
        e_loss, e_gl, e_gs, e_res = _eager(P, crit, locs, scores, det, gt)
        assert lv == e_loss
        assert torch.equal(gl, e_gl) and torch.equal(gs, e_gs)
        _same_det(res, e_res)
        locs.grad, scores.grad = g_gl, g_gs


def test_stage_and_replay_equals_eager():
    """The one-call submit (C++: GT packing, graph launch, detect event) gives the eager results."""
    B = 8
    P, crit, locs, scores, det = _setup(B, seed=9)
    stage = core.GtStaging(B, 16, DEV)
    side = torch.cuda.Stream()

    def body(gt, capture):
        loss = crit(locs, scores, gt, None)
        h = core.detect(locs.detach(), det, 0.01, 0.45, 200, P, async_=True, capture=capture)
        loss.backward()
        return loss, h

    gt1 = _gt(B, 11)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            locs.grad = None
            scores.grad = None
            _, h = body(stage.stage(*gt1), False)
            h.wait()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    locs.grad = None
    scores.grad = None
    g = torch.cuda.CUDAGraph()
    pack = stage.stage(*gt1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=side):
        g_loss, g_h = body(pack, True)
    g_gl, g_gs = locs.grad, scores.grad
    g_h._event.record(side)                             # the raw event exists from here on
    torch.cuda.synchronize()
    launches = core.graph_launches([(g, side)])
    for seed in (12, 13):
        gt = _gt(B, seed)
        packed = stage.stage_and_replay(list(gt[0]), list(gt[1]), launches, g_h._event.cuda_event,
                                        side.cuda_stream)
        if L.host_ext is None:
            pytest.skip('host extension not built')
        assert packed is not None and packed.counts == [b.shape[0] for b in gt[0]]
        res = g_h.rearmed().wait()
        torch.cuda.synchronize()
        gl, gs = g_gl.clone(), g_gs.clone()
        lv = g_loss.item()
        e_loss, e_gl, e_gs, e_res = _eager(P, crit, locs, scores, det, gt)
        assert lv == e_loss
        assert torch.equal(gl, e_gl) and torch.equal(gs, e_gs)
        _same_det(res, e_res)
        locs.grad, scores.grad = g_gl, g_gs


def test_captured_pack_cache_survives_growth():
    """a criterion captured on list GT packs into the stream's cached pack buffers
    (pack_gt(reuse=True)); a later eager batch that outgrows them must RETIRE those buffers (the
    graph writes them on every replay), not hand them back to the allocator.  The replay after
    the growth still gives the capture-time loss and gradients bit for bit."""
    if L.host_ext is None:
        pytest.skip('host extension not built (no cached pack path)')
    B = 2
    P, crit, locs, scores, det = _setup(B, seed=41)
    gt1 = _gt(B, 42)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):                               # warm-up: the cached pack buffers exist
            locs.grad = None
            scores.grad = None
            crit(locs, scores, gt1[0], gt1[1]).backward()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        locs.grad = None
        scores.grad = None
        l0 = crit(locs, scores, gt1[0], gt1[1])
        l0.backward()
    torch.cuda.synchronize()
    ref_loss, ref_gl, ref_gs = l0.item(), locs.grad.clone(), scores.grad.clone()
    locs.grad = None
    scores.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        g_loss = crit(locs, scores, gt1[0], gt1[1])
        g_loss.backward()
    g_gl, g_gs = locs.grad, scores.grad
    key = (DEV.index, side.cuda_stream, B)
    captured = core._PACK_CACHE[key][0].data_ptr()
    assert captured in core._PACK_CAPTURED
    big_b, big_l = synth.make_gt(B, seed=43, max_objects=300)   # tiled to 300 objects per image
    big_b = [torch.cat([b] * (300 // b.shape[0] + 1))[:300].to(DEV) for b in big_b]
    big_l = [torch.cat([l] * (300 // l.shape[0] + 1))[:300].to(DEV) for l in big_l]
    with torch.cuda.stream(side):                        # 600 rows > the cache's 512: it grows
        locs.grad = None
        scores.grad = None
        crit(locs, scores, big_b, big_l).backward()
    torch.cuda.synchronize()
    assert any(t[0].data_ptr() == captured for t in core._PACK_RETIRED)
    junk = [torch.full((1 << 16,), 7.0, device=DEV) for _ in range(8)]   # reuse freed memory
    locs.grad, scores.grad = g_gl, g_gs
    g.replay()
    torch.cuda.synchronize()
    assert g_loss.item() == ref_loss
    assert torch.equal(g_gl, ref_gl) and torch.equal(g_gs, ref_gs)
    del junk


def test_workspace_allocation_under_capture_refused():
    """A workspace the captured call would allocate under capture fails loudly instead."""
    B = 2
    P, crit, locs, scores, det = _setup(B, seed=6)
    gt = _gt(B, 8)
    stage = core.GtStaging(B, 16, DEV)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    pack = stage.stage(*gt)
    torch.cuda.synchronize()
    with pytest.raises(L.SbodError, match='under hipGraph capture'):
        with torch.cuda.graph(g, stream=s):               # never warmed up on s
            crit(locs, scores, pack, None)


def test_graph_span_timing():
    """A timed kernel captured into a graph overwrites its own span record on every replay; the host
    reads the latest launch without writing anything between replays."""
    B = 4
    P, crit, locs, scores, det = _setup(B, seed=5)
    gt = _gt(B, 7)
    stage = core.GtStaging(B, 16, DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            locs.grad = None
            crit(locs, scores, stage.stage(*gt), None).backward()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    L.timing_enable('k_multibox')
    g = torch.cuda.CUDAGraph()
    locs.grad = None
    scores.grad = None
    with torch.cuda.graph(g, stream=s):
        loss = crit(locs, scores, stage.stage(*gt), None)
        loss.backward()
    L.timing_enable(None)
    assert L.timing_query('k_multibox')[0] == 0          # never replayed yet
    times = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        n, ms = L.timing_query('k_multibox')
        assert n == 1
        times.append(ms)
    assert all(0.0005 < t < 5.0 for t in times), times
    del g
    L.call('sbod_timing_reset_graphs')


@pytest.mark.parametrize('depth,two,submit,fold', [(2, True, 'graph', False), (3, True, 'graph', False),
                                                    (3, False, 'graph', False), (4, True, 'direct', True),
                                                    (4, True, 'direct', False), (4, True, 'fork', False)])
def test_bench_pipelined_step_equals_eager(depth, two, submit, fold):
    """bench.Step as the bench runs it: per-batch criterion and detect graphs, each alternating over
    two streams (or, ``two`` False, one graph per step holding both), submitted by the one-call C++
    path — or, ``submit='direct'``, the recorded entry-point calls issued again without graphs —
    — or, ``submit='fork'``, one graph per step with detect forked onto its stream inside it —
    with ``depth`` steps in flight and a criterion stream current.  Every step's loss, gradients and
    per-image detections equal the eager two-stream step on the same batch, across two rotations
    of the resident batches.  ``fold``: the direct submit's GT packing folded into the matcher's
    first launch (sbod_criterion_focal_lists) instead of a separate sbod_gt_pack launch."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    st = bench.Step(DEV, 4, 0, 1, graph=True, two_streams=two, priority='detect', n_batches=4, det_streams=2,
                    crit_streams=2, depth=depth, submit=submit, gt_fold=fold)
    ref = []
    for bt in st.batches:          # eager reference per batch (also warms both detect streams)
        loss, dets = st.eager_split()
        ref.append((loss.item(), bt.locs.grad.clone(), bt.scores.grad.clone(),
                    [[t.clone() for t in part] for part in dets]))
    for _ in range(2):
        st.eager_split()
    torch.cuda.synchronize()
    st.capture()
    got = []
    with torch.cuda.stream(st.cap_stream):
        for k in range(2 * len(st.batches)):
            out = st.pipelined()
            if out is not None:
                got.append(out)
        got.extend(st.drain())
    torch.cuda.synchronize()
    assert len(got) == 2 * len(st.batches)
    for k, (loss, dets) in enumerate(got):
        rl, rgl, rgs, rd = ref[k % len(st.batches)]
        assert loss.item() == rl
        for part, rpart in zip(dets, rd):
            assert len(part) == len(rpart) == 4
            for a, b in zip(part, rpart):
                assert torch.equal(a, b)
    for i, bt in enumerate(st.batches):   # the captured backward left the same gradients
        assert torch.equal(bt.locs.grad, ref[i][1]) and torch.equal(bt.scores.grad, ref[i][2])


def test_step_program_parts_equal_whole():
    """The native step submit's ``parts`` mask (scripts/gpu_interval.py submits one chain alone):
    the GT packing + criterion (parts=1) and the detect + event (parts=2) issued as two calls leave
    the same loss, gradients and per-image detections as the eager step on the same batch — the
    same launches as the whole submit (parts=3) that test_bench_pipelined_step_equals_eager checks."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    if L.host_ext is None:
        pytest.skip('the _sbodhost extension is not built')
    st = bench.Step(DEV, 4, 0, 1, graph=True, priority='detect', n_batches=4, det_streams=2, crit_streams=2,
                    depth=4, submit='direct', gt_fold=True)
    ref = []
    for bt in st.batches:
        loss, dets = st.eager_split()
        ref.append((loss.item(), bt.locs.grad.clone(), bt.scores.grad.clone(),
                    [[t.clone() for t in part] for part in dets]))
    for _ in range(2):
        st.eager_split()
    torch.cuda.synchronize()
    st.capture()
    assert all(p is not None for p in st.programs)
    for k in range(len(st.batches)):
        i = st.k % len(st.slots)
        bt = st._next_batch()
        _, _, loss, h = st.slots[i]
        order = (2, 1) if k % 2 else (1, 2)   # either chain first
        for parts in order:
            assert L.host_ext.submit_step_program(st.programs[i], bt.boxes, bt.labels, parts) is True
        dets = h.rearmed().wait()
        torch.cuda.synchronize()
        rl, rgl, rgs, rd = ref[i]
        assert loss.item() == rl
        assert torch.equal(bt.locs.grad, rgl) and torch.equal(bt.scores.grad, rgs)
        for part, rpart in zip(dets, rd):
            assert len(part) == len(rpart) == 4
            for a, b in zip(part, rpart):
                assert torch.equal(a, b)
