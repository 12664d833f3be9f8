"""detect with the per-class NMS and the per-image merge in ONE launch (k_det_nms: the image's
last class runs the merge) against the two-launch form (k_det_segment + k_det_merge with its
inline second window) and the oracle: boxes, labels, scores and counts bit-identical, including
images whose first 64-candidate windows cannot decide the output (the one-launch form reports
-1 and the host re-runs the call wider)."""
import numpy as np
import pytest
import torch

from oracle import match_ref as M
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models.priors import prior_table

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('B,bg,top_k', [(32, 6.0, 200), (4, 2.0, 50), (3, 9.0, 200), (2, 6.0, 400),
                                        (5, 0.0, 200), (4, 4.0, 20)])
def test_one_launch_equals_two_launches(B, bg, top_k):
    Pn = prior_table('SSD512')
    P = torch.from_numpy(Pn).to(DEV)
    locs, scores = synth.make_preds(B, Pn.shape[0], 21, seed=100 + B, bg_shift=bg)
    l, s = locs.to(DEV), scores.to(DEV)
    one = core.detect(l, s, 0.01, 0.45, top_k, P, two_pass=False)
    two = core.detect(l, s, 0.01, 0.45, top_k, P, two_pass=True)
    for a, b in zip(one, two):
        assert len(a) == len(b) == B
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    if B <= 5:   # and the oracle on the kernels' own activations / decodes
        (ob, ol, os_), probs, bxs = core.detect(l, s, 0.01, 0.45, top_k, P, debug=True, two_pass=False)
        rb, rl, rs = M.detect(probs.cpu().numpy(), bxs.cpu().numpy(), 0.01, 0.45, top_k, nms_variant='tv')
        for i in range(B):
            np.testing.assert_array_equal(ol[i].cpu().numpy(), rl[i])
            np.testing.assert_array_equal(os_[i].cpu().numpy(), rs[i])
            np.testing.assert_array_equal(ob[i].cpu().numpy(), rb[i])


def test_one_launch_counters_left_zero_and_repeatable():
    """Repeated calls on the cached workspace (candidate counters and per-image arrival words are
    left zero by the image's merge) give identical outputs, across batch sizes."""
    Pn = prior_table('SSD512')
    P = torch.from_numpy(Pn).to(DEV)
    locs, scores = synth.make_preds(6, Pn.shape[0], 21, seed=7, bg_shift=6.0)
    l, s = locs.to(DEV), scores.to(DEV)
    res = [core.detect(l[:B].contiguous(), s[:B].contiguous(), 0.01, 0.45, 200, P, two_pass=False)
           for B in (6, 3, 6)]
    for a, b in zip(res[0], res[2]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    for a, b in zip(res[1], res[0]):   # B=3 of the same seed: the first three images
        for x, y in zip(a, b[:3]):
            assert torch.equal(x, y)


def test_counter_prefix_clean_across_batch_sizes():
    """The zero-on-entry prefix is the ALIGNED counter region: B=3 puts its decoded boxes inside
    the alignment padding of B=6's prefix, B=6 (larger, so it zeroes its own prefix) must zero
    that padding too, because B=8 then trusts the same aligned prefix to be zero (its counters
    reach into it).  Every call on one stream's workspace equals the same call on a fresh one."""
    Pn = prior_table('SSD512')
    P = torch.from_numpy(Pn).to(DEV)
    locs, scores = synth.make_preds(8, Pn.shape[0], 21, seed=41, bg_shift=6.0)
    l, s = locs.to(DEV), scores.to(DEV)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        seq = [core.detect(l[:B].contiguous(), s[:B].contiguous(), 0.01, 0.45, 200, P, two_pass=tp)
               for tp in (False, True) for B in (3, 6, 8)]
    torch.cuda.current_stream().wait_stream(side)
    for B, got in zip((3, 6, 8) * 2, seq):
        fresh = torch.cuda.Stream()
        fresh.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(fresh):
            ref = core.detect(l[:B].contiguous(), s[:B].contiguous(), 0.01, 0.45, 200, P)
        torch.cuda.current_stream().wait_stream(fresh)
        for a, b in zip(got, ref):
            for x, y in zip(a, b):
                assert torch.equal(x, y)


@pytest.mark.parametrize('fused', [False, True])
def test_poisoned_candidate_region_reports_corrupt_not_fault(fused):
    """a detect workspace whose zero-on-entry contract is broken (stale counters
    and candidate keys that decode to prior indices >= P) must never read out of bounds: the
    image's count comes back SBOD_DETECT_CORRUPT (-2) through the C ABI, the other images are
    exact, the call leaves the counters zero, and the next call on the same workspace is exact."""
    from shape_based_object_detection_amd import _lib as L
    Pn = prior_table('SSD512')
    pri = torch.from_numpy(Pn).to(DEV)
    B, C, P, top_k = 3, 21, Pn.shape[0], 200
    locs, scores = synth.make_preds(B, P, C, seed=13, bg_shift=6.0)
    l, s = locs.to(DEV), scores.to(DEV)
    lib = L.lib()
    nb = lib.sbod_detect_workspace_bytes(B, P, C)
    ws = torch.zeros(nb, dtype=torch.uint8, device=DEV)
    out_b = torch.empty(B, top_k, 4, device=DEV)
    out_l = torch.empty(B, top_k, dtype=torch.int64, device=DEV)
    out_s = torch.empty(B, top_k, device=DEV)
    cnt = torch.empty(B, dtype=torch.int32, device=DEV)
    flags = L.DETECT_COUNTERS_ZEROED | (L.DETECT_FUSED if fused else 0)

    def run():
        L.call('sbod_detect_f32', L.ptr(l), L.ptr(s), B, P, C, L.ptr(pri), None, L.BOX['offset'], L.ACT['softmax'],
               0.01, 0.45, top_k, -1.0, 0, flags, L.ptr(out_b), L.ptr(out_l), L.ptr(out_s), L.ptr(cnt), None, None,
               None, L.ptr(ws), nb, L.stream_of(s))
        torch.cuda.synchronize()
        return cnt.cpu().tolist(), out_b.clone(), out_l.clone(), out_s.clone()

    good = run()   # a clean workspace (zeroed above)
    # the contract broken on purpose: image 0, class 1 claims 100 stale candidates whose keys carry
    # the highest score (so they are selected) and a prior index far beyond P
    cnt_off = 0
    cand_off = -(-(B * C * 4 + B * 4) // 256) * 256   # the keys follow the counters (no box plane since r6)
    counters = ws[cnt_off:cnt_off + B * C * 4].view(torch.int32)
    counters[1] = 100
    seg = ws[cand_off + (0 * C + 1) * P * 8:cand_off + (0 * C + 1) * P * 8 + 100 * 8].view(torch.int64)
    seg.fill_(-0xfefeff)   # 0xffffffff_ff010101: score ord 0xffffffff, prior index 0x00fefefe >= P
    torch.cuda.synchronize()
    bad = run()
    assert bad[0][0] == L.DETECT_CORRUPT, bad[0]
    for i in (1, 2):   # the other images are untouched
        n = good[0][i]
        assert bad[0][i] == n
        for k in (1, 2, 3):
            assert torch.equal(bad[k][i, :n], good[k][i, :n])
    assert int(counters.abs().sum()) == 0   # left zero by the merge, as after any call
    again = run()
    assert again[0] == good[0]
    for k in (1, 2, 3):
        assert torch.equal(again[k], good[k])
