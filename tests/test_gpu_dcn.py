"""DeformConv2d (a14) on the HIP path vs the reference's golden vectors and the CPU oracle.

Truth: the reference's arithmetic evaluated in fp64 (the oracle, oracle/dcn_ref.py, on float64
inputs; the golden cases' module in fp64 with the golden parameters).  Our fp32 result is
compared with it per element:

    |ours - truth| <= 1e-4 * |truth| + atol,   atol = LAMBDA * sqrt(K) * eps32 * S

with K the number of fp32 products summed into one element and S the largest magnitude one
product can have —
  out     K = C*k²        S = max|x| * max|W|
  grad_x  K = 4*k²*O * 4  S = max|W| * max|grad_out|     (4 corners; neighbouring pixels' samples
                                                          may land on one input pixel: x4)
  grad_offset / grad_mask  K = 4*C*O  S = max|x| * max|W| * max|grad_out|
  grad_W  K = 4*B*Ho*Wo   S = max|x| * max|grad_out|
so entries above the floor atol / 1e-4 are held to 1e-4 RELATIVE, the rest to atol.  sqrt(K) is
the statistical growth of K rounding errors; LAMBDA = 4 because a sequential fp32 sum's error is
not a pure random walk (each rounding scales with the running partial sum) and the maximum over
10^5-10^6 elements sits several standard deviations out: the reference's OWN fp32 evaluation
(the golden vectors, or the oracle in fp32) measured against the same truth needs LAMBDA up to
~1.5 on the small golden cases (reported as ref32_* in every record).  The p_conv / m_conv
parameter gradients and the module's grad_x add the error their inputs' own 1e-4 propagates
(1e-4 * the fp64 contraction of the absolute values) to each element's tolerance.
Every comparison records K, atol, the entries above the floor, the observed maximum relative
error above it and the largest error / tolerance ratio (ours and the fp32 reference's); `pytest -s`
prints them (DCN-TOL lines) and SBOD_DCN_TOL_REPORT=<path> appends them as JSON lines.
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from oracle import dcn_ref as DR
from shape_based_object_detection_amd import core
from shape_based_object_detection_amd.operators.Deformable_convolution import DeformConv2d

pytestmark = pytest.mark.gpu
DEV = 'cuda'
EPS32 = float(np.finfo(np.float32).eps)
LAMBDA = 4.0


def _np(t):
    return t.detach().float().cpu().numpy() if torch.is_tensor(t) else np.asarray(t)


def _amax(t):
    a = _np(t)
    return float(np.abs(a).max()) if a.size else 0.0


def close(ours, truth, K, S, what, ref32=None, extra_atol=None):
    """ours (HIP, fp32) vs `truth` — the reference's arithmetic evaluated in fp64 (the oracle on
    float64 inputs) — per element: |ours - truth| <= 1e-4 |truth| + sqrt(K) eps32 S (+ extra_atol,
    an element-wise array: error a previous step's own 1e-4 propagates into this one).  ref32 (the
    fp32 reference: the golden vectors) is measured against the same truth and reported, not
    asserted: two fp32 evaluations of one contraction differ by both of their errors."""
    ours, truth = _np(ours).astype(np.float64), _np(truth).astype(np.float64)
    assert ours.shape == truth.shape, (what, ours.shape, truth.shape)
    atol = LAMBDA * float(np.sqrt(K)) * EPS32 * S
    tol = 1e-4 * np.abs(truth) + atol + (extra_atol if extra_atol is not None else 0.0)
    err = np.abs(ours - truth)
    big = np.abs(truth) > atol / 1e-4
    rec = {'what': what, 'K': int(K), 'lambda': LAMBDA, 'atol': atol, 'entries_above_floor': int(big.sum()), 'n': int(err.size),
           'max_rel_above_floor': float((err[big] / np.abs(truth[big])).max()) if big.any() else 0.0,
           'max_err_over_tol': float((err / tol).max()) if err.size else 0.0}
    if ref32 is not None:
        r = np.abs(_np(ref32).astype(np.float64) - truth)
        rec['ref32_max_rel_above_floor'] = float((r[big] / np.abs(truth[big])).max()) if big.any() else 0.0
        rec['ref32_max_err_over_tol'] = float((r / tol).max()) if r.size else 0.0
    print('DCN-TOL %s' % json.dumps(rec))
    path = os.environ.get('SBOD_DCN_TOL_REPORT')
    if path:
        with open(path, 'a') as f:
            f.write(json.dumps(rec) + '\n')
    worst = np.unravel_index(int(np.argmax(err / tol)), err.shape) if err.size else ()
    assert rec['max_err_over_tol'] <= 1.0, (what, rec, 'worst at', worst, float(ours[worst]), float(truth[worst]))


def atols(B, C, O, Ho, Wo, ks, x, w, gout):
    """(K, S) per tensor, as the module docstring states."""
    N = ks * ks
    mx, mw, mg = _amax(x), _amax(w), _amax(gout)
    return {'out': (C * N, mx * mw), 'gx': (16 * N * O, mw * mg), 'goff': (4 * C * O, mx * mw * mg),
            'gmask': (4 * C * O, mx * mw * mg), 'gw': (4 * B * Ho * Wo, mx * mg)}


def test_golden_module_fwd_bwd():
    """The module (offset / mask convs + DCN) on the golden inputs and parameters: every output
    and gradient per element against the fp64 evaluation of the same module (oracle on float64),
    the golden (the reference run in fp32) reported against the same truth."""
    d = load_golden('dcn.npz')
    for k in range(int(d['n_cases'])):
        pre = 'c%d_' % k
        B, C, O, H, W, stride = [int(v) for v in d[pre + 'shape']]
        m = DeformConv2d(C, O, kernel_size=3, padding=1, stride=stride).to(DEV)
        with torch.no_grad():
            for n, p in m.named_parameters():
                p.copy_(torch.from_numpy(d[pre + 'w_' + n.replace('.', '_')]))
        x = torch.from_numpy(d[pre + 'x']).to(DEV).requires_grad_(True)
        gcap = {}   # the offset / mask gradients the p_conv / m_conv backward contracts
        for cn in ('p_conv', 'm_conv'):
            getattr(m, cn).register_full_backward_hook(
                lambda mod, gi, go, cn=cn: gcap.__setitem__(cn, go[0].detach().clone()))
        out = m(x)
        gout = torch.from_numpy(d[pre + 'gout']).to(DEV)
        out.backward(gout)
        Ho, Wo = out.shape[2], out.shape[3]
        # the truth: the same module in fp64 (oracle), its gradients by autograd
        prm = {n: torch.from_numpy(d[pre + 'w_' + n.replace('.', '_')]).double().requires_grad_(True)
               for n, _ in m.named_parameters()}
        x64 = torch.from_numpy(d[pre + 'x']).double().requires_grad_(True)
        t_out = DR.deform_module(x64, prm['p_conv.weight'], prm['p_conv.bias'], prm['m_conv.weight'],
                                 prm['m_conv.bias'], prm['conv.weight'], 3, 1, stride)
        t_out.backward(torch.from_numpy(d[pre + 'gout']).double())
        tol = atols(B, C, O, Ho, Wo, 3, x, m.conv.weight, gout)
        close(out, t_out, *tol['out'], pre + 'out', ref32=d[pre + 'out'])
        # x.grad of the MODULE also holds the offset / mask convs' backward (MIOpen) of our offset /
        # mask gradients g, whose own <= 1e-4 relative error that contraction propagates as at
        # most 1e-4 * sum|w_conv||g| per element (fp64), added to the element's tolerance
        prop_x = sum(torch.nn.grad.conv2d_input(tuple(x.shape), getattr(m, cn).weight.detach().double().abs().cpu(),
                                                gcap[cn].double().abs().cpu(), stride=getattr(m, cn).stride,
                                                padding=getattr(m, cn).padding) for cn in ('p_conv', 'm_conv'))
        close(x.grad, x64.grad, *tol['gx'], pre + 'gx', ref32=d[pre + 'gx'], extra_atol=1e-4 * prop_x.numpy())
        for n, p in m.named_parameters():
            ref = d[pre + 'g_' + n.replace('.', '_')]
            if n == 'conv.weight':
                close(p.grad, prm[n].grad, *tol['gw'], pre + 'g_' + n, ref32=ref)
            else:
                # p_conv / m_conv parameters: torch's conv backward (MIOpen) of OUR offset / mask
                # gradient g, a second contraction over every output pixel (K = B*Ho*Wo products
                # per element).  g carries its own <= 1e-4 relative error (the goff / gmask checks),
                # which the contraction propagates as at most 1e-4 * sum|x||g| per element: that
                # sum (fp64) is added to the element's tolerance.
                cn = n.split('.')[0]
                conv = getattr(m, cn)
                g = gcap[cn].double().cpu()
                xd = x.detach().double().cpu()
                if n.endswith('weight'):
                    prop = torch.nn.grad.conv2d_weight(xd.abs(), conv.weight.shape, g.abs(), stride=conv.stride,
                                                       padding=conv.padding)
                    S2 = _amax(xd) * _amax(g)
                else:
                    prop, S2 = g.abs().sum((0, 2, 3)), _amax(g)
                close(p.grad, prm[n].grad, B * Ho * Wo, S2, pre + 'g_' + n, ref32=ref,
                      extra_atol=1e-4 * prop.numpy())


def _oracle_case(B, C, O, H, W, ks, pad, stride, modulation, off_scale, seed):
    g = torch.Generator().manual_seed(seed)
    N = ks * ks
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    x = torch.randn(B, C, H, W, generator=g)
    off = torch.randn(B, 2 * N, Ho, Wo, generator=g) * off_scale
    ml = torch.randn(B, N, Ho, Wo, generator=g) * 2 if modulation else None
    w = torch.randn(O, C, ks, ks, generator=g) / (C * N) ** 0.5
    gout = torch.randn(B, O, Ho, Wo, generator=g)
    # truth: the oracle (the reference's forward restated in torch) on float64 inputs, autograd;
    # the same in fp32 (the reference's own precision) is reported against it
    res = {}
    for dt in (torch.float64, torch.float32):
        xr, offr, wr = (t.detach().clone().to(dt).requires_grad_(True) for t in (x, off, w))
        mlr = ml.detach().clone().to(dt).requires_grad_(True) if modulation else None
        ref = DR.deform_conv2d(xr, offr, torch.sigmoid(mlr) if modulation else None, wr, ks, pad, stride)
        ref.backward(gout.to(dt))
        res[dt] = (ref.detach(), xr.grad, offr.grad, wr.grad, mlr.grad if modulation else None)
    ref, gxr, goffr, gwr, gmr = res[torch.float64]
    r32 = res[torch.float32]
    # HIP path
    xd, offd, wd = (t.to(DEV).requires_grad_(True) for t in (x, off, w))
    mld = ml.to(DEV).requires_grad_(True) if modulation else None
    out = core.deform_conv2d(xd, offd, mld, wd, ks, pad, stride)
    out.backward(gout.to(DEV))
    tag = 'B%d C%d O%d %dx%d k%d pad%d s%d mod%d' % (B, C, O, H, W, ks, pad, stride, modulation)
    tol = atols(B, C, O, Ho, Wo, ks, x, w, gout)
    close(out, ref, *tol['out'], tag + ' out', ref32=r32[0])
    close(xd.grad, gxr, *tol['gx'], tag + ' gx', ref32=r32[1])
    close(offd.grad, goffr, *tol['goff'], tag + ' goff', ref32=r32[2])
    close(wd.grad, gwr, *tol['gw'], tag + ' gw', ref32=r32[3])
    if modulation:
        close(mld.grad, gmr, *tol['gmask'], tag + ' gmask', ref32=r32[4])


@pytest.mark.parametrize('B,C,O,H,W,ks,pad,stride,mod,off_scale', [
    (1, 8, 6, 9, 9, 3, 1, 1, True, 1.0),
    (2, 5, 4, 7, 10, 3, 1, 2, True, 2.0),
    (2, 7, 5, 8, 6, 3, 0, 1, True, 1.5),       # no zero padding
    (1, 6, 3, 9, 7, 3, 2, 1, False, 1.0),      # wider padding, no modulation
    (1, 4, 7, 8, 8, 5, 2, 1, True, 1.0),       # kernel 5
    (1, 8, 16, 9, 9, 7, 3, 1, True, 1.0),      # kernel 7 (the forward's coefficient LDS > 64 KB)
    (1, 3, 4, 6, 6, 2, 1, 1, True, 0.7),       # even kernel
    (2, 6, 5, 7, 7, 3, 1, 1, True, 8.0),       # offsets far outside: border clamp everywhere
    (1, 64, 96, 13, 11, 3, 1, 1, True, 1.0),   # K, M, O not multiples of the tiles
    (2, 32, 300, 9, 9, 3, 1, 2, True, 1.0),    # O > 256: two output-channel groups
    (2, 40, 64, 11, 13, 3, 1, 1, True, 1.0),   # C not a multiple of 32 (partial channel tiles)
    (1, 16, 32, 9, 9, 3, 1, 1, True, 6.0),     # large offsets, stride 1
    (1, 24, 32, 10, 10, 1, 0, 1, True, 1.0),   # kernel 1
    (1, 8, 32, 8, 8, 2, 1, 1, False, 1.0),     # even kernel, no modulation
])
def test_against_oracle(B, C, O, H, W, ks, pad, stride, mod, off_scale):
    _oracle_case(B, C, O, H, W, ks, pad, stride, mod, off_scale, seed=B * 1000 + C * 10 + ks)


def test_c4_dcn_full_channels_vs_oracle():
    # C4 channel count (256 -> 256) at a spatial size the CPU oracle finishes in seconds
    _oracle_case(2, 256, 256, 16, 16, 3, 1, 1, True, 1.0, seed=4)


def test_c4_dcn_64x64_random_offsets_vs_oracle():
    # C4's largest map (64 x 64, 256 -> 256) with random offsets and modulation, one image
    _oracle_case(1, 256, 256, 64, 64, 3, 1, 1, True, 1.0, seed=64)


def test_c4_dcn_b16_8x8_full_shape_vs_oracle():
    # C4's smallest map at its full shape (B=16, 256 -> 256, 3x3, 8x8) with random offsets and
    # modulation, forward and all four gradients against the oracle
    _oracle_case(16, 256, 256, 8, 8, 3, 1, 1, True, 1.0, seed=88)


@pytest.mark.parametrize('H,stride', [(64, 1), (32, 1), (16, 2), (8, 1)])
def test_c4_dcn_zero_offset_equals_conv_at_full_size(H, stride):
    """Size-independent property at BASELINE C4 sizes (B=16, 256->256): with zero offsets and no
    modulation every sample lands on an integer grid point, so DeformConv2d(k=3, pad=1, stride)
    is exactly conv2d(x, W, stride, padding=1); gradients w.r.t. x and W must agree too."""
    g = torch.Generator(device=DEV).manual_seed(H)
    B, C, O = 16, 256, 256
    Ho = (H - 1) // stride + 1
    x = torch.randn(B, C, H, H, device=DEV, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, 3, 3, device=DEV, generator=g) / 48.0).requires_grad_(True)
    off = torch.zeros(B, 18, Ho, Ho, device=DEV)
    out = core.deform_conv2d(x, off, None, w, 3, 1, stride)
    gout = torch.randn(out.shape, device=DEV, generator=g)
    out.backward(gout)
    gx, gw = x.grad.clone(), w.grad.clone()
    x.grad = None
    w.grad = None
    # the truth: conv2d in fp64 (torch's GPU fallback convolution), gradients by autograd
    x64, w64 = x.detach().double().requires_grad_(True), w.detach().double().requires_grad_(True)
    ref = F.conv2d(x64, w64, stride=stride, padding=1)
    ref.backward(gout.double())
    tol = atols(B, C, O, Ho, Ho, 3, x, w, gout)
    tag = 'zero-offset %dx%d s%d ' % (H, H, stride)
    close(out, ref, *tol['out'], tag + 'out')
    close(gx, x64.grad, *tol['gx'], tag + 'gx')
    close(gw, w64.grad, *tol['gw'], tag + 'gw')


def test_module_surface_and_host_path():
    """Same parameters as the reference module; CPU tensors take the host path
    (hostpath.deform_conv2d), device tensors the HIP kernels — and the two agree."""
    m = DeformConv2d(4, 6)
    names = sorted(n for n, _ in m.named_parameters())
    assert names == ['conv.weight', 'm_conv.bias', 'm_conv.weight', 'p_conv.bias', 'p_conv.weight']
    assert float(m.p_conv.weight.abs().sum()) == 0.0 and float(m.m_conv.weight.abs().sum()) == 0.0
    with torch.no_grad():
        m.p_conv.weight.normal_(0, 0.3)
        m.m_conv.weight.normal_(0, 0.3)
    x = torch.randn(2, 4, 7, 7)
    host = m(x)
    prm = {n: p.detach().double() for n, p in m.named_parameters()}
    truth = DR.deform_module(x.double(), prm['p_conv.weight'], prm['p_conv.bias'], prm['m_conv.weight'],
                             prm['m_conv.bias'], prm['conv.weight'])
    dev = m.to(DEV)(x.to(DEV)).cpu()
    S = _amax(x) * _amax(m.conv.weight)
    close(dev, truth, 4 * 9, S, 'module device vs fp64', ref32=host)
    close(host, truth, 4 * 9, S, 'module host vs fp64')


@pytest.mark.parametrize('which', ['x', 'offset', 'mask', 'weight', 'offset+mask'])
def test_partial_gradients_match_full_backward(which):
    """Each subset of requested gradients (the backward skips the dx gather, the dcols rows or the
    weight MFMA accordingly) equals the same gradients from a full backward."""
    g = torch.Generator(device=DEV).manual_seed(11)
    B, C, O, H, ks = 2, 48, 64, 12, 3
    x = torch.randn(B, C, H, H, device=DEV, generator=g)
    off = torch.randn(B, 2 * ks * ks, H, H, device=DEV, generator=g)
    ml = torch.randn(B, ks * ks, H, H, device=DEV, generator=g)
    w = torch.randn(O, C, ks, ks, device=DEV, generator=g) / 20
    gout = torch.randn(B, O, H, H, device=DEV, generator=g)
    full = [t.clone().requires_grad_(True) for t in (x, off, ml, w)]
    core.deform_conv2d(*full, ks, 1, 1).backward(gout)
    names = ['x', 'offset', 'mask', 'weight']
    want = set(which.split('+'))
    part = [t.clone().requires_grad_(n in want) for n, t in zip(names, (x, off, ml, w))]
    core.deform_conv2d(*part, ks, 1, 1).backward(gout)
    for n, pf, pp in zip(names, full, part):
        if n == 'weight' and n in want:
            # the weight gradient's pixel slices are summed in slice order (k_wgrad_fold): bitwise
            assert torch.equal(pp.grad, pf.grad), 'partial weight not bit-identical'
        elif n in want:
            # (dx entries and the offset / mask partials are combined by float atomics)
            np.testing.assert_allclose(_np(pp.grad), _np(pf.grad), rtol=1e-5, atol=1e-6 * _amax(pf.grad),
                                       err_msg='partial ' + n)
        else:
            assert pp.grad is None


def test_state_backward_stateless_backward_and_retained_graph():
    """The training form (forward state kept by autograd, sbod_dcn_bwd_state_f32) against the
    C-ABI's stateless sbod_dcn_bwd_f32 (state re-derived in its own workspace), a retained graph's
    second backward (the backward only reads the state) against its first, and the inference
    forward (no state) against the training forward.  The dx entries and the offset / mask
    partials are combined by atomics in arbitrary order: equal within fp32 rounding, not bitwise;
    the weight gradient (per-slice planes summed in slice order) is bitwise."""
    from shape_based_object_detection_amd import _lib as L
    g = torch.Generator(device=DEV).manual_seed(21)
    B, C, O, H, ks = 2, 40, 48, 11, 3
    x = torch.randn(B, C, H, H, device=DEV, generator=g).requires_grad_(True)
    off = torch.randn(B, 2 * ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    ml = torch.randn(B, ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, ks, ks, device=DEV, generator=g) / 20).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=DEV, generator=g)
    ins = (x, off, ml, w)
    out = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
    first = torch.autograd.grad(out, ins, gout, retain_graph=True)
    second = torch.autograd.grad(out, ins, gout)
    with torch.no_grad():
        inf = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
    dims = (B, C, H, H, O, ks, 1, 1)
    nb = L.lib().sbod_dcn_workspace_bytes(*dims)
    ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
    stateless = [torch.empty_like(t) for t in ins]
    L.call('sbod_dcn_bwd_f32', *[L.ptr(t) for t in ins], L.ptr(gout), *dims, *[L.ptr(t) for t in stateless],
           L.ptr(ws), nb, L.stream_of(gout))
    torch.cuda.synchronize()
    np.testing.assert_allclose(_np(inf), _np(out), rtol=1e-5, atol=1e-6 * _amax(out), err_msg='inference fwd')
    assert torch.equal(second[3], first[3]) and torch.equal(stateless[3], first[3]), 'weight gradient not bitwise'
    for n, a, b, c in zip(('x', 'offset', 'mask', 'weight'), first, second, stateless):
        np.testing.assert_allclose(_np(b), _np(a), rtol=1e-5, atol=1e-6 * _amax(a), err_msg='retained ' + n)
        np.testing.assert_allclose(_np(c), _np(a), rtol=1e-5, atol=1e-6 * _amax(a), err_msg='stateless ' + n)


@pytest.mark.parametrize('H', [8, 24])
def test_captured_fwd_bwd_equals_eager(H):
    """A hipGraph captured over forward + autograd backward (as bench.py times DCN) replays to the
    eager values, also after the inputs change in place between replays."""
    g = torch.Generator(device=DEV).manual_seed(H)
    B, C, O, ks = 3, 64, 32, 3
    x = torch.randn(B, C, H, H, device=DEV, generator=g).requires_grad_(True)
    off = torch.randn(B, 2 * ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    ml = torch.randn(B, ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, ks, ks, device=DEV, generator=g) / 24).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=DEV, generator=g)
    ins = (x, off, ml, w)

    def step():
        out = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
        return (out,) + tuple(torch.autograd.grad(out, ins, gout))

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        cap = step()
    for k in range(2):
        with torch.no_grad():   # new inputs in place: the replay must follow them
            x.mul_(0.5 if k else 1.0)
            off.add_(0.25 * k)
        graph.replay()
        torch.cuda.synchronize()
        want = step()
        for n, a, b in zip(('out', 'x', 'offset', 'mask', 'weight'), cap, want):
            np.testing.assert_allclose(_np(a), _np(b), rtol=1e-5, atol=1e-6 * _amax(b), err_msg='replay %d %s' % (k, n))


def test_eager_side_stream_branches_equal_captured_single_stream():
    """At M x O >= 2^24 an eager call runs its independent branches on a side stream (the weight
    layouts beside the transpose + coefficients, the dx scan + fill beside the backward-data
    contraction, the dx gather beside the weight gradient; dcn.hip dcn_side); a captured call keeps
    one stream.  Both give the same values (the fork and the joins only order launches)."""
    g = torch.Generator(device=DEV).manual_seed(64)
    B, C, O, H, ks = 16, 64, 256, 64, 3
    x = torch.randn(B, C, H, H, device=DEV, generator=g).requires_grad_(True)
    off = torch.randn(B, 2 * ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    ml = torch.randn(B, ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, ks, ks, device=DEV, generator=g) / 24).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=DEV, generator=g)
    ins = (x, off, ml, w)
    assert B * H * H * O >= 1 << 24   # dcn.hip kEagerForkWork

    def step():
        out = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
        return (out,) + tuple(torch.autograd.grad(out, ins, gout))

    side = torch.cuda.Stream()   # eager calls and the capture on one stream (see the test below)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        eager = [t.clone() for t in step()]   # the forked form
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        cap = step()
    graph.replay()
    torch.cuda.synchronize()
    for n, a, b in zip(('out', 'x', 'offset', 'mask', 'weight'), cap, eager):
        if n == 'x':   # the dx gather sums each pixel's entries in fill order (atomics): not bitwise
            np.testing.assert_allclose(_np(a), _np(b), rtol=1e-5, atol=1e-6 * _amax(b), err_msg=n)
        else:
            assert torch.equal(a, b), n


@pytest.mark.parametrize('H', [8, 24])
def test_capture_after_eager_default_stream_and_stateless_backward(H):
    """VERDICT r4 item 2 — the sequence that crashed round 4 in capture_end ("DCN
    capture"), restored: an eager forward + backward on the DEFAULT stream, the C-ABI's stateless
    sbod_dcn_bwd_f32 with its own workspace (freed), then a warm-up and a hipGraph capture of
    forward + backward on a side stream.

    Cause: the eager result kept its autograd graph alive, and with it the AccumulateGrad nodes of
    x / offset / mask / weight, which torch creates on the stream current at the forward — the
    default stream.  The side-stream forward reuses those cached nodes, so backward's input
    buffers synchronise the side stream with the DEFAULT stream (torch warns: "The AccumulateGrad
    node's stream does not match ..."); inside the capture that pulls the legacy default stream
    into the graph without a join, and this HIP runtime segfaults in hipStreamEndCapture instead
    of returning an error.  Nothing in libsbod_hip.so is involved (the same crash with both library
    builds; the same sequence with the eager graph released captures fine).  This test shows the
    reuse — a side-stream forward's AccumulateGrad nodes ARE the eager call's while its graph is
    alive (never capturing in that state) — then releases the graph (torch's own advice),
    captures, and checks the replays."""
    from shape_based_object_detection_amd import _lib as L
    g = torch.Generator(device=DEV).manual_seed(H)
    B, C, O, ks = 3, 64, 32, 3
    x = torch.randn(B, C, H, H, device=DEV, generator=g).requires_grad_(True)
    off = torch.randn(B, 2 * ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    ml = torch.randn(B, ks * ks, H, H, device=DEV, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, ks, ks, device=DEV, generator=g) / 24).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=DEV, generator=g)
    ins = (x, off, ml, w)

    def step():
        out = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
        return (out,) + tuple(torch.autograd.grad(out, ins, gout))

    def serial():   # the stateless C-ABI backward: its own workspace, freed at return
        dims = (B, C, H, H, O, ks, 1, 1)
        nb = L.lib().sbod_dcn_workspace_bytes(*dims)
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        res = [torch.empty_like(t) for t in ins]
        L.call('sbod_dcn_bwd_f32', *[L.ptr(t) for t in ins], L.ptr(gout), *dims, *[L.ptr(t) for t in res],
               L.ptr(ws), nb, L.stream_of(gout))
        torch.cuda.synchronize()
        return res

    eager = step()                      # default stream; its graph stays alive in `eager[0]`
    ref = serial()
    for n, a, b in zip(('x', 'offset', 'mask', 'weight'), eager[1:], ref):
        np.testing.assert_allclose(_np(a), _np(b), rtol=1e-5, atol=1e-6 * _amax(b), err_msg='eager ' + n)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())

    def acc_nodes(out):   # the AccumulateGrad nodes of x / offset / mask / weight under `out`
        return [f for f, _ in out.grad_fn.next_functions if f is not None and type(f).__name__ == 'AccumulateGrad']

    # while the eager graph is alive, a side-stream forward reuses its (default-stream) nodes —
    # the state in which a capture crashed (never captured here)
    with torch.cuda.stream(side):
        out_s = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
    reused = acc_nodes(out_s)
    assert len(reused) == 4 and all(a is b for a, b in zip(acc_nodes(eager[0]), reused))
    del out_s, reused
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    eager = [t.detach() for t in eager]   # release the autograd graph (and its default-stream nodes)
    with torch.cuda.stream(side):         # warm-up on the capture stream: its own nodes now
        step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        cap = step()
    for k in range(2):
        with torch.no_grad():   # new inputs in place: the replay must follow them
            x.mul_(0.5 if k else 1.0)
            off.add_(0.25 * k)
        graph.replay()
        torch.cuda.synchronize()
        with torch.cuda.stream(side):   # (eager check on the capture stream: its nodes are the graph's)
            want = step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        for n, a, b in zip(('out', 'x', 'offset', 'mask', 'weight'), cap, want):
            np.testing.assert_allclose(_np(a), _np(b), rtol=1e-5, atol=1e-6 * _amax(b), err_msg='replay %d %s' % (k, n))
