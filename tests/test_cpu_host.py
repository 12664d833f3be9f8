"""CPU-only checks: the C-ABI library loads and exports every declared symbol (no compute calls),
host-side logic (criterion specs, config handling, loud rejection of CPU tensors)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import REPO
from shape_based_object_detection_amd import _lib as L
from shape_based_object_detection_amd import core, synth
from shape_based_object_detection_amd.models import criteria as CR
from shape_based_object_detection_amd.models.priors import prior_table


def declared_symbols():
    src = open(os.path.join(REPO, 'include', 'sbod.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(sbod_[a-z0-9_]+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    lib = L.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert missing == [], missing
    assert set(syms) <= set(L.SIGNATURES), set(syms) - set(L.SIGNATURES)
    assert L.MISSING == []
    assert lib.sbod_abi_version() == 4
    assert b'gfx950' in lib.sbod_version()


def test_fastcall_wraps_every_launch_entry_point():
    # _sbodcall (generated from SIGNATURES) covers every int / size_t entry point and returns
    # what the ctypes binding returns for the same arguments
    lib = L.lib()
    want = sorted(n for n, (res, args) in L.SIGNATURES.items()
                  if res in (L.I32, L.SZ) and ctypes.c_char_p not in args)
    assert L.fastcall_names() == want
    for n in ('sbod_loss_workspace_bytes', 'sbod_detect_workspace_bytes', 'sbod_match_workspace_bytes_p'):
        args = (32, 10248, 21)[:len(L.SIGNATURES[n][1])]
        assert L._fast[n](*args) == getattr(lib, n)(*args)
    with pytest.raises(TypeError):
        L._fast['sbod_multibox_loss'](1, 2)


def test_invalid_arguments_return_status_not_crash():
    # argument validation happens on the host before any HIP call
    with pytest.raises(L.SbodError, match='bad arguments'):
        L.call('sbod_match_f32', None, None, None, 0, 0, None, None, None, 0, 0.5, 0.01, 0,
               None, None, None, None, 0, None)
    with pytest.raises(L.SbodError, match='workspace'):
        L.call('sbod_multibox_loss', 8, 8, 0, 1, 1, 21, 8, None, None, 8, 8, 8, 8, 8, 8, 8, 0.5, 0.4,
               0.01, 2, 0, 0, 3, 1.0, 0.25, 2.0, None, None, 8, 8, 0, None)


def test_cpu_tensors_rejected_loudly():
    boxes, labels = synth.make_gt(2, seed=0)
    with pytest.raises(L.SbodError, match='ROCm device'):
        core.pack_gt(boxes, labels)
    with pytest.raises(RuntimeError, match='non-zero size'):
        core.pack_gt([torch.zeros(0, 4)], [torch.zeros(0, dtype=torch.long)])


class Cfg(dict):
    __getattr__ = dict.__getitem__


@pytest.mark.parametrize('cls,reg,clsl,exp_reg,exp_cls,exp_flags', [
    (CR.MultiBoxLoss512, 'diou', 'focal', 'diou', 'focal', L.LOSS_UNFUSED_FINISH),
    (CR.MultiBoxLoss512, 'smoothl1', 'ce', 'smoothl1', 'ce', L.POOL['nonpos']),
    (CR.MultiBoxLoss300, 'l1', 'ce', 'l1', 'ce', L.POOL['global_neg']),
    (CR.MultiBoxLoss300, 'DIoU', 'Focal', 'diou', 'focal', L.LOSS_UNFUSED_FINISH),
    (CR.RetinaFocalLoss, 'diou', 'focal', 'diou', 'focal', L.LOSS_FOCAL_NORM | L.LOSS_UNFUSED_FINISH),
    (CR.RetinaFocalLoss, 'smoothl1', 'ce', 'smoothl1', 'ce', L.POOL['neg']),
])
def test_criterion_specs_follow_reference(cls, reg, clsl, exp_reg, exp_cls, exp_flags, monkeypatch):
    # construct without touching the device: patch the codec used for priors_xy
    monkeypatch.setattr(CR, 'cxcy_to_xy', lambda t: t)
    c = cls(priors_cxcy=torch.zeros(4, 4), config=Cfg(reg_weights=2.0, device='cpu', n_classes=21,
                                                      reg_loss=reg, cls_loss=clsl))
    s = c._spec()
    # focal: the separate loss finish is the default (criteria.py separate_finish)
    assert (s.reg, s.cls, s.flags) == (L.REG[exp_reg], L.CLS[exp_cls], exp_flags)
    if exp_cls == 'focal':
        c.separate_finish = False
        assert c._spec().flags == exp_flags & ~L.LOSS_UNFUSED_FINISH
        c.separate_finish = True
    assert s.reg_weight == 2.0 and s.neg_pos_ratio == 3
    c.increase_threshold()
    assert abs(c.threshold - 0.6) < 1e-12
    if cls is CR.MultiBoxLoss300 and clsl == 'ce':
        c.distributed = True   # global mining across ranks: same spec, pools exchanged per call
        assert c._spec().flags == exp_flags


def test_criterion_entry_names():
    assert CR.criterion_entry('ssd512') is CR.MultiBoxLoss512
    assert CR.criterion_entry('RETINA101') is CR.RetinaFocalLoss
    assert CR.criterion_entry('refinedet') is CR.RefineDetLoss
    with pytest.raises(NotImplementedError):
        CR.criterion_entry('FCOS50')


def test_synth_recipe_is_deterministic():
    b1, l1 = synth.make_gt(3, seed=5)
    b2, l2 = synth.make_gt(3, seed=5)
    assert all(torch.equal(x, y) for x, y in zip(b1, b2))
    assert all(torch.equal(x, y) for x, y in zip(l1, l2))
    for b in b1:
        assert (b[:, 2:] > b[:, :2]).all() and (b >= 0).all() and (b <= 1.02).all()
    loc, sc = synth.make_preds(2, prior_table('SSD300').shape[0], 21, seed=1, bg_shift=6.0)
    assert loc.shape == (2, 8732, 4) and sc.shape == (2, 8732, 21)
    assert sc[..., 0].mean() > 5.0


def test_no_kernel_spills_to_scratch():
    """Every HIP kernel keeps its locals in registers/LDS: a scratch (private memory) array is
    the classic silent slowdown (a conditionally written local array demoted by the compiler).
    The table is written by build.py from the compiler's kernel-resource-usage remarks."""
    import json
    path = os.path.join(REPO, 'shape_based_object_detection_amd', 'lib', 'kernel_resources.json')
    if not os.path.exists(path):
        pytest.skip('library not built with resource remarks')
    usage = json.load(open(path))
    assert len(usage) >= 20
    ours = {k: v for k, v in usage.items() if 'sbod' in k}     # library (rocPRIM) kernels excluded
    assert len(ours) >= 20
    bad = {k: v['ScratchSize'] for k, v in ours.items() if v.get('ScratchSize', 0) > 0}
    assert bad == {}, bad


def test_product_library_has_no_ab_variants():
    """the losing A/B forms are out of the product library — no one-launch
    criterion kernel (k_multibox<..., true>: workgroups waiting on each other), no multi-tile loss
    pass (k_multibox_tiles), and sbod_build_variants() says so; asking for the one-launch form
    raises instead of silently running two launches."""
    import json
    path = os.path.join(REPO, 'shape_based_object_detection_amd', 'lib', 'kernel_resources.json')
    if not os.path.exists(path):
        pytest.skip('library not built with resource remarks')
    usage = json.load(open(path))
    assert not [k for k in usage if 'k_multibox' in k and 'Lb1E' in k]
    assert not [k for k in usage if 'k_multibox_tiles' in k]
    assert L.lib().sbod_build_variants() == 0
    assert not hasattr(L.lib(), 'sbod_set_multibox_tiles')
    spec = core.CriterionSpec(L.REG['diou'], L.CLS['focal'])
    with pytest.raises(L.SbodError, match='variant library'):
        core.criterion_focal(torch.zeros(1, 8, 4), torch.zeros(1, 8, 21), None, None, None, spec, 0.5, 0.4,
                             two_launch=False)


def test_stress_anchor_generator_size():
    # SURVEY §8 C3 stress size: RetinaNet's generator on 896x896 maps
    assert prior_table('RETINA896').shape == (100254, 4)


def test_model_entry_registry():
    """models/__init__.py:8-32 contract: (network, criterion class) from config.model['arch']."""
    from shape_based_object_detection_amd import models as MD

    class Cfg(dict):
        __getattr__ = dict.__getitem__

    made = {}

    def ssd512(n_classes, device=None):
        made['ssd512'] = (n_classes, device)
        return 'net512'

    def refinedet(n_classes, config=None):
        made['refine'] = (n_classes, config is not None)
        return 'netrefine'

    MD.register_network('SSD512', ssd512)
    MD.register_network('refinedet', refinedet)
    net, crit = MD.model_entry(Cfg(model={'arch': 'ssd512'}, n_classes=21, device='cpu'))
    assert net == 'net512' and crit is MD.MultiBoxLoss512 and made['ssd512'] == (21, 'cpu')
    net, crit = MD.model_entry(Cfg(model={'arch': 'RefineDet'}, n_classes=21, device='cpu'))
    assert net == 'netrefine' and crit is MD.RefineDetLoss and made['refine'] == (21, True)
    with pytest.raises(NotImplementedError, match='register_network'):
        MD.model_entry(Cfg(model={'arch': 'RETINA50'}, n_classes=21, device='cpu'))
    with pytest.raises(NotImplementedError):
        MD.model_entry(Cfg(model={'arch': 'FCOS50'}, n_classes=21, device='cpu'))


def test_workspace_layout_queries():
    """Size / offset queries answer from the layout alone (no workspace): the mining pool sits
    past the per-block partials and inside the loss workspace; the detect counters lead theirs."""
    lib = L.lib()
    for B, P in ((8, 8732), (32, 10248), (1, 7)):
        off, nb = lib.sbod_loss_pool_offset(B, P), lib.sbod_loss_workspace_bytes(B, P)
        assert 0 < off and off + 4 * B * P <= nb
    assert lib.sbod_detect_counter_bytes(32, 21) <= lib.sbod_detect_workspace_bytes(32, 10248, 21)
    assert lib.sbod_match_ssd_workspace_bytes(5, 8732) >= 5 * 8 + 8732 * 8
    assert lib.sbod_match_ssd_workspace_bytes(0, 8732) == 0
    assert 0 < lib.sbod_dcn_fwd_workspace_bytes(2, 8, 9, 9, 8, 3, 1, 1) < lib.sbod_dcn_workspace_bytes(2, 8, 9, 9, 8, 3, 1, 1)
    assert lib.sbod_dcn_workspace_bytes(2, 8, 9, 9, 8, 3, 0, 1) == 0      # stride 0: invalid, no SIGFPE
    # the training form: forward-only workspace < state; the stateless backward's workspace is
    # exactly the state followed by the scratch
    d = (16, 256, 64, 64, 256, 3, 1, 1)
    assert lib.sbod_dcn_fwd_workspace_bytes(*d) < lib.sbod_dcn_state_bytes(*d)
    assert lib.sbod_dcn_state_bytes(*d) + lib.sbod_dcn_scratch_bytes(*d) == lib.sbod_dcn_workspace_bytes(*d)
    assert lib.sbod_dcn_state_bytes(2, 8, 9, 9, 8, 3, 0, 1) == lib.sbod_dcn_scratch_bytes(2, 8, 9, 9, 8, 3, 0, 1) == 0
