"""Malformed host-side inputs to the C ABI and the _sbodhost extension (host ASan on the
C-ABI shim).  CPU only — every case fails validation, or takes the early return, before any HIP
call.  Runs in the normal CPU suite and, via scripts/asan_host.sh, under AddressSanitizer +
UBSan builds of libsbod_hip.so (host code), _sbodhost.so and _sbodcall.so.
"""
import ctypes

import pytest
import torch

from shape_based_object_detection_amd import _lib as L


@pytest.fixture(scope='module')
def ext():
    L.lib()
    if L.host_ext is None:
        pytest.skip('_sbodhost not built')
    return L.host_ext


def _pack(ext, boxes, labels, capacity=64, per_image=16):
    return ext.pack_device_lists(boxes, labels, capacity, per_image, 0, 0, 0, 0, None, False)


def test_pack_device_lists_rejects_malformed_batches(ext):
    b = [torch.zeros(3, 4), torch.zeros(2, 4)]
    l = [torch.zeros(3, dtype=torch.long), torch.zeros(2, dtype=torch.long)]
    assert _pack(ext, b, l) is None                       # CPU tensors -> the Python path
    assert _pack(ext, tuple(b), l) is None                # not lists
    assert _pack(ext, b, l[:1]) is None                   # length mismatch
    assert _pack(ext, [], []) is None                     # empty batch
    assert _pack(ext, [1, 2], [3, 4]) is None             # not tensors
    assert _pack(ext, [None], [None]) is None
    assert _pack(ext, [torch.zeros(3)], [torch.zeros(3, dtype=torch.long)]) is None
    big = [torch.zeros(100, 4)] * 2
    assert _pack(ext, big, [torch.zeros(100, dtype=torch.long)] * 2) is None
    with pytest.raises(TypeError):
        ext.pack_device_lists(b, l)
    with pytest.raises(TypeError):
        ext.pack_device_lists(b, l, 'x', 1, 0, 0, 0, 0, None, False)


def test_stage_and_replay_rejects_malformed_launches(ext):
    b = [torch.zeros(3, 4)]
    l = [torch.zeros(3, dtype=torch.long)]
    args = [b, l, 64, 16, 0, 0, 0, 0, None, False]
    with pytest.raises(TypeError):
        ext.stage_and_replay(*args, [(0, 0)], None, None, None)      # launches not a tuple
    with pytest.raises(TypeError):
        ext.stage_and_replay(*args, ((0,),), None, None, None)       # pair of the wrong size
    with pytest.raises(TypeError):
        ext.stage_and_replay(*args, ((0, 0),), None, None)           # argument count
    assert ext.stage_and_replay(*args, ((0, 0),), None, None, None) is None   # CPU lists


def _call_all(value):
    lib = L.lib()
    out = {}
    skip = {'sbod_timing_enable', 'sbod_timing_query', 'sbod_timing_every', 'sbod_timing_reset_graphs',
            'sbod_memcpy_d2h_async', 'sbod_stream_wait'}
    for name, (res, args) in L.SIGNATURES.items():
        if name in skip or not args:
            continue
        conv = []
        for t in args:
            if t is ctypes.c_void_p:
                conv.append(None)
            elif t in (ctypes.c_float, ctypes.c_double):
                conv.append(float(value))
            else:
                conv.append(value)
        out[name] = getattr(lib, name)(*conv)
    return out


@pytest.mark.parametrize('value', [0, -1, 7])
def test_every_entry_point_validates_null_and_bad_sizes(value):
    """NULL pointers with zero, negative and small positive sizes: every launching entry point
    returns a status (never dereferences, never launches); size queries return a number."""
    res = _call_all(value)
    for name, (rt, _) in L.SIGNATURES.items():
        if name not in res:
            continue
        if rt is ctypes.c_int and value != 0:
            assert res[name] != 0 or name in ('sbod_codec_f32',), (name, res[name])
    msg = L.lib().sbod_last_error()
    assert isinstance(msg, bytes)


def test_stream_wait_same_stream_is_a_noop():
    assert L.lib().sbod_stream_wait(None, None) == 0


def test_step_program_rejects_malformed_recordings(ext):
    """make_step_program parses the recorded argument tuples once: wrong arities are TypeErrors,
    and submit_step_program needs the capsule it made (nothing is launched on either failure)."""
    def recorded(name):   # a recording of the right types: NULL pointers, zero sizes
        vals = []
        for t in L.SIGNATURES[name][1]:
            vals.append(None if t is ctypes.c_void_p else (0.0 if t in (ctypes.c_float, ctypes.c_double) else 0))
        return tuple(vals)
    pack = (64, 16, 0, 0, 0, 0, None)
    crit = recorded('sbod_criterion_focal')
    det = recorded('sbod_detect_f32')
    assert len(crit) == 28 and len(det) == 25
    with pytest.raises(TypeError):
        ext.make_step_program(pack[:6], crit, det, None, None)
    with pytest.raises(TypeError):
        ext.make_step_program(pack, crit[:27], det, None, None)
    with pytest.raises(TypeError):
        ext.make_step_program(pack, crit, det + (None,), None, None)
    with pytest.raises(TypeError):
        ext.make_step_program(pack, crit, det, None)                          # argument count
    prog = ext.make_step_program(pack, crit, det, None, None, True)
    with pytest.raises((TypeError, ValueError)):
        ext.submit_step_program(object(), [], [])                            # not the capsule
    with pytest.raises(TypeError):
        ext.submit_step_program(prog, [])
    b = [torch.zeros(3, 4)]
    l = [torch.zeros(3, dtype=torch.long)]
    assert ext.submit_step_program(prog, b, l) is None                       # CPU lists: Python path
    assert ext.submit_step_program(prog, b, l, 1) is None                    # the criterion alone too
    for bad in (0, 4, -1):                                                   # parts: 1, 2 or 3
        with pytest.raises(ValueError):
            ext.submit_step_program(prog, b, l, bad)
