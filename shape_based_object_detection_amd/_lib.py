"""ctypes binding of libsbod_hip.so (the C ABI in include/sbod.h).

The library is loaded AFTER ``import torch`` so its SONAME ``libamdhip64.so.7`` binds to the HIP
runtime torch already mapped.  There is no fallback: if the library is missing or a call
fails, this raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen; see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SBOD_LIB', os.path.join(_HERE, 'lib', 'libsbod_hip.so'))
FAST_PATH = os.path.join(os.path.dirname(LIB_PATH), '_sbodcall.so')
HOST_PATH = os.path.join(os.path.dirname(LIB_PATH), '_sbodhost.so')

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float
SZ = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/sbod.h one to one.
SIGNATURES = {
    'sbod_version': (ctypes.c_char_p, []),
    'sbod_abi_version': (I32, []),
    'sbod_last_error': (ctypes.c_char_p, []),
    'sbod_build_variants': (I32, []),
    'sbod_null_kernel': (I32, [I32, P]),
    'sbod_iou_pairwise_f32': (I32, [P, P, I32, I32, P, I64, I32, I32, P, P]),
    'sbod_match_workspace_bytes': (SZ, [I32, I32]),
    'sbod_match_workspace_bytes_p': (SZ, [I32, I32, I32]),
    'sbod_match_f32': (I32, [P, P, P, I32, I32, P, P, P, I32, F32, F32, I32, P, P, P, P, SZ, P]),
    'sbod_match_lists_f32': (I32, [P, P, P, I64, P, P, P, I32, I32, P, P, P, I32, F32, F32, I32, P, P, P, P, SZ,
                                   P]),
    'sbod_match_expand_f32': (I32, [P, P, P, I32, P, P, P, P, I32, F32, F32, I32, P, P, P, P, P]),
    'sbod_match_ssd_workspace_bytes': (SZ, [I32, I32]),
    'sbod_match_ssd_f32': (I32, [P, P, I32, P, I32, F32, F32, F32, I32, P, P, P, SZ, P]),
    'sbod_codec_f32': (I32, [I32, P, P, I64, I64, F32, F32, P, P]),
    'sbod_loss_workspace_bytes': (SZ, [I32, I32]),
    'sbod_multibox_loss': (I32, [P, P, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P, P, F32, F32,
                                 F32, I32, I32, I32, I32, F32, F32, F32, P, P, P, P, SZ, P]),
    'sbod_loss_pool_offset': (SZ, [I32, I32]),
    'sbod_loss_zero_bytes': (SZ, [I32, I32]),
    'sbod_criterion_workspace_bytes': (SZ, [I32, I32, I32]),
    'sbod_criterion_zero_bytes': (SZ, [I32, I32, I32]),
    'sbod_criterion_focal': (I32, [P, P, I32, I32, I32, I32, P, P, P, P, P, I32, F32, F32, I32, I32, F32, F32, F32,
                                   P, P, P, P, P, P, P, SZ, P]),
    'sbod_criterion_focal_lists': (I32, [P, P, P, I64, P, P, I32, I32, I32, I32, P, P, P, P, P, I32, F32, F32, I32,
                                         I32, F32, F32, F32, P, P, P, P, P, P, P, SZ, P]),
    'sbod_criterion_status': (I32, [P, P]),
    'sbod_loss_finish_status': (I32, [P, I32, I32, I32, P]),
    'sbod_multibox_mine_global': (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, F32, P, I64, I64, P,
                                        P, P, SZ, P]),
    'sbod_scale_inplace': (I32, [P, I32, I64, P, P]),
    'sbod_scale2_inplace': (I32, [P, I64, P, I64, I32, P, P]),
    'sbod_aligned_overlap_f32': (I32, [I32, P, P, I64, P, P, P, P]),
    'sbod_smooth_l1_f32': (I32, [P, P, I64, F32, P, P, P]),
    'sbod_focal_f32': (I32, [I32, P, P, I64, I32, F32, F32, F32, P, P, P]),
    'sbod_detect_workspace_bytes': (SZ, [I32, I32, I32]),
    'sbod_detect_counter_bytes': (SZ, [I32, I32]),
    'sbod_detect_f32': (I32, [P, P, I32, I32, I32, P, P, I32, I32, F32, F32, I32, F32, I32, I32, P, P,
                              P, P, P, P, P, P, SZ, P]),
    'sbod_nms_workspace_bytes': (SZ, [I64]),
    'sbod_nms_f32': (I32, [P, P, I64, F32, I32, I32, F32, P, P, P, SZ, P]),
    'sbod_map_workspace_bytes': (SZ, [I64, I64]),
    'sbod_map_f32': (I32, [P, P, P, P, P, P, P, P, I32, I32, I64, I64, ctypes.c_double, P, P, P, P, SZ, P]),
    'sbod_timing_enable': (I32, [ctypes.c_char_p]),
    'sbod_timing_query': (I32, [ctypes.c_char_p, P, P]),
    'sbod_timing_every': (I32, [I32]),
    'sbod_timing_reset_graphs': (I32, []),
    'sbod_timing_clock_hz': (ctypes.c_double, []),
    'sbod_memcpy_d2h_async': (I32, [P, P, SZ, P]),
    'sbod_graph_launch': (I32, [P, P]),
    'sbod_event_record': (I32, [P, P]),
    'sbod_stream_wait': (I32, [P, P]),
    'sbod_stream_abort_capture': (I32, [P]),
    'sbod_gt_pack': (I32, [P, P, P, I32, I64, P, P, P, P]),
    'sbod_dcn_workspace_bytes': (SZ, [I32, I32, I32, I32, I32, I32, I32, I32]),
    'sbod_dcn_fwd_workspace_bytes': (SZ, [I32, I32, I32, I32, I32, I32, I32, I32]),
    'sbod_dcn_state_bytes': (SZ, [I32, I32, I32, I32, I32, I32, I32, I32]),
    'sbod_dcn_scratch_bytes': (SZ, [I32, I32, I32, I32, I32, I32, I32, I32]),
    'sbod_dcn_fwd_train_f32': (I32, [P, P, P, P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, SZ, P]),
    'sbod_dcn_bwd_state_f32': (I32, [P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, P, P, P, SZ, P, SZ, P]),
    'sbod_dcn_fwd_f32': (I32, [P, P, P, P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, SZ, P]),
    'sbod_dcn_bwd_f32': (I32, [P, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, I32, P, P, P, P,
                               P, SZ, P]),
}

# Constants of include/sbod.h.
IOU_METRICS, IOU_PLAIN, IOU_INTER = 0, 1, 2
MATCH_BINARY, MATCH_ODM, MATCH_WS_ZEROED = 1, 2, 256
CODEC = dict(xy_to_cxcy=0, cxcy_to_xy=1, encode_tenfive=2, decode_tenfive=3, encode_var=4,
             decode_var=5, decode_tenfive_xy=6)
REG = dict(smoothl1=0, l1=1, diou=2)
CLS = dict(focal=0, ce=1)
DT_F32, DT_BF16 = 0, 1
LOSS_FOCAL_NORM = 4
LOSS_DEFER_MINING = 64
LOSS_WS_ZEROED = 128
LOSS_UNFUSED_FINISH = 512
CRIT_WS_ZEROED, CRIT_TWO_LAUNCH = 128, 1024
POOL = dict(nonpos=0, neg=8, global_neg=16, nonpos_not_easy=32)
OV = dict(iou=0, giou=1, diou=2, ciou=3)
FOCAL = dict(softmax=0, sigmoid=1, bce=2)
BOX = dict(offset=0, center=1, corner=2)
ACT = dict(softmax=0, sigmoid=1)
NMS = dict(tv=0, ref=1, diou=2)
DETECT_COUNTERS_ZEROED, DETECT_INPUT_BF16, DETECT_FUSED = 1, 2, 8
DETECT_CORRUPT = -2
VARIANT_ONE_LAUNCH_CRITERION = 1


class SbodError(RuntimeError):
    pass


_lib = None
_fast = {}     # name -> _sbodcall wrapper (same C entry point, no ctypes argument conversion)
host_ext = None  # the _sbodhost extension (csrc/hostpack.cpp), when built
MISSING = []   # declared in include/sbod.h but not exported (tests assert this is empty)


def lib():
    """The loaded library (raises SbodError when it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SbodError('libsbod_hip.so not found at %s — build it with '
                            '`python -m shape_based_object_detection_amd.build`' % LIB_PATH)
        check_stamp()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                MISSING.append(name)
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
        _load_fast()
    return _lib


def check_stamp():
    """Refuse a library that was not built from the sources in this tree: build.py records the
    sha256 of the sources, flags and arch in lib/build_stamp.json, and it must match what the
    tree holds now.  (An explicit SBOD_LIB — a diagnostic or A/B variant — is not checked.)"""
    if 'SBOD_LIB' in os.environ:
        return
    from . import build as B
    have, want = B.read_stamp(), B.source_digest()
    if have != want:
        raise SbodError('libsbod_hip.so in %s was built from other sources (stamp %s, tree %s): '
                        'rebuild with `python -m shape_based_object_detection_amd.build`'
                        % (os.path.dirname(LIB_PATH), (have or 'missing')[:12], want[:12]))


def _load_fast():
    """The _sbodcall extension built next to the library (build.py), if present: a CPython
    METH_FASTCALL wrapper per entry point, calling the very same C functions.  Without it the
    ctypes binding is used (same kernels, more host time per call)."""
    # the extension links libsbod_hip.so by name: a variant library (SBOD_LIB=..._phase.so etc.)
    # keeps the ctypes path so every call reaches the library that was asked for
    if (not os.path.exists(FAST_PATH) or os.environ.get('SBOD_NO_FASTCALL')
            or os.path.basename(LIB_PATH) != 'libsbod_hip.so'):
        return
    import importlib.util
    spec = importlib.util.spec_from_file_location('_sbodcall', FAST_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for name in SIGNATURES:
        f = getattr(mod, name, None)
        if f is not None:
            _fast[name] = f
    global host_ext
    if os.path.exists(HOST_PATH):
        spec = importlib.util.spec_from_file_location('_sbodhost', HOST_PATH)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        host_ext = mod


def fastcall_names():
    lib()
    return sorted(_fast)


_recorder = []   # recording stack: (list to append (name, args) to) — see record_calls()


def record_calls(into):
    """Context manager: every sbod_* call made inside also appends (name, args) to ``into`` (and
    still runs).  A caller can then replay the same launches with ``replay_calls`` — e.g. a
    native-submit step: the calls' pointers (outputs, workspaces, streams) are the recording
    call's, so the caller keeps those buffers alive and unchanged, as a captured graph would."""
    import contextlib

    @contextlib.contextmanager
    def cm():
        _recorder.append(into)
        try:
            yield into
        finally:
            _recorder.pop()
    return cm()


def replay_calls(calls):
    """Issue recorded (name, args) calls again, in order, through the fast wrappers."""
    for name, args in calls:
        f = _fast.get(name)
        st = f(*args) if f is not None else getattr(lib(), name)(*args)
        if st != 0:
            msg = lib().sbod_last_error().decode(errors='replace')
            raise SbodError('%s failed (%d): %s' % (name, st, msg))


def call(name, *args):
    """Invoke an sbod_* entry point; raise SbodError with sbod_last_error() on failure."""
    if _recorder:
        _recorder[-1].append((name, args))
    f = _fast.get(name)
    st = f(*args) if f is not None else getattr(lib(), name)(*args)
    if st != 0:
        msg = lib().sbod_last_error().decode(errors='replace')
        raise SbodError('%s failed (%d): %s' % (name, st, msg))
    return st


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


_raw_stream = torch._C._cuda_getCurrentRawStream


def stream_of(t):
    """hipStream_t (as int) of torch's current stream on t's device (no Stream object built)."""
    return _raw_stream(t.get_device())


def require_device(*tensors, what='sbod'):
    """The HIP path only: CPU tensors are rejected (no silent CPU fallback)."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise SbodError('%s: expected ROCm device tensors, got a %s tensor. The sbod hot path '
                            'has no CPU implementation; move inputs to the GPU.' % (what, t.device))


def timing_enable(kernel_filter):
    """Bracket launches of ``kernel_filter`` (a kernel name, '*' = all instrumented kernels,
    None = off) with HIP events on their launch stream; clears earlier records."""
    call('sbod_timing_enable', None if kernel_filter is None else kernel_filter.encode())


def timing_query(kernel):
    """(launches, total_ms) recorded for ``kernel`` since timing_enable (waits for the events)."""
    n, ms = ctypes.c_int(0), ctypes.c_double(0.0)
    call('sbod_timing_query', kernel.encode(), ctypes.byref(n), ctypes.byref(ms))
    return n.value, ms.value
