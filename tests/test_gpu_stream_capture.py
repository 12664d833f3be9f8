"""sbod_stream_abort_capture (include/sbod.h): a no-op on a stream that is not capturing, and it
ends an active capture so the stream can be used again (the bench's fallback after a failed
hipGraph capture, DESIGN.md "Data-parallel path, rehearsed on one GPU").  The capture is begun in
relaxed mode on a raw stream of its own, so nothing else in the test process is restricted."""
import ctypes

import pytest
import torch

from shape_based_object_detection_amd import _lib as L

pytestmark = pytest.mark.gpu

HIP_CAPTURE_MODE_RELAXED = 2


def _hip():
    torch.cuda.init()
    return ctypes.CDLL('libamdhip64.so')


def _status(hip, s):
    st = ctypes.c_int(-1)
    assert hip.hipStreamIsCapturing(s, ctypes.byref(st)) == 0
    return st.value


def test_abort_capture_is_noop_then_ends_an_active_capture():
    hip = _hip()
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    try:
        L.call('sbod_stream_abort_capture', s.value)          # not capturing: a no-op
        assert _status(hip, s) == 0
        assert hip.hipStreamBeginCapture(s, HIP_CAPTURE_MODE_RELAXED) == 0
        assert _status(hip, s) == 1                             # active
        L.call('sbod_stream_abort_capture', s.value)
        assert _status(hip, s) == 0                             # ended, graph discarded
        # the stream takes work again
        x = torch.ones(1024, device='cuda')
        ext = torch.cuda.ExternalStream(s.value)
        with torch.cuda.stream(ext):
            y = x * 3
        ext.synchronize()
        assert float(y.sum()) == 3072.0
    finally:
        torch.cuda.synchronize()
        hip.hipStreamDestroy(s)
