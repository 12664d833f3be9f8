"""Probe: what a failed hipGraph capture leaves behind on this runtime, and the recovery the
bench's eager fallback uses (default stream + fresh side streams).  GPU box only:
    python scripts/probe_capture_abort.py"""
import sys, os, torch
sys.path.insert(0, os.getcwd())
from shape_based_object_detection_amd import _lib as L
import ctypes
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
L.lib()
hip = ctypes.CDLL('libamdhip64.so')
def status(s):
    st = ctypes.c_int(-1)
    r = hip.hipStreamIsCapturing(ctypes.c_void_p(s), ctypes.byref(st))
    return r, st.value
cs = torch.cuda.Stream(dev)
x = torch.ones(1024, device=dev)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g, stream=cs):
        y = x * 2
        torch.cuda.synchronize()   # prohibited under capture
except Exception as ex:
    print('capture failed:', repr(ex)[:200])
print('after: cs', status(cs.cuda_stream), 'null', status(0), 'cur', status(torch.cuda.current_stream().cuda_stream),
      'is_capturing', torch.cuda.is_current_stream_capturing())
try:
    L.call('sbod_stream_abort_capture', cs.cuda_stream)
    print('abort: ended')
except L.SbodError as ex:
    print('abort:', ex)
print('after abort: cs', status(cs.cuda_stream), 'null', status(0))
try:
    z = x + 1
    torch.cuda.synchronize()
    print('eager ok', float(z[0]))
except Exception as ex:
    print('eager failed:', repr(ex)[:300])
# recovery: leave the poisoned stream, use the default stream and a fresh side stream
torch.cuda.set_stream(torch.cuda.default_stream(dev))
try:
    z = x + 1
    big = torch.empty(64 << 20, dtype=torch.uint8, device=dev)   # a fresh allocation (hipMalloc)
    torch.cuda.synchronize()
    print('default stream ok', float(z[0]))
    s2 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s2):
        w = x * 3
    torch.cuda.synchronize()
    print('fresh stream ok', float(w[0]), 'status cs', status(cs.cuda_stream), 's2', status(s2.cuda_stream))
except Exception as ex:
    print('recovery failed:', repr(ex)[:300])
# the same failure under a thread-local capture: other threads' calls stay allowed
import threading
cs3 = torch.cuda.Stream(dev)
g3 = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g3, stream=cs3, capture_error_mode='thread_local'):
        y = x * 2
        torch.cuda.synchronize()
except Exception as ex:
    print('thread_local capture failed:', repr(ex)[:120])
torch.cuda.set_stream(torch.cuda.default_stream(dev))
res = {}
def other():
    try:
        s4 = torch.cuda.Stream(dev)
        with torch.cuda.stream(s4):
            q = x * 5
        s4.synchronize()
        res['other'] = float(q[0])
    except Exception as ex:
        res['other'] = repr(ex)[:200]
t = threading.Thread(target=other); t.start(); t.join()
print('thread_local other thread:', res)
try:
    s5 = torch.cuda.Stream(dev)
    with torch.cuda.stream(s5):
        q = x * 7
    torch.cuda.synchronize()
    print('thread_local main thread fresh stream + sync ok', float(q[0]))
except Exception as ex:
    print('thread_local main thread failed:', repr(ex)[:200])
