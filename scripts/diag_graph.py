"""Diagnostic: the bench step captured into a hipGraph, replayed with progress output per
replay, in stages (mode argument):
  single       one-stream capture of criterion fwd + detect + backward, no timing
  single_span  the same with the dominant kernel's span record read back every replay
Prints one line per replay (flushed) so a fault names the replay it happened in."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402

mode = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else 'k_det_prepare'
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
L.lib()
st = bench.Step(dev, 32, 0, 1, graph=True)
side = st.cap_stream
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    for _ in range(3):
        st.eager()
torch.cuda.current_stream(dev).wait_stream(side)
torch.cuda.synchronize()
for i in range(20):
    st.eager()
torch.cuda.synchronize()
print('eager ok', flush=True)
if mode == 'single_span':
    L.timing_enable('*')
    st.eager()
    torch.cuda.synchronize()
    L.timing_enable(kernel)
st.capture()
L.timing_enable(None)
print('captured', flush=True)
for i in range(12):
    loss, res = st()
    msg = 'replay %d loss %.6f n_det %d' % (i, loss.item(), sum(int(x.shape[0]) for x in res[0]))
    if mode == 'single_span':
        msg += ' span %s' % (L.timing_query(kernel),)
    print(msg, flush=True)
print('done', mode, flush=True)
