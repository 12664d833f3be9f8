"""Probe: can a captured hipGraph carry timing events around a kernel node on this runtime?
Tries torch.cuda.Event(external=True) records inside torch.cuda.graph capture and reports the
elapsed time after replays (diagnostic only)."""
import torch

dev = torch.device('cuda', 0)
x = torch.randn(1 << 24, device=dev)
y = torch.empty_like(x)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        torch.mul(x, 2.0, out=y)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
for kw in ({'enable_timing': True, 'external': True},):
    try:
        e0, e1 = torch.cuda.Event(**kw), torch.cuda.Event(**kw)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            torch.mul(x, 2.0, out=y)
            e0.record()
            torch.mul(x, 3.0, out=y)
            e1.record()
            torch.mul(x, 4.0, out=y)
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            print('external events', kw, 'elapsed ms', e0.elapsed_time(e1), flush=True)
    except Exception as ex:  # noqa: BLE001
        print('FAILED', kw, repr(ex)[:300], flush=True)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
torch.mul(x, 3.0, out=y)
b.record()
torch.cuda.synchronize()
print('eager mul ms', a.elapsed_time(b))
