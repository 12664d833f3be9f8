#!/usr/bin/env python3
"""Which DeformConv2d calls can torch.cuda.graph capture (diagnostic): fwd + autograd bwd of one
shape captured on a side stream after `warm` eager warm-ups there (and, with `pre`, an eager call
on the default stream first).  Prints 'ok' or dies in capture_end.
    python scripts/dcn_capture_probe.py B C O H warm pre [stateless]
stateless = 1: a call of the C-ABI's stateless backward (its own torch workspace, freed at once)
before the warm-ups, as tests/test_gpu_dcn.py's fork-join test did."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core  # noqa: E402

B, C, O, H, warm, pre = (int(a) for a in sys.argv[1:7])
dev = torch.device('cuda', 0)
g = torch.Generator(device=dev).manual_seed(H)
ks = 3
x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(True)
off = torch.randn(B, 2 * ks * ks, H, H, device=dev, generator=g).requires_grad_(True)
ml = torch.randn(B, ks * ks, H, H, device=dev, generator=g).requires_grad_(True)
w = (torch.randn(O, C, ks, ks, device=dev, generator=g) / 24).requires_grad_(True)
gout = torch.randn(B, O, H, H, device=dev, generator=g)
ins = (x, off, ml, w)


def step():
    out = core.deform_conv2d(x, off, ml, w, ks, 1, 1)
    return (out,) + tuple(torch.autograd.grad(out, ins, gout))


if pre:
    step()
if len(sys.argv) > 7 and int(sys.argv[7]):
    from shape_based_object_detection_amd import _lib as L
    dims = (B, C, H, H, O, ks, 1, 1)
    nb = L.lib().sbod_dcn_workspace_bytes(*dims)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    res = [torch.empty_like(t) for t in ins]
    L.call('sbod_dcn_bwd_f32', *[L.ptr(t) for t in ins], L.ptr(gout), *dims, *[L.ptr(t) for t in res],
           L.ptr(ws), nb, L.stream_of(gout))
    torch.cuda.synchronize()
    del ws, res
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(warm):
        step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print('capturing', sys.argv[1:], flush=True)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph, stream=side):
    cap = step()
graph.replay()
torch.cuda.synchronize()
print('ok', sys.argv[1:], flush=True)
