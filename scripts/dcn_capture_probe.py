#!/usr/bin/env python3
"""Which DeformConv2d calls can torch.cuda.graph capture (diagnostic): fwd + autograd bwd of one
shape captured on a side stream after `warm` eager warm-ups there (and, with `pre`, an eager call
on the default stream first).  Prints 'ok' or dies in capture_end.
    python scripts/dcn_capture_probe.py B C O H warm pre"""
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
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(warm):
        step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print('capturing', sys.argv[1:7], flush=True)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph, stream=side):
    cap = step()
graph.replay()
torch.cuda.synchronize()
print('ok', sys.argv[1:7], flush=True)
