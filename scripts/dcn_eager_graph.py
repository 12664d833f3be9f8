#!/usr/bin/env python3
"""DeformConv2d fwd+bwd at one map, eager or hipGraph-replayed only (diagnostic, for a kernel trace
of each mode):  python scripts/dcn_eager_graph.py --mode eager|graph [--H 64] [--iters 10]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--mode', choices=('eager', 'graph'), default='eager')
    ap.add_argument('--H', type=int, default=64)
    ap.add_argument('--iters', type=int, default=10)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    B, C, O, H = 16, 256, 256, a.H
    g = torch.Generator(device=dev).manual_seed(H)
    x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(True)
    off = torch.randn(B, 18, H, H, device=dev, generator=g).requires_grad_(True)
    ml = torch.randn(B, 9, H, H, device=dev, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, 3, 3, device=dev, generator=g) / 48).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=dev, generator=g)
    params = (x, off, ml, w)

    def step():
        return torch.autograd.grad(core.deform_conv2d(x, off, ml, w), params, gout)

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    fn = step
    if a.mode == 'graph':
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=side):
            step()
        fn = graph.replay
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(a.mode, H, round(e0.elapsed_time(e1) / a.iters, 4), 'ms')


if __name__ == '__main__':
    main()
