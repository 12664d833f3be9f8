#!/usr/bin/env python3
"""Probe (diagnostic): the DCN weight gradient at C4 64x64 with and without the offset / mask
gradients (k_dcn_bwd_weight3<true> reads the 604 MB dcols rows, <false> does not), eager, under
`rocprofv3 --kernel-trace` for the per-kernel times.  GPU box only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(3)
    B, C, O, H, ks = 16, 256, 256, 64, 3
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    off = torch.randn(B, 2 * ks * ks, H, H, device=dev, generator=g)
    ml = torch.randn(B, ks * ks, H, H, device=dev, generator=g)
    w = torch.randn(O, C, ks, ks, device=dev, generator=g) / 50
    gout = torch.randn(B, O, H, H, device=dev, generator=g)
    for want in ('weight', 'all'):
        ins = [t.clone().requires_grad_(want == 'all' or i == 3) for i, t in enumerate((x, off, ml, w))]
        for _ in range(6):
            for t in ins:
                t.grad = None
            core.deform_conv2d(*ins, ks, 1, 1).backward(gout)
        torch.cuda.synchronize()
        print(want, 'done', flush=True)


if __name__ == '__main__':
    main()
