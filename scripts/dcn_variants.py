#!/usr/bin/env python3
"""DeformConv2d at C4's 64x64 map (B=16, 256 -> 256, 3x3, modulated) with a chosen subset of input
gradients, so a kernel trace of each run splits the backward's cost by what it computes:

  all     x, offset, mask and weight gradients (the bench's figure)
  weight  weight gradient only (k_dcn_bwd_weight without the offset / mask reduction, no dcols)
  x       x gradient only (k_dcn_bwd_data + the dx gather, no weight-gradient kernel)
  om      offset + mask gradients only (dcols, then k_dcn_bwd_weight's reduction without dW)

    rocprofv3 --kernel-trace -d gpurun_out/dv_all -o run --output-format csv -- \\
        python3 scripts/dcn_variants.py all
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else 'all'
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(H)
    B, C, O = 16, 256, 256
    want = {'all': (1, 1, 1, 1), 'weight': (0, 0, 0, 1), 'x': (1, 0, 0, 0), 'om': (0, 1, 1, 0)}[which]
    x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(bool(want[0]))
    off = torch.randn(B, 18, H, H, device=dev, generator=g).requires_grad_(bool(want[1]))
    ml = torch.randn(B, 9, H, H, device=dev, generator=g).requires_grad_(bool(want[2]))
    w = (torch.randn(O, C, 3, 3, device=dev, generator=g) / 48).requires_grad_(bool(want[3]))
    gout = torch.randn(B, O, H, H, device=dev, generator=g)
    params = [t for t in (x, off, ml, w) if t.requires_grad]
    for _ in range(12):
        torch.autograd.grad(core.deform_conv2d(x, off, ml, w), params, gout)
    torch.cuda.synchronize()
    print('done', which, H, flush=True)


if __name__ == '__main__':
    main()
