#!/usr/bin/env python3
"""Event-timed k_dcn_dx_gather (and k_dcn_bwd_data / k_dcn_bwd_weight) at C4's 64² and 8² maps,
eager DCN fwd+bwd; select the library with SBOD_LIB to A/B builds on one box.
    SBOD_LIB=... python scripts/gx_ab.py LABEL"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import _lib as L  # noqa: E402
from shape_based_object_detection_amd import core  # noqa: E402

dev = torch.device('cuda', 0)
res = {'label': sys.argv[1] if len(sys.argv) > 1 else 'default'}
for H in (64, 8):
    g = torch.Generator(device=dev).manual_seed(H)
    B, C, O = 16, 256, 256
    x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(True)
    off = torch.randn(B, 18, H, H, device=dev, generator=g).requires_grad_(True)
    ml = torch.randn(B, 9, H, H, device=dev, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, 3, 3, device=dev, generator=g) / 48).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=dev, generator=g)
    ins = (x, off, ml, w)
    for _ in range(3):
        torch.autograd.grad(core.deform_conv2d(x, off, ml, w), ins, gout)
    torch.cuda.synchronize()
    out = {}
    for k in ('k_dcn_dx_gather', 'k_dcn_bwd_data', 'k_dcn_bwd_weight'):
        L.timing_enable(k)
        for _ in range(10):
            torch.autograd.grad(core.deform_conv2d(x, off, ml, w), ins, gout)
        torch.cuda.synchronize()
        n, ms = L.timing_query(k)
        L.timing_enable(None)
        out[k] = round(ms * 1e3 / n, 2) if n else None
    res[str(H)] = out
print(json.dumps(res), flush=True)
