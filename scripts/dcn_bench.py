"""DeformConv2d (a14) timing at BASELINE C4 sizes: B=16, 256 -> 256, 3x3, H=W in {64,32,16,8}.

Times forward and forward+backward through the HIP path with HIP events on the launch stream and
prints one JSON line per size: ms, TFLOP/s of the contraction (fwd 2*M*O*K, bwd 4*M*O*K) and the
fraction of the f32 MFMA peak (157.3 TFLOP/s, MI355X_MICROARCH.md)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shape_based_object_detection_amd import core  # noqa: E402

PEAK = 157.3


def run(H, iters, warm, B=16, C=256, O=256):
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(H)
    x = torch.randn(B, C, H, H, device=dev, generator=g).requires_grad_(True)
    off = torch.randn(B, 18, H, H, device=dev, generator=g).requires_grad_(True)
    ml = torch.randn(B, 9, H, H, device=dev, generator=g).requires_grad_(True)
    w = (torch.randn(O, C, 3, 3, device=dev, generator=g) / 48).requires_grad_(True)
    gout = torch.randn(B, O, H, H, device=dev, generator=g)
    M, K = B * H * H, C * 9
    res = {'H': H, 'B': B, 'C': C, 'O': O}
    for mode in ('fwd', 'fwd+bwd'):
        for _ in range(warm):
            y = core.deform_conv2d(x, off, ml, w)
            if mode != 'fwd':
                y.backward(gout)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            y = core.deform_conv2d(x, off, ml, w)
            if mode != 'fwd':
                y.backward(gout)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        flops = 2.0 * M * O * K * (1 if mode == 'fwd' else 3)
        tf = flops / ms / 1e9
        res[mode] = {'ms': round(ms, 4), 'tflops': round(tf, 2), 'mfma_frac': round(tf / PEAK, 4)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='64,32,16,8')
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    a = ap.parse_args()
    for H in [int(s) for s in a.sizes.split(',')]:
        print(json.dumps(run(H, a.iters, a.warmup)), flush=True)


if __name__ == '__main__':
    main()
