#!/usr/bin/env python3
"""DeformConv2d (config C4) forward+backward per map size, as bench.py's ``dcn`` key reports it:
replayed from one hipGraph (the kernels' own time) and launched eagerly through autograd.

    python scripts/dcn_maps.py [--maps 64,32,16,8] [--iters 20] > gpurun_out/dcn_maps.jsonl

Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split (grid sizes tell the maps
apart)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--maps', default='64,32,16,8')
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    for H in (int(h) for h in a.maps.split(',')):
        r = BM.dcn_figure(dev, H=H, iters=a.iters)
        r['lib'] = os.environ.get('SBOD_LIB', 'libsbod_hip.so')
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
