#!/usr/bin/env python3
"""Event-timed criterion kernels (k_match_tile, k_match_final, k_multibox) over eager criterion
halves alone (as bench.py's roofline legs), for C2 (B=16 bf16) and the headline (B=32 f32).
Select the library with SBOD_LIB to A/B builds on one box.
    SBOD_LIB=... python scripts/mb_ab.py LABEL"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
res = {'label': sys.argv[1] if len(sys.argv) > 1 else os.environ.get('SBOD_LIB', 'default')}
for name, B, dt in (('c2_bf16_b16', 16, torch.bfloat16), ('c1_f32_b32', 32, torch.float32)):
    st = BM.Step(dev, B, 0, 1, graph=False, n_batches=12 if B == 16 else 6, dtype=dt, priority='detect')
    for _ in range(5):
        st.eager_half('criterion')
    torch.cuda.synchronize()
    out = {}
    for k in ('k_match_tile', 'k_match_final', 'k_multibox'):
        L.timing_enable(k)
        for _ in range(48):
            st.eager_half('criterion')
        torch.cuda.synchronize()
        n, ms = L.timing_query(k)
        L.timing_enable(None)
        out[k] = round(ms * 1e3 / n, 2) if n else None
    res[name] = out
    del st
    torch.cuda.synchronize()
print(json.dumps(res), flush=True)
