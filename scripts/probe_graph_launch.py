"""Probe: per-node cost of hipGraph replay vs eager launches on this runtime (diagnostic).

A chain of N tiny kernels on one stream (and a fork/join variant across two streams) is timed
eagerly and as a captured graph: GPU time per chain (events) and host wall time per chain.
Run under different runtime environment settings by the caller."""
import json
import os
import sys
import time

import torch

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
dev = torch.device('cuda', 0)
x = torch.zeros(1 << 16, device=dev)
y = torch.zeros(1 << 16, device=dev)
s2 = torch.cuda.Stream()


def chain():
    for _ in range(N):
        x.add_(1.0)


def fork():
    cur = torch.cuda.current_stream()
    s2.wait_stream(cur)
    with torch.cuda.stream(s2):
        for _ in range(N // 2):
            y.add_(1.0)
    for _ in range(N // 2):
        x.add_(1.0)
    cur.wait_stream(s2)


def measure(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6, e0.elapsed_time(e1) / iters * 1e3


out = {'env': {k: os.environ.get(k) for k in ('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'HIP_FORCE_DEV_KERNARG',
                                               'AMD_SERIALIZE_KERNEL')}, 'N': N}
for name, fn in (('chain', chain), ('fork', fork)):
    out[name + '_eager_us'] = measure(fn)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    out[name + '_graph_us'] = measure(g.replay)
print(json.dumps(out), flush=True)
