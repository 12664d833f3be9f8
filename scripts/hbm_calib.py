"""Calibration: what a plain streaming kernel (torch copy / reduction) reaches at the detect
prepare's sizes (B=32 SSD512: scores 27.5 MB) on this GPU, back-to-back, HIP-event timed."""
import json
import torch
dev = torch.device('cuda')
x = torch.randn(32, 10248, 21, device=dev)
y = torch.empty_like(x)
big = torch.randn(256 << 20, device=dev)   # 1 GiB
bigy = torch.empty_like(big)
res = {}
def t(name, fn, nbytes, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    res[name] = {'us': round(us, 2), 'GBps': round(nbytes / us / 1e3, 1)}
t('copy_27.5MB', lambda: y.copy_(x), 2 * x.numel() * 4)
t('sum_27.5MB', lambda: x.sum(), x.numel() * 4)
t('copy_1GiB', lambda: bigy.copy_(big), 2 * big.numel() * 4, iters=20)
t('sum_1GiB', lambda: big.sum(), big.numel() * 4, iters=20)
print(json.dumps(res))
