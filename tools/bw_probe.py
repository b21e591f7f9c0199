"""Practical HBM ceilings on this box for write-dominated and copy streams (torch fill_ / copy_),
to read the streaming kernels' fractions against: python tools/bw_probe.py"""
import torch

def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    return sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(n))[n // 2]

n = 2_490_000_000 // 8
a = torch.empty(n, dtype=torch.float64, device="cuda")
b = torch.empty(n, dtype=torch.float64, device="cuda")
ms = timed(lambda: a.fill_(1.0))
print(f"fill  {n * 8 / 1e9:.2f} GB written: {ms:.3f} ms, {n * 8 / ms / 1e6:.0f} GB/s")
ms = timed(lambda: b.copy_(a))
print(f"copy  {n * 8 / 1e9:.2f} GB read + written: {ms:.3f} ms, {2 * n * 8 / ms / 1e6:.0f} GB/s")
