"""Achievable HBM write / copy bandwidth on this box for the pass-C' output size (reference numbers)."""
import torch
n = 8 * 240 * 240 * 160
y = torch.empty(n, device="cuda")
x = torch.randn(n, device="cuda")
for name, fn in (("fill", lambda: y.fill_(1.0)), ("copy", lambda: y.copy_(x))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    mult = 1 if name == "fill" else 2
    print(f"{name}: {ms*1e3:.1f} us for {n*4/1e6:.0f} MB -> {mult*n*4/ms/1e6:.0f} GB/s")
