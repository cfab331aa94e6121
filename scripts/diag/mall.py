#!/usr/bin/env python3
"""Does a streaming read pay for the previous kernel's dirty lines?  Times a 285 MB read (x.sum)
after (a) another read of x and (b) a 294 MB write of y (fill_), HIP events around the read only."""
import torch

x = torch.randn((2, 4, 240, 240, 155), device="cuda")
y = torch.empty((2, 4, 240, 240, 160), device="cuda")
z = torch.empty((64 << 20,), device="cuda")  # 256 MiB


def t(fn, pre, n=20):
    ts = []
    for _ in range(n):
        pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


rd = lambda: x.sum()
for name, pre in (("after a read of x", lambda: x.sum()), ("after a 294 MB write (y.fill_)", lambda: y.fill_(0.5)),
                  ("after 256 MiB written elsewhere", lambda: z.fill_(0.5)),
                  ("after y.fill_ then a 256 MiB read", lambda: (y.fill_(0.5), z.sum()))):
    us = t(rd, pre)
    print(f"x.sum() {name:38s} {us:7.1f} us  {x.numel() * 4 / us / 1e3:6.2f} TB/s", flush=True)
us = t(lambda: y.fill_(0.25), lambda: x.sum())
print(f"y.fill_ after a read                      {us:7.1f} us  {y.numel() * 4 / us / 1e3:6.2f} TB/s")
us = t(lambda: y.fill_(0.25), lambda: y.fill_(0.5))
print(f"y.fill_ after y.fill_                     {us:7.1f} us  {y.numel() * 4 / us / 1e3:6.2f} TB/s")
