#!/usr/bin/env python3
"""Achievable HBM rates on this box for the shapes of pass C' (a write-dominated stream): torch fill_
(write only), copy_ (read + write) and sum (read only) over C3's filter output, 2x4x240x240x155
float32 (285.7 MB), HIP events, median of 20.  Puts C''s 0.53 of the 8 TB/s peak in context."""
import torch


def timeit(fn, n=20):
    ts = []
    for _ in range(n + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[3:])
    return ts[len(ts) // 2]


def main():
    n = 2 * 4 * 240 * 240 * 155
    for mb in (n, 2 * n):
        y = torch.empty(mb, device="cuda")
        x = torch.randn(mb, device="cuda")
        nb = mb * 4
        t = timeit(lambda: y.fill_(1.0))
        print(f"fill_ {nb / 1e6:7.1f} MB: {t * 1e3:6.1f} us  {nb / t / 1e9:6.2f} TB/s (write)", flush=True)
        t = timeit(lambda: y.copy_(x))
        print(f"copy_ {nb / 1e6:7.1f} MB: {t * 1e3:6.1f} us  {2 * nb / t / 1e9:6.2f} TB/s (read + write)", flush=True)
        t = timeit(lambda: x.sum())
        print(f"sum   {nb / 1e6:7.1f} MB: {t * 1e3:6.1f} us  {nb / t / 1e9:6.2f} TB/s (read)", flush=True)
        del x, y


if __name__ == "__main__":
    main()
