#!/usr/bin/env python3
"""Read+write streaming reference for the one-pass filter kernels (measurement tool): device copies of
the C3 volume batch [2, 4, 240, 240, 155] fp32 -- contiguous, and into the U-Net's D-padded [.., 160]
layout (the wrap / closed-form kernels' exact byte pattern) -- timed with HIP events, best / mean of 20."""
import json
import torch

dev = torch.device("cuda", 0)
x = torch.randn((2, 4, 240, 240, 155), device=dev)
y = torch.empty_like(x)
yp = torch.zeros((2, 4, 240, 240, 160), device=dev)
yp_v = yp[..., :155]


def bench(fn, nbytes, name):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    best, mean = min(ts), sum(ts) / len(ts)
    print(json.dumps({"copy": name, "bytes": nbytes, "best_us": round(best, 1), "mean_us": round(mean, 1),
                      "best_TBs": round(nbytes / best / 1e6, 3)}))


n = x.numel() * 4
bench(lambda: y.copy_(x), 2 * n, "contiguous 285.7 MB -> 285.7 MB")
bench(lambda: yp_v.copy_(x), n + yp.numel() * 4 * 155 // 160, "into the D-padded rows (strided)")
bench(lambda: yp.copy_(yp), 2 * yp.numel() * 4, "padded -> padded in place")
