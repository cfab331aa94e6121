#!/usr/bin/env python3
"""Median time of the hand-written conv kernels at their C3 shapes (forward and input gradient), and the
max error of each against float64 on a slice.  Run per environment variant (diagnostic)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "medical-vision-textural-bias_amd"))
from texbias import conv  # noqa: E402


def timeit(f, n=13):
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[3:])
    return ts[len(ts) // 2] * 1e3


def err(ours, ref):
    return (ours.double() - ref).abs().max().item() / ref.abs().max().item()


torch.manual_seed(0)
tag = os.environ.get("TAG", "")
cases = [("fwd16", 16, (2, 120, 120, 80)), ("mfma32", 32, (2, 60, 60, 40)), ("mfma64", 64, (2, 30, 30, 20))]
for name, C, (N, D, H, W) in cases:
    x = torch.randn((N, C, D, H, W), device="cuda")
    w = torch.randn((C, C, 3, 3, 3), device="cuda") * (1.0 / (27 * C) ** 0.5)
    b = torch.randn(C, device="cuda")
    fw = (lambda: conv.conv_fwd16(x, w, b)) if C == 16 else (lambda: conv.conv_mfma(x, w, b))
    dg = (lambda: conv.conv_fwd16_dgrad(x, w)) if C == 16 else (lambda: conv.conv_mfma_dgrad(x, w))
    tf, td = timeit(fw), timeit(dg)
    xs = x[:1, :, :12].contiguous()
    y64 = F.conv3d(xs.double(), w.double(), b.double(), padding=1)
    ys = conv.conv_fwd16(xs, w, b) if C == 16 else conv.conv_mfma(xs, w, b)
    g64 = F.conv_transpose3d(xs.double(), w.double(), None, padding=1)
    gs = conv.conv_fwd16_dgrad(xs, w) if C == 16 else conv.conv_mfma_dgrad(xs, w)
    print(f"{tag} {name}: fwd {tf:.1f} us dgrad {td:.1f} us  err fwd {err(ys, y64):.2e} dgrad {err(gs, g64):.2e}",
          flush=True)
