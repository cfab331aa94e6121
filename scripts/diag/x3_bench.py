#!/usr/bin/env python3
"""Split-precision (bf16x3) vs f32-MFMA 16-channel conv at the C3 shape: time and error vs float64.
Run twice, TEXBIAS_CONV_X3=0 and =1 (diagnostic)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "medical-vision-textural-bias_amd"))
from texbias import conv  # noqa: E402

torch.manual_seed(0)
N, D, H, W = 2, 120, 120, 80
x = torch.randn((N, 16, D, H, W), device="cuda")
w = torch.randn((16, 16, 3, 3, 3), device="cuda") * 0.1
b = torch.randn(16, device="cuda")
ts = []
for _ in range(13):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    y = conv.conv_fwd16(x, w, b)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
ts = sorted(ts[3:])
xs = x[:1, :, :24].double()
y64 = F.conv3d(xs, w.double(), b.double(), padding=1)
ys = conv.conv_fwd16(x[:1, :, :24].contiguous(), w, b).double()
y32 = F.conv3d(x[:1, :, :24], w, b, padding=1).double()
scale = y64.abs().max().item()
print(f"x3={os.environ.get('TEXBIAS_CONV_X3', '1')} median {ts[len(ts) // 2] * 1e3:.1f} us  "
      f"err ours {(ys - y64).abs().max().item() / scale:.3e}  aten {(y32 - y64).abs().max().item() / scale:.3e}")
