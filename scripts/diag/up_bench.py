#!/usr/bin/env python3
"""HIP-event timings of the direct full-resolution stride-2 kernels (csrc/conv_up.hip) at the bench shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402

from texbias import conv as C  # noqa: E402


def timeit(fn, n=10):
    ts = []
    for _ in range(n + 3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[3:])
    return ts[len(ts) // 2] * 1e3


x = torch.randn((2, 4, 240, 240, 160), device="cuda")
w = torch.randn((16, 4, 3, 3, 3), device="cuda")
K = C.s2_pairs(w)
t = timeit(lambda: C.conv_s2_fewin(x, K, None, 16))
print(f"conv_s2_fewin 4->16 (entry conv fwd)      {t:8.1f} us  {2 * 16 * 4 * 27 * 2 * 120 * 120 * 80 / t / 1e6:6.1f} TF/s")
xt = torch.randn((2, 32, 120, 120, 80), device="cuda")
wt = torch.randn((32, 3, 3, 3, 3), device="cuda")
t = timeit(lambda: C.convT_fewout(xt, wt, None))
print(f"convT_fewout 32->3 (exit convT fwd)       {t:8.1f} us  {2 * 32 * 3 * 27 * 2 * 120 * 120 * 80 / t / 1e6:6.1f} TF/s")
gy = torch.randn((2, 3, 240, 240, 160), device="cuda")
Kt = C.s2_pairs(wt)
t = timeit(lambda: C.conv_s2_fewin(gy, Kt, None, 32))
print(f"conv_s2_fewin 3->32 (exit convT dgrad)    {t:8.1f} us  {2 * 32 * 3 * 27 * 2 * 120 * 120 * 80 / t / 1e6:6.1f} TF/s")
x16 = torch.randn((2, 16, 120, 120, 80), device="cuda")
w16 = torch.randn((16, 16, 3, 3, 3), device="cuda")
t = timeit(lambda: C.conv_fwd16(x16, w16, None))
print(f"conv_fwd16 16->16 (120x120x80)            {t:8.1f} us  {2 * 16 * 16 * 27 * 2 * 120 * 120 * 80 / t / 1e6:6.1f} TF/s")
t = timeit(lambda: torch.nn.functional.conv3d(x16, w16, None, padding=1))
print(f"  MIOpen conv3d 16->16                    {t:8.1f} us")
x64 = torch.randn((2, 64, 60, 60, 40), device="cuda")
w64 = torch.randn((64, 16, 3, 3, 3), device="cuda")
t = timeit(lambda: C.convT_mfma64(x64, w64, None))
print(f"convT_mfma64 64->16 (up1 convT fwd)       {t:8.1f} us  {2 * 64 * 16 * 27 * 2 * 60 * 60 * 40 / t / 1e6:6.1f} TF/s")
t = timeit(lambda: torch.nn.functional.conv_transpose3d(x64, w64, None, stride=2, padding=1, output_padding=1))
print(f"  MIOpen conv_transpose3d 64->16          {t:8.1f} us")
for ch, sh in ((32, (2, 32, 60, 60, 40)), (64, (2, 64, 30, 30, 20))):
    xc = torch.randn(sh, device="cuda")
    wc = torch.randn((ch, ch, 3, 3, 3), device="cuda")
    fl = 2 * ch * ch * 27 * 2 * sh[2] * sh[3] * sh[4]
    t = timeit(lambda: C.conv_mfma(xc, wc, None))
    print(f"conv_mfma {ch}->{ch} {sh[2:]}        {t:8.1f} us  {fl / t / 1e6:6.1f} TF/s")
    t = timeit(lambda: torch.nn.functional.conv3d(xc, wc, None, padding=1))
    print(f"  MIOpen conv3d {ch}->{ch}                    {t:8.1f} us")
gy32 = torch.randn((2, 32, 60, 60, 40), device="cuda")
w32 = torch.randn((32, 16, 3, 3, 3), device="cuda")
t = timeit(lambda: C.convT_mfma(gy32, w32, None))
print(f"convT_mfma 32->16 (down1 s2 dgrad)        {t:8.1f} us  {2 * 32 * 16 * 27 * 2 * 60 * 60 * 40 / t / 1e6:6.1f} TF/s")
t = timeit(lambda: torch.nn.functional.conv_transpose3d(gy32, w32, None, stride=2, padding=1, output_padding=1))
print(f"  MIOpen conv_transpose3d 32->16          {t:8.1f} us")
