#!/usr/bin/env python3
"""HIP-event timings of the implicit-GEMM convolutions (csrc/conv_gemm.hip) at the U-Net's C3 layer
shapes, MIOpen's forward / input gradient for the same layer beside them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from texbias import conv as C  # noqa: E402

torch.backends.cudnn.benchmark = True


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


# (name, mode, cin, cout, input spatial, stride, ksize); ConvT rows: cin -> cout of the transposed conv
LAYERS = [("down1 16->32 s2", "conv", 16, 32, (120, 120, 80), 2, 3), ("down2 32->64 s2", "conv", 32, 64, (60, 60, 40), 2, 3),
          ("down3 64->128 s2", "conv", 64, 128, (30, 30, 20), 2, 3), ("d3 128->128", "conv", 128, 128, (15, 15, 10), 1, 3),
          ("bot 128->256", "conv", 128, 256, (15, 15, 10), 1, 3), ("bot 256->256", "conv", 256, 256, (15, 15, 10), 1, 3),
          ("bot res 1x1", "conv", 128, 256, (15, 15, 10), 1, 1), ("up3 T 384->64", "convT", 384, 64, (15, 15, 10), 2, 3),
          ("up2 T 128->32", "convT", 128, 32, (30, 30, 20), 2, 3),
          ("down2 stk 32->128", "conv", 32, 128, (60, 60, 40), 2, 3), ("down3 stk 64->256", "conv", 64, 256, (30, 30, 20), 2, 3),
          ("down1 stk 16->64", "conv", 16, 64, (120, 120, 80), 2, 3)]
N = 2
for name, mode, ci, co, sp, s, k in LAYERS:
    x = torch.randn((N, ci) + sp, device="cuda")
    if mode == "conv":
        w = torch.randn((co, ci, k, k, k), device="cuda") * 0.05
        y = F.conv3d(x, w, None, s, (k - 1) // 2)
        t_m = timeit(lambda: F.conv3d(x, w, None, s, (k - 1) // 2))
        t_o = timeit(lambda: C.conv_gemm(x, w, None, "conv", s, k))
        P = y[0, 0].numel() * N
        fl = 2.0 * co * ci * k ** 3 * P
        gy = torch.randn_like(y)
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [s] * 3, [(k - 1) // 2] * 3, [1] * 3,
                                                                   False, [0] * 3, 1, [True, False, False]))
        dmode = "dgrad" if s == 1 else "convT"
        t_od = timeit(lambda: C.conv_gemm(gy, w, None, dmode, s, k))
        cfg = C.conv_gemm_config(x.shape, co, "conv", s, k)
        cfgd = C.conv_gemm_config(gy.shape, ci, dmode, s, k)
        t_mw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [s] * 3, [(k - 1) // 2] * 3, [1] * 3,
                                                                   False, [0] * 3, 1, [False, True, False]))
        t_ow = timeit(lambda: C.wgrad(gy, x, w.shape, s, 1)) if k == 3 else float("nan")
    else:
        w = torch.randn((ci, co, 3, 3, 3), device="cuda") * 0.05
        y = F.conv_transpose3d(x, w, None, 2, 1, 1)
        t_m = timeit(lambda: F.conv_transpose3d(x, w, None, 2, 1, 1))
        t_o = timeit(lambda: C.conv_gemm(x, w, None, "convT", 2, 3))
        fl = 2.0 * co * ci * 27 * x[0, 0].numel() * N
        gy = torch.randn_like(y)
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [2] * 3, [1] * 3, [1] * 3, True,
                                                                   [1] * 3, 1, [True, False, False]))
        t_od = timeit(lambda: C.conv_gemm(gy, w, None, "conv", 2, 3))  # dX of ConvT(s2) = Conv3d(s2) with W
        cfg = C.conv_gemm_config(x.shape, co, "convT", 2, 3)
        cfgd = C.conv_gemm_config(gy.shape, ci, "conv", 2, 3)
        t_mw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [2] * 3, [1] * 3, [1] * 3, True,
                                                                   [1] * 3, 1, [False, True, False]))
        t_ow = timeit(lambda: C.wgrad(x, gy, w.shape, 2, 1))
    tf = lambda t: fl / t / 1e6  # noqa: E731
    print(f"{name:17s} {fl / 1e9:6.2f} GF | fwd MIOpen {t_m:7.1f} ({tf(t_m):5.1f} TF/s)  gemm {t_o:7.1f} ({tf(t_o):5.1f}) "
          f"[{cfg['BM']}x{cfg['BP']} s{cfg['nsplit']} b{cfg['blocks']}] | dX MIOpen {t_md:7.1f} ({tf(t_md):5.1f})  "
          f"gemm {t_od:7.1f} ({tf(t_od):5.1f}) [{cfgd['BM']}x{cfgd['BP']} s{cfgd['nsplit']} b{cfgd['blocks']}] | "
          f"dW MIOpen {t_mw:7.1f} texbias {t_ow:7.1f}", flush=True)
