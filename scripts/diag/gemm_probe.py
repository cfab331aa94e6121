#!/usr/bin/env python3
"""f32 GEMM rates (torch.mm -> hipBLASLt / rocBLAS) at the U-Net deep layers' im2col shapes, beside
MIOpen's conv forward / backward for the same layers (HIP events, median of 10)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

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


# (name, Cin, Cout, input spatial, stride)
LAYERS = [("16->32 s2", 16, 32, (120, 120, 80), 2), ("32->64 s2", 32, 64, (60, 60, 40), 2),
          ("64->128 s2", 64, 128, (30, 30, 20), 2), ("128->128", 128, 128, (15, 15, 10), 1),
          ("128->256", 128, 256, (15, 15, 10), 1), ("256->256", 256, 256, (15, 15, 10), 1)]
N = 2
for name, ci, co, sp, s in LAYERS:
    x = torch.randn((N, ci) + sp, device="cuda", requires_grad=True)
    w = torch.randn((co, ci, 3, 3, 3), device="cuda", requires_grad=True) * 0.05
    y = F.conv3d(x, w, None, s, 1)
    P = y[0, 0].numel() * N
    K = ci * 27
    fl = 2.0 * co * K * P
    t_f = timeit(lambda: F.conv3d(x, w, None, s, 1))
    gy = torch.randn_like(y)
    t_dx = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [s] * 3, [1] * 3, [1] * 3, False,
                                                                [0] * 3, 1, [True, False, False]))
    t_dw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [s] * 3, [1] * 3, [1] * 3, False,
                                                                [0] * 3, 1, [False, True, False]))
    A = torch.randn(co, K, device="cuda")
    B = torch.randn(K, P, device="cuda")
    Bt = torch.randn(P, K, device="cuda")
    G = torch.randn(co, P, device="cuda")
    t_mm = timeit(lambda: torch.mm(A, B))          # forward: W [M, K] . col [K, P]
    t_mmt = timeit(lambda: torch.mm(A, Bt.t()))    # forward with col stored [P, K]
    t_dc = timeit(lambda: torch.mm(A.t(), G))      # dgrad cols: W^T [K, M] . G [M, P]
    t_wg = timeit(lambda: torch.mm(G, Bt))         # wgrad: G [M, P] . col^T [P, K]
    tf = lambda t: fl / t / 1e6  # noqa: E731
    print(f"{name:11s} M={co:4d} K={K:5d} P={P:6d} {fl / 1e9:6.2f} GF | MIOpen fwd {t_f:7.1f} ({tf(t_f):5.1f} TF/s) "
          f"dx {t_dx:7.1f} ({tf(t_dx):5.1f}) dw {t_dw:7.1f} ({tf(t_dw):5.1f}) | mm {t_mm:7.1f} ({tf(t_mm):5.1f}) "
          f"mm_t {t_mmt:7.1f} ({tf(t_mmt):5.1f}) dcol {t_dc:7.1f} ({tf(t_dc):5.1f}) wg {t_wg:7.1f} ({tf(t_wg):5.1f})",
          flush=True)
