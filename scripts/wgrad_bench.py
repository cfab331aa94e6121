#!/usr/bin/env python3
"""Time tb_conv3d_wgrad_f32 and tb_channel_sum_f32 on the U-Net's C3 layer shapes (HIP events,
median of 10); prints one line per (layer, variant).  Diagnostic for tuning, not the headline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402

from texbias import conv as C  # noqa: E402

LAYERS = [  # name, G shape, X shape, stride (G = grad_out / low-res x, X = input / hi-res grad)
    ("L0.conv1 16->16 s1", (2, 16, 120, 120, 80), (2, 16, 120, 120, 80), 1),
    ("L0.conv0 4->16 s2", (2, 16, 120, 120, 80), (2, 4, 240, 240, 160), 2),
    ("L1.conv0 16->32 s2", (2, 32, 60, 60, 40), (2, 16, 120, 120, 80), 2),
    ("L1.conv1 32->32 s1", (2, 32, 60, 60, 40), (2, 32, 60, 60, 40), 1),
    ("L2.conv1 64->64 s1", (2, 64, 30, 30, 20), (2, 64, 30, 30, 20), 1),
    ("Up0.ru 3->3 s1", (2, 3, 240, 240, 160), (2, 3, 240, 240, 160), 1),
    ("Up0.convT 32->3 s2", (2, 32, 120, 120, 80), (2, 3, 240, 240, 160), 2),
]


def timeit(fn, n=10):
    ts = []
    for _ in range(n + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts = sorted(ts[2:])
    return ts[len(ts) // 2]


def main():
    torch.manual_seed(0)
    tag = os.environ.get("TAG", "")
    for name, gs, xs, s in LAYERS:
        G = torch.randn(gs, device="cuda")
        X = torch.randn(xs, device="cuda")
        w_shape = (gs[1], xs[1], 3, 3, 3)
        ms = timeit(lambda: C.wgrad(G, X, w_shape, s, 1))
        flop = 2.0 * gs[1] * xs[1] * 27 * gs[0] * gs[2] * gs[3] * gs[4]
        print(f"{tag} wgrad {name:22s} {ms * 1e3:9.1f} us  {flop / ms / 1e9:7.1f} TF/s", flush=True)
    g = torch.randn((2, 16, 120, 120, 80), device="cuda")
    ms = timeit(lambda: C.channel_sum(g))
    ms2 = timeit(lambda: g.sum((0, 2, 3, 4)))
    err = (C.channel_sum(g) - g.double().sum((0, 2, 3, 4)).float()).abs().max().item()
    print(f"{tag} channel_sum 2x16x120x120x80: {ms * 1e3:.1f} us ({g.numel() * 4 / ms / 1e6:.0f} GB/s) vs torch "
          f"{ms2 * 1e3:.1f} us; max abs err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
