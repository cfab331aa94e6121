#!/usr/bin/env python3
"""Time tb_conv3d_small_f32 (the top ResidualUnit's 3->3 conv, 2 x 3 x 240 x 240 x 160) with HIP events,
median of 10.  Diagnostic; TEXBIAS_SMALL_CONV_Z=0 selects the per-plane kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402

from texbias import conv as C  # noqa: E402


def main():
    torch.manual_seed(0)
    x = torch.randn((2, 3, 240, 240, 160), device="cuda")
    w = torch.randn((3, 3, 3, 3, 3), device="cuda")
    b = torch.randn(3, device="cuda")
    ts = []
    for _ in range(12):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        C.small_conv(x, w, b)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts[2:])[5]
    print(f"{os.environ.get('TAG', '')} small_conv 3->3 2x240x240x160: {ms * 1e3:.1f} us "
          f"({2 * 2 * 3 * 3 * 27 * 240 * 240 * 160 / ms / 1e9:.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
