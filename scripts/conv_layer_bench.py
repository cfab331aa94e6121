#!/usr/bin/env python3
"""Time MIOpen's conv forward and input gradient (torch.nn.functional, NCDHW f32) on the U-Net's C3
layer shapes (HIP events, median of 10).  Run under rocprofv3 --kernel-trace --stats to see what each
call is made of (CK kernels, layout transposes, im2col / col2im GEMMs).  Diagnostic, not the headline."""
import os
import sys

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True

LAYERS = [  # name, (N, Cin, D, H, W), Cout, stride, transposed
    ("down0.u0 4->16 s2", (2, 4, 240, 240, 160), 16, 2, False),
    ("down0.u1 16->16 s1", (2, 16, 120, 120, 80), 16, 1, False),
    ("down1.u0 16->32 s2", (2, 16, 120, 120, 80), 32, 2, False),
    ("down1.u1 32->32 s1", (2, 32, 60, 60, 40), 32, 1, False),
    ("down2.u0 32->64 s2", (2, 32, 60, 60, 40), 64, 2, False),
    ("down2.u1 64->64 s1", (2, 64, 30, 30, 20), 64, 1, False),
    ("up1.ct 64->16 s2T", (2, 64, 60, 60, 40), 16, 2, True),
    ("up1.ru 16->16 s1", (2, 16, 120, 120, 80), 16, 1, False),
    ("up0.ct 32->3 s2T", (2, 32, 120, 120, 80), 3, 2, True),
    ("up0.ru 3->3 s1", (2, 3, 240, 240, 160), 3, 1, False),
]


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
    return ts[len(ts) // 2]


def main():
    torch.manual_seed(0)
    only = sys.argv[1:]
    for name, xs, co, s, tr in LAYERS:
        if only and not any(o in name for o in only):
            continue
        cl = os.environ.get("CL") == "1"  # channels_last_3d activations and weights (NDHWC)
        mf = torch.channels_last_3d if cl else torch.contiguous_format
        x = torch.randn(xs, device="cuda").to(memory_format=mf).requires_grad_(True)
        if tr:
            w = (torch.randn((xs[1], co, 3, 3, 3), device="cuda") * 0.05).to(memory_format=mf)
            fwd = lambda: F.conv_transpose3d(x, w, stride=s, padding=1, output_padding=s - 1)
        else:
            w = (torch.randn((co, xs[1], 3, 3, 3), device="cuda") * 0.05).to(memory_format=mf)
            fwd = lambda: F.conv3d(x, w, stride=s, padding=1)
        y = fwd()
        g = torch.randn_like(y).to(memory_format=mf)
        tf = timeit(fwd)
        tb = timeit(lambda: torch.autograd.grad(y, x, g, retain_graph=True))
        flop = 2.0 * xs[0] * co * xs[1] * 27 * (y[0, 0].numel() if not tr else x[0, 0].numel())
        print(f"{name:22s} fwd {tf * 1e3:8.1f} us ({flop / tf / 1e9:6.1f} TF/s)  dgrad {tb * 1e3:8.1f} us "
              f"({flop / tb / 1e9:6.1f} TF/s)", flush=True)
        if os.environ.get("PROFILE"):
            from torch.profiler import ProfilerActivity, profile
            for tag, fn in (("fwd", fwd), ("dgrad", lambda: torch.autograd.grad(y, x, g, retain_graph=True))):
                torch.cuda.synchronize()
                with profile(activities=[ProfilerActivity.CUDA]) as prof:
                    fn()
                    torch.cuda.synchronize()
                evs = [e for e in prof.key_averages() if e.device_time_total > 0]
                for e in sorted(evs, key=lambda e: -e.device_time_total)[:8]:
                    print(f"    {tag:5s} {e.device_time_total:9.1f} us  x{e.count:<3d} {e.key[:100]}", flush=True)


if __name__ == "__main__":
    main()
