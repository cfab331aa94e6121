#!/usr/bin/env python3
"""Per-pass timing of the filter chain under bench-like cache conditions (measurement tool).

bench.py runs the U-Net step between two chain calls, so every pass starts with caches full of
unrelated dirty lines; `bench.py --filter-only` runs the chains back to back instead, which moves
the pass times (k_band_inv 88 us in the bench, 110-125 us filter-only).  This runs the C3 (or C2)
chain with a cache flush between calls -- a read-modify-write sweep over a buffer larger than the
Infinity Cache -- and prints one line per pass (HIP events on the launch stream).

Usage: python scripts/pass_bench.py [--config c3|c2] [--iters N] [--flush-mb MB] [--tag TEXT]
(TEXBIAS_LIB selects a library variant.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c3", "c2"), default="c3")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--flush-mb", type=int, default=1024)
    ap.add_argument("--tag", default=os.environ.get("TEXBIAS_LIB", "default"))
    a = ap.parse_args()
    from texbias import runtime as rt
    from texbias.pipeline import FusedChain, reference_c3_chain
    from texbias.synth import brats_like

    dev = torch.device("cuda", 0)
    c2 = a.config == "c2"
    B, shape, pad = (16, (128, 128, 128), 0) if c2 else (2, (240, 240, 155), 5)
    pool = [brats_like(B, 4, shape, seed=i, device=dev) for i in range(2)]
    chain, tr = reference_c3_chain(0)
    if c2:
        chain = FusedChain([tr["disk"]])
    junk = torch.zeros(a.flush_mb * (1 << 20) // 4, device=dev) if a.flush_mb else None
    for i in range(a.warmup):
        chain(pool[i % 2], pad=pad)
    torch.cuda.synchronize()
    rt.set_pass_timing(True)
    for i in range(a.iters):
        if junk is not None:
            junk.add_(1.0)
        chain(pool[i % 2], pad=pad)
    torch.cuda.synchronize()
    ms, cnt, nbytes, kernels = rt.pass_stats()
    rt.set_pass_timing(False)
    out = {"tag": a.tag, "config": a.config, "flush_mb": a.flush_mb}
    for i, nm in enumerate(["forward", "kspace", "inverse", "salt_pepper"]):
        if cnt[i]:
            avg = ms[i] / cnt[i]
            e = {"kernel": kernels[i], "us": round(1e3 * avg, 1)}
            if nbytes[i] > 0:
                gbs = nbytes[i] / cnt[i] / (avg * 1e-3) / 1e9
                e.update(GB_s=round(gbs, 0), frac=round(gbs / 8000.0, 3))
            out[nm] = e
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
