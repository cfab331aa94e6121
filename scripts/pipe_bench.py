#!/usr/bin/env python3
"""Experiment: the C3 filter chain over a batch of 2 as one call vs two one-sample calls on two
streams at once (can the latency-bound passes B' and S&P of one sample hide under the other's
bandwidth-bound passes?).  HIP events around each variant, cache flush between calls, median of 20."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    from texbias.pipeline import reference_c3_chain
    from texbias.synth import brats_like
    dev = torch.device("cuda", 0)
    x = brats_like(2, 4, (240, 240, 155), seed=0, device=dev)
    ch = [reference_c3_chain(0)[0] for _ in range(3)]
    junk = torch.zeros(1024 * (1 << 20) // 4, device=dev)
    ss = [torch.cuda.Stream(), torch.cuda.Stream()]
    parts = [x[0:1], x[1:2]]

    def one():
        return ch[0](x, pad=5, seed=7)

    def two():
        cur = torch.cuda.current_stream()
        out = [None, None]
        for i in range(2):
            ss[i].wait_stream(cur)
            with torch.cuda.stream(ss[i]):
                out[i] = ch[1 + i](parts[i], pad=5, seed=7 + i)
        for i in range(2):
            cur.wait_stream(ss[i])
        return out

    for name, fn in (("batch of 2, one stream", one), ("2 x 1 sample, two streams", two),
                     ("batch of 2, one stream", one)):
        for _ in range(3):
            fn()
        ts = []
        for _ in range(20):
            junk.add_(1.0)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        print(f"{name:28s} median {ts[10] * 1e3:7.1f} us  min {ts[0] * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
