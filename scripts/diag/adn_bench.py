"""Diagnostic: per-call time of the ADN sweeps (adn_forward = statistics + apply, adn_backward =
statistics + finalize + apply) and of the bias-gradient channel sum at the C3 U-Net's ADN shapes,
timed with HIP events over 20 calls.  TEXBIAS_LIB selects a library variant for A/B runs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "medical-vision-textural-bias_amd")]
import torch  # noqa: E402

from texbias import conv as C  # noqa: E402
from texbias.norm import adn_backward, adn_forward  # noqa: E402

SHAPES = {"full 3ch": (2, 3, 240, 240, 160), "L1 16ch": (2, 16, 120, 120, 80), "L2 32ch": (2, 32, 60, 60, 40),
          "L3 64ch": (2, 64, 30, 30, 20), "L4 128ch": (2, 128, 15, 15, 10)}


def timed(fn, n=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / n


def main():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    tot = [0.0, 0.0, 0.0]
    for name, sh in SHAPES.items():
        z = torch.randn(sh, device=dev) * 1.5 + 0.3
        r = torch.randn(sh, device=dev)
        g = torch.randn(sh, device=dev)
        w = torch.tensor([0.25], device=dev)
        y, mean, rstd = adn_forward(z, w, 1e-5, res=r)
        tf = timed(lambda: adn_forward(z, w, 1e-5, res=r))
        tb = timed(lambda: adn_backward(z, g, mean, rstd, w, need_w=True, need_bias=True))
        tc = timed(lambda: C.channel_sum(g))
        mb = z.numel() * 4 / 1e6
        print(f"{name:9s} {mb:7.1f} MB/tensor  fwd {tf:7.1f} us  bwd {tb:7.1f} us  channel_sum {tc:6.1f} us  "
              f"(fwd {4 * mb / tf:.2f} TB/s over 4 tensors, bwd {5 * mb / tb:.2f} over 5)", flush=True)
        tot[0] += tf
        tot[1] += tb
        tot[2] += tc
    print(f"total fwd {tot[0]:.1f} bwd {tot[1]:.1f} channel_sum {tot[2]:.1f} us")
    y, _, _ = adn_forward(z, w, 1e-5)
    print("checksum", float(y.double().sum()), flush=True)


if __name__ == "__main__":
    main()
