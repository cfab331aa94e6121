"""Diagnostic: one ADN block (InstanceNorm3d + PReLU) of the bench-shaped U-Net step in isolation.
Captures the block's float64 input x and output gradient dy from the float64 reference step, then
runs the block's forward + backward on float32(x), float32(dy) with (a) the texbias fused kernels and
(b) ATen's InstanceNorm3d + PReLU, and compares y, dx and the PReLU weight gradient with float64."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "medical-vision-textural-bias_amd")]
import torch  # noqa: E402

from texbias import conv as C  # noqa: E402
from texbias import losses as L  # noqa: E402
from texbias import norm as N  # noqa: E402
from texbias.train import reference_model  # noqa: E402
from texbias.unet import ADN  # noqa: E402


def relmax(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-300)).item()


def main():
    torch.manual_seed(6)
    model = reference_model(4, 3).cuda()
    x = torch.randn((2, 4, 240, 240, 160), device="cuda")
    lab = (torch.rand((2, 3, 240, 240, 160), device="cuda") > 0.85).float()
    names = sys.argv[1:] or ["model.1.submodule.1.submodule.0.conv.unit0.adn", "model.0.conv.unit0.adn",
                             "model.2.0.adn"]
    C.ENABLED = N.ENABLED = L.ENABLED = False
    m64 = copy.deepcopy(model).double()
    cap = {}
    hooks = []
    for name, mod in m64.named_modules():
        if name in names:
            def fh(mod_, inp, out, name=name):
                cap.setdefault(name, {})["x"] = inp[0].detach().clone()
            def bh(mod_, gin, gout, name=name):
                cap[name]["dy"] = gout[0].detach().clone()
            hooks += [mod.register_forward_hook(fh), mod.register_full_backward_hook(bh)]
    L.DiceLoss(sigmoid=True, squared_pred=True)(m64(x.double()), lab.double()).backward()
    for h in hooks:
        h.remove()
    for name in names:
        x64, dy64 = cap[name]["x"], cap[name]["dy"]
        adn = dict(m64.named_modules())[name]
        w = adn.A.weight.detach()
        res = {}
        for tag, dt, tb in (("f64", torch.float64, False), ("aten", torch.float32, False), ("texbias", torch.float32, True)):
            N.ENABLED = tb
            blk = ADN(x64.shape[1]).cuda().to(dt)
            blk.A.weight.data.copy_(w.to(dt))
            xi = x64.detach().to(dt).clone().requires_grad_(True)
            y = blk(xi)
            y.backward(dy64.to(dt))
            res[tag] = (y.detach(), xi.grad.detach(), blk.A.weight.grad.detach().clone())
        N.ENABLED = False
        ref = res["f64"]
        m = x64.mean((2, 3, 4)).abs().max().item()
        s = x64.std((2, 3, 4)).min().item()
        print(f"{name}: x {tuple(x64.shape)} max|mean| {m:.3e} min std {s:.3e}")
        for tag in ("aten", "texbias"):
            y, dx, dw = res[tag]
            print(f"   {tag:8s} y {relmax(y, ref[0]):.3e}  dx {relmax(dx, ref[1]):.3e}  dw {relmax(dw, ref[2]):.3e} "
                  f"(dw {dw.item():.6e} vs f64 {ref[2].item():.6e})")


if __name__ == "__main__":
    main()
