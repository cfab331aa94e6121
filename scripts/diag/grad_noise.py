"""Diagnostic: where does the texbias train step's gradient noise enter?  Runs the bench-shaped U-Net
step (2 x 4 x 240 x 240 x 160, DiceLoss) three times on the same weights and batch -- float64 ATen
(the reference), float32 ATen (texbias switched off) and float32 texbias -- and prints, per ADN block
(InstanceNorm3d + PReLU) in backward order, the normwise error against float64 of
  dy  the gradient arriving at the block's output, and
  dx  the gradient it passes down (its input gradient),
plus each conv's input gradient.  A block whose dx error jumps past ATen's while its dy error does
not is the kernel that adds the noise.  Usage: python scripts/diag/grad_noise.py [--shape H,W,D]"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="240,240,160")
    a = ap.parse_args()
    H, W, D = (int(v) for v in a.shape.split(","))
    torch.manual_seed(6)
    model = reference_model(4, 3).cuda()
    x = torch.randn((2, 4, H, W, D), device="cuda")
    lab = (torch.rand((2, 3, H, W, D), device="cuda") > 0.85).float()
    loss_fn = L.DiceLoss(sigmoid=True, squared_pred=True)
    ref = {}
    errs = {}

    def run(m, xin, tag):
        hooks = []
        for name, mod in m.named_modules():
            if isinstance(mod, (ADN, C.Conv3d, C.ConvTranspose3d)):
                def hk(mod_, gin, gout, name=name):
                    for k, g in (("dy", gout[0]), ("dx", gin[0])):
                        if g is None:
                            continue
                        key = (name, k)
                        if tag == "f64":
                            ref[key] = g.detach().clone()
                        else:
                            errs.setdefault(key, {})[tag] = relmax(g, ref[key])
                hooks.append(mod.register_full_backward_hook(hk))
        l = loss_fn(m(xin), lab.to(xin.dtype))
        l.backward()
        for h in hooks:
            h.remove()
        return l.item()

    saved = (C.ENABLED, N.ENABLED, L.ENABLED)
    C.ENABLED = N.ENABLED = L.ENABLED = False
    m64 = copy.deepcopy(model).double()
    l64 = run(m64, x.double(), "f64")
    g64 = {n: p.grad.detach().clone() for n, p in m64.named_parameters()}
    del m64
    mat = copy.deepcopy(model)
    lat = run(mat, x, "aten")
    gat = {n: relmax(p.grad, g64[n]) for n, p in mat.named_parameters()}
    del mat
    C.ENABLED, N.ENABLED, L.ENABLED = saved
    ltb = run(model, x, "texbias")
    gtb = {n: relmax(p.grad, g64[n]) for n, p in model.named_parameters()}
    print(f"loss f64 {l64:.10f} aten {lat:.10f} texbias {ltb:.10f}")
    print(f"{'module':48s} {'grad':3s} {'aten':>10s} {'texbias':>10s} {'ratio':>7s}")
    for (name, k), e in errs.items():  # backward order (hooks fire as gradients arrive)
        if "aten" in e and "texbias" in e:
            print(f"{name:48s} {k:3s} {e['aten']:10.3e} {e['texbias']:10.3e} {e['texbias'] / max(e['aten'], 1e-12):7.2f}")
    print("parameter gradients (normwise vs float64):")
    for n in gtb:
        print(f"  {n:60s} aten {gat[n]:10.3e} texbias {gtb[n]:10.3e} ratio {gtb[n] / max(gat[n], 1e-12):7.2f}")
    # one texbias family at a time (the others on ATen): which one moves the scalar (PReLU) gradients
    print("scalar parameter gradients with ONE texbias family enabled (conv / norm / loss):")
    fams = {}
    for fam in ("conv", "norm", "loss"):
        C.ENABLED, N.ENABLED, L.ENABLED = fam == "conv", fam == "norm", fam == "loss"
        mf = copy.deepcopy(model)
        mf.zero_grad(set_to_none=True)
        loss_fn(mf(x), lab).backward()
        fams[fam] = {n: relmax(p.grad, g64[n]) for n, p in mf.named_parameters()}
        del mf
    # ATen again with the batch order reversed: the same mathematics, other reduction orders -- the
    # spread of ATen's own float32 error on these cancellation-dominated scalars
    C.ENABLED = N.ENABLED = L.ENABLED = False
    mf = copy.deepcopy(model)
    mf.zero_grad(set_to_none=True)
    loss_fn(mf(x.flip(0)), lab.flip(0)).backward()
    fams["aten_flip"] = {n: relmax(p.grad, g64[n]) for n, p in mf.named_parameters()}
    del mf
    C.ENABLED, N.ENABLED, L.ENABLED = saved
    for n, p in model.named_parameters():
        if p.numel() == 1:
            print(f"  {n:60s} aten {gat[n]:9.2e} aten(flipped batch) {fams['aten_flip'][n]:9.2e} texbias {gtb[n]:9.2e}")
    for n, p in model.named_parameters():
        if p.numel() == 1:
            print(f"  {n:60s} aten {gat[n]:9.2e} all {gtb[n]:9.2e} conv {fams['conv'][n]:9.2e} "
                  f"norm {fams['norm'][n]:9.2e} loss {fams['loss'][n]:9.2e}")


if __name__ == "__main__":
    main()
