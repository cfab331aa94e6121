"""Fused InstanceNorm3d + PReLU (tb_instnorm_prelu_{fwd,bwd}_f32) against torch's own
instance_norm -> prelu in float64 on the same inputs: y, dx and the PReLU weight gradient.
Tolerance: max-abs error <= 2e-5 x max|ref| (float32 arithmetic, different summation order)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, w, eps):
    x = x.detach().double().requires_grad_(True)
    w = w.detach().double().requires_grad_(True)
    y = F.prelu(F.instance_norm(x, eps=eps), w)
    return x, w, y


def _close(a, b, tol=2e-5):
    a, b = a.double(), b.double()
    err = (a - b).abs().max().item()
    assert err <= tol * max(b.abs().max().item(), 1e-12), f"max err {err} vs scale {b.abs().max().item()}"


@pytest.mark.parametrize("shape,offset", [((2, 16, 24, 20, 16), 0.0), ((2, 3, 15, 15, 10), 3.0),
                                          ((1, 2, 64, 64, 64), -1.5), ((2, 8, 7, 9, 5), 0.5)])
@pytest.mark.parametrize("a", [0.25, -0.1])
def test_instnorm_prelu_fwd_bwd(gpu, shape, offset, a):
    from texbias.norm import instnorm_prelu
    torch.manual_seed(0)
    x = (torch.randn(shape, device=gpu) * 2.0 + offset).requires_grad_(True)
    w = torch.tensor([a], device=gpu, requires_grad=True)
    y = instnorm_prelu(x, w, 1e-5)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    xr, wr, yr = _ref(x, w, 1e-5)
    (yr * g.double()).sum().backward()
    _close(y, yr)
    _close(x.grad, xr.grad)
    _close(w.grad, wr.grad, tol=1e-5)


def test_adn_module_uses_fused_path(gpu):
    from texbias import unet
    torch.manual_seed(0)
    m = unet.ADN(8).to(gpu)
    x = torch.randn(2, 8, 12, 10, 8, device=gpu, requires_grad=True)
    y = m(x)
    assert y.grad_fn is not None and "InstNormPReLU" in type(y.grad_fn).__name__
    yr = torch.nn.Sequential.forward(m, x)
    _close(y, yr, tol=1e-5)


def test_unet_fused_matches_plain_modules(gpu, monkeypatch):
    """A whole small U-Net step: fused ADN vs the plain InstanceNorm/PReLU modules (both on HIP)."""
    from texbias import unet
    from texbias.losses import DiceLoss
    torch.manual_seed(0)
    m = unet.UNet(3, 4, 3, (16, 32, 64, 128, 256), (2, 2, 2, 2), num_res_units=2).to(gpu)
    x = torch.randn(2, 4, 32, 32, 32, device=gpu)
    lab = (torch.rand(2, 3, 32, 32, 32, device=gpu) > 0.7).float()
    loss_fn = DiceLoss(sigmoid=True, squared_pred=True)
    outs = []
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(unet.ADN, "forward", torch.nn.Sequential.forward)
        m.zero_grad(set_to_none=True)
        loss = loss_fn(m(x), lab)
        loss.backward()
        outs.append((loss.detach(), [p.grad.detach().clone() for p in m.parameters()]))
    (l1, g1), (l2, g2) = outs
    assert abs(l1.item() - l2.item()) <= 1e-5 * abs(l2.item())
    # conv biases in front of an InstanceNorm have an exactly-zero true gradient (the norm removes
    # the mean): compare every gradient against the largest gradient scale, not its own rounding noise
    scale = max(b.abs().max().item() for b in g2)
    for a, b in zip(g1, g2):
        err = (a.double() - b.double()).abs().max().item()
        assert err <= 2e-3 * max(b.abs().max().item(), 1e-4 * scale), (err, b.abs().max().item())


@pytest.mark.parametrize("shape", [(2, 16, 24, 20, 16), (2, 3, 15, 15, 10), (1, 5, 33, 31, 7)])
def test_adn_strided_residual_bias(gpu, shape):
    """tb_adn_fwd/bwd_f32 on channel slices of wider tensors (the stacked unit + residual conv output),
    the residual summed into the store, the producing conv's bias gradient (= dx summed over n and the
    voxels), the PReLU weight gradient; bit-identical on a second run (block-ordered reductions)."""
    from texbias.norm import adn_backward, adn_forward
    torch.manual_seed(1)
    N, C = shape[:2]
    wide = torch.randn((N, 2 * C) + shape[2:], device=gpu) * 1.5 + 0.3
    z = wide[:, :C]                        # conv output: first half of the stacked tensor
    r = wide[:, C:]                        # residual: second half
    w = torch.tensor([0.2], device=gpu)
    out = torch.empty((N, 3 * C) + shape[2:], device=gpu)[:, C:2 * C]
    y, mean, rstd = adn_forward(z, w, 1e-5, res=r, out=out)
    assert y.data_ptr() == out.data_ptr()
    zr, wr, yr = _ref(z, w, 1e-5)
    _close(y, yr + r.double())
    g = torch.randn((N, C) + shape[2:], device=gpu)
    dxbuf = torch.empty((N, 2 * C) + shape[2:], device=gpu)
    dx, dw, db = adn_backward(z, g, mean, rstd, w, need_w=True, need_bias=True, dx_out=dxbuf[:, :C])
    (yr * g.double()).sum().backward()
    _close(dx, zr.grad)
    _close(dw, wr.grad, tol=1e-5)
    # the bias gradient's exact value is 0 (the norm removes a bias): the float64 value from the statistics
    # and the float32 dx summed agree to dx's rounding (6e-8 |dx| per voxel, random: ~sqrt(N S) of them)
    tol = 6e-8 * dx.abs().max().item() * (N * math.prod(shape[2:])) ** 0.5 * 4
    torch.testing.assert_close(db.double(), dx.double().sum(dim=(0, 2, 3, 4)), rtol=0, atol=tol)
    dx2, dw2, db2 = adn_backward(z, g, mean, rstd, w, need_w=True, need_bias=True)
    assert torch.equal(dx2, dx) and torch.equal(dw2, dw) and torch.equal(db2, db)
    # the residual conv's bias gradient out of the same sweep: dy summed over n and the voxels (float64 sums)
    ds = torch.full((C,), float("nan"), device=gpu)
    dx3, _, _ = adn_backward(z, g, mean, rstd, w, need_w=False, need_bias=False, dysum_out=ds)
    assert torch.equal(dx3, dx)
    torch.testing.assert_close(ds.double(), g.double().sum(dim=(0, 2, 3, 4)), rtol=1e-6, atol=1e-6)
    y2, m2, s2 = adn_forward(z, w, 1e-5, res=r)
    assert torch.equal(y2, y) and torch.equal(m2, mean) and torch.equal(s2, rstd)
    from texbias.norm import counters
    assert int(counters(z.device, 1).abs().sum().item()) == 0   # every counter left at zero


def test_skip_buffer_matches_cat(gpu, monkeypatch):
    """The skip concatenation written in place (the submodule's last unit stores into the buffer's upper
    channels, only x copied; strided gradient slices read in place) gives the same loss and parameter
    gradients as torch.cat of separate tensors."""
    from texbias import unet
    from texbias.losses import DiceLoss
    torch.manual_seed(2)
    m = unet.UNet(3, 4, 3, (16, 32, 64, 128, 256), (2, 2, 2, 2), num_res_units=2).to(gpu)
    x = torch.randn(2, 4, 32, 32, 32, device=gpu)
    lab = (torch.rand(2, 3, 32, 32, 32, device=gpu) > 0.7).float()
    loss_fn = DiceLoss(sigmoid=True, squared_pred=True)
    skips = [mod for mod in m.modules() if isinstance(mod, unet.SkipConnection)]
    assert sum(s._tail_unit() is not None for s in skips) == 3   # every level but the bottom
    outs = []
    for inplace in (True, False):
        if not inplace:
            monkeypatch.setattr(unet.SkipConnection, "_tail_unit", lambda self: None)
        m.zero_grad(set_to_none=True)
        y = m(x)
        loss = loss_fn(y, lab)
        loss.backward()
        outs.append((y.detach().clone(), loss.detach(), [p.grad.detach().clone() for p in m.parameters()]))
    (y1, l1, g1), (y2, l2, g2) = outs
    torch.testing.assert_close(y1, y2, rtol=1e-6, atol=1e-6)
    assert abs(l1.item() - l2.item()) <= 1e-6
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * max(b.abs().max().item(), 1e-3))


@pytest.mark.parametrize("shape", [(2, 3, 240, 240, 160), (2, 16, 20, 24, 16), (1, 5, 33, 31, 7)])
def test_channel_sum_partials(gpu, shape):
    """texbias.conv.channel_sum (a conv's bias gradient: float64 block partials summed in block order)
    against float64 sums; bit-identical on a second call."""
    from texbias.conv import channel_sum
    torch.manual_seed(3)
    g = torch.randn(shape, device=gpu) + 0.25
    a = channel_sum(g)
    ref = g.double().sum(dim=(0, 2, 3, 4))
    torch.testing.assert_close(a.double(), ref, rtol=1e-6, atol=1e-6 * math.sqrt(g[:, 0].numel()))
    assert torch.equal(channel_sum(g), a)
