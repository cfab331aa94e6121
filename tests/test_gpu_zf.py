"""RandZF (k-space undersampling, TB_OP_ZF) on the GPU: the drop-in transform equals the oracle
with the device's mask replayed (relative max error <= 1e-5), on 2-D slices and a 3-D volume;
the kept fraction is 1 - p; inside a low-pass program the band passes agree with the full ones."""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,p", [((1, 128, 128), 0.3), ((3, 40, 36, 30), 0.6), ((2, 33, 17), 1.0), ((1, 64, 64), 0.0)])
def test_randzf_matches_oracle(gpu, shape, p):
    import utils2
    torch.manual_seed(0)
    x = torch.randn(shape)
    t = utils2.RandZF(p)
    y = t(x.cuda()).cpu().numpy()
    keep = O.zf_keep_mask(shape, p, t.last_seed)
    assert abs(keep.mean() - (1 - p)) < 6 * np.sqrt(p * (1 - p) / keep.size) + 1e-12
    ref = O.rand_zf(x.numpy(), keep)
    if p < 1.0:
        assert relerr(y, ref) < 1e-5
    else:
        assert np.abs(y).max() == 0.0


def test_zf_inside_band_program(gpu):
    from texbias import runtime as rt
    torch.manual_seed(1)
    x = torch.randn((2, 4, 48, 40, 36), device="cuda")
    geo = K.geometry((48, 40, 36))
    prog = [K.disk_op(9.0, False), K.zf_op(0.4, 77, geo.hwd), K.wrap_op(0.5)]
    yb = rt.kspace_filter(x, 3, [prog, prog], 4)
    try:
        rt.set_band_plans(False)
        yf = rt.kspace_filter(x, 3, [prog, prog], 4)
    finally:
        rt.set_band_plans(True)
    assert (yb - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    # and the numpy chain: disk -> ZF (replayed mask over the [C, *spatial] sample) -> wrap
    xs = x[1].cpu().numpy()
    keep = O.zf_keep_mask(xs.shape, 0.4, 77)
    ref = O.wrap_artifact(O.rand_zf(O.fourier_disk(xs, 9.0), keep), 0.5)
    assert relerr(yb[1].cpu().numpy(), ref) < 1e-5


def _freq_loss_fft(real, fake):
    """reconGan_freq.py:131-142 as written: MSE of the real and imaginary parts of fftn(dim=(-2, -1))."""
    l2 = torch.nn.MSELoss()
    rk = torch.fft.fftn(real, dim=(-2, -1))
    fk = torch.fft.fftn(fake, dim=(-2, -1))
    return l2(rk.real, fk.real) + l2(rk.imag, fk.imag)


@pytest.mark.parametrize("shape", [(4, 2, 128, 128), (3, 1, 33, 17)])
def test_freq_consistency_closed_form_gpu(gpu, shape):
    """The Parseval closed form equals the reference's FFT formulation (value and gradient, 1e-5)."""
    import utils2
    torch.manual_seed(1)
    real = torch.randn(shape, device="cuda")
    fake = (real + 0.3 * torch.randn(shape, device="cuda")).requires_grad_(True)
    v = utils2.freq_consistency_loss(real, fake)
    g, = torch.autograd.grad(v, fake)
    f2 = fake.detach().clone().requires_grad_(True)
    r = _freq_loss_fft(real, f2)
    gr, = torch.autograd.grad(r, f2)
    assert abs(v.item() - r.item()) <= 1e-5 * abs(r.item())
    assert (g - gr).abs().max().item() <= 1e-5 * gr.abs().max().item()
