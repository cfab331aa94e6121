"""The frequency-consistency loss of reconGan_freq.py:131-142 in its Parseval closed form
(utils2.freq_consistency_loss = H W MSE) against the reference's FFT formulation, float64 on the CPU
(the function is plain torch; tolerance 1e-12 relative)."""
import pytest
import torch


@pytest.mark.parametrize("shape", [(2, 2, 16, 12), (1, 7, 9), (5, 31)])
def test_freq_consistency_closed_form_cpu(shape):
    import utils2
    torch.manual_seed(0)
    real = torch.randn(shape, dtype=torch.float64)
    fake = torch.randn(shape, dtype=torch.float64, requires_grad=True)
    v = utils2.freq_consistency_loss(real, fake)
    g, = torch.autograd.grad(v, fake)
    f2 = fake.detach().clone().requires_grad_(True)
    l2 = torch.nn.MSELoss()
    rk, fk = torch.fft.fftn(real, dim=(-2, -1)), torch.fft.fftn(f2, dim=(-2, -1))
    r = l2(rk.real, fk.real) + l2(rk.imag, fk.imag)
    gr, = torch.autograd.grad(r, f2)
    assert abs(v.item() - r.item()) <= 1e-12 * abs(r.item())
    assert torch.allclose(g, gr, rtol=0, atol=1e-12 * gr.abs().max().item())
    assert utils2.FreqConsistencyLoss()(real, fake).item() == v.item()
