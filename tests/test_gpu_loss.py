"""Fused Dice statistics (tb_dice_sums_f32 / _bwd) against the plain PyTorch formula of
DiceLoss(sigmoid=True, squared_pred=True) -- forward value and input gradient (float32)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,squared,batch", [((2, 3, 24, 20, 18), True, False), ((1, 2, 16, 9, 7), False, False),
                                                 ((2, 3, 12, 10, 8), True, True)])
def test_dice_fused_matches_plain(gpu, shape, squared, batch):
    from texbias.losses import DiceLoss
    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda", requires_grad=True)
    t = (torch.rand(shape, device="cuda") > 0.6).float()
    loss = DiceLoss(sigmoid=True, squared_pred=squared, batch=batch)
    lf = loss(x, t)
    gf, = torch.autograd.grad(lf, x)
    xc = x.detach().cpu().double().requires_grad_(True)
    lr = loss(xc, t.cpu().double())   # CPU float64: the plain formula
    gr, = torch.autograd.grad(lr, xc)
    assert abs(lf.item() - lr.item()) < 1e-5
    torch.testing.assert_close(gf.cpu().double(), gr, rtol=1e-4, atol=1e-7)
