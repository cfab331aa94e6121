"""Fused Dice statistics (tb_dice_sums_f32 / _bwd) against the plain PyTorch formula of
DiceLoss(sigmoid=True, squared_pred=True) -- forward value and input gradient (float32)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,squared,batch,red", [((2, 3, 24, 20, 18), True, False, "mean"),
                                                     ((1, 2, 16, 9, 7), False, False, "mean"),
                                                     ((2, 3, 12, 10, 8), True, True, "mean"),
                                                     ((2, 3, 12, 10, 8), True, False, "sum"),
                                                     ((3, 2, 8, 6, 4), True, False, "none"),
                                                     ((3, 2, 8, 6, 4), False, True, "none")])
def test_dice_fused_matches_plain(gpu, shape, squared, batch, red):
    """The fused loss (sums sweep + one-launch finalize, and the one-launch gradient of the sums) vs the
    plain formula on the CPU in float64, every reduction."""
    from texbias.losses import DiceLoss
    torch.manual_seed(0)
    x = torch.randn(shape, device="cuda", requires_grad=True)
    t = (torch.rand(shape, device="cuda") > 0.6).float()
    loss = DiceLoss(sigmoid=True, squared_pred=squared, batch=batch, reduction=red)
    lf = loss(x, t)
    gup = torch.rand(lf.shape, device="cuda") + 0.5
    gf, = torch.autograd.grad(lf, x, gup)
    xc = x.detach().cpu().double().requires_grad_(True)
    lr = loss(xc, t.cpu().double())   # CPU float64: the plain formula
    gr, = torch.autograd.grad(lr, xc, gup.cpu().double())
    assert lf.shape == lr.shape
    torch.testing.assert_close(lf.cpu().double(), lr, rtol=0, atol=1e-5)
    torch.testing.assert_close(gf.cpu().double(), gr, rtol=1e-4, atol=1e-7)
