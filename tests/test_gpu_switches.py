"""The documented run-time switches of the train step (INTEGRATION.md "Switches"): each module-level
switch turned off routes its part of the U-Net step to ATen (MIOpen / CK / PyTorch reductions) and must
give the same loss and gradients as the texbias kernels, to float32 rounding of a different summation
order -- so every switch left in the product is exercised.  Shape: [2, 4, 32, 32, 32] (the routes
exercised at this size: fwd16 / mfma / small / gemm convs, the fused ADN, the Dice sums).

Tolerance: loss |dl| <= 1e-5 |l|; per parameter ||dg|| <= 2e-3 ||g|| + 1e-6 (float32, two summation orders
of 10^4 - 10^6 term reductions)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(model, x, y):
    from texbias.losses import DiceLoss
    model.zero_grad(set_to_none=True)
    loss = DiceLoss(sigmoid=True, squared_pred=True)(model(x), y)
    loss.backward()
    return loss.detach(), [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("switch", ["conv.ENABLED", "norm.ENABLED", "losses.ENABLED", "unet.FUSED", "conv.GEMM"])
def test_switch_off_matches(gpu, monkeypatch, switch):
    import importlib

    from texbias.train import reference_model
    from texbias.unet import pack_parameters
    torch.manual_seed(3)
    model = reference_model(4, 3).to(gpu)
    pack_parameters(model)
    x = torch.randn(2, 4, 32, 32, 32, device=gpu)
    y = (torch.rand(2, 3, 32, 32, 32, device=gpu) > 0.7).float()
    l0, g0 = _step(model, x, y)
    mod, attr = switch.split(".")
    m = importlib.import_module(f"texbias.{mod}")
    assert getattr(m, attr) is True
    monkeypatch.setattr(m, attr, False)
    for sub in model.modules():  # cached conv routes were chosen with the switch on
        sub.__dict__.pop("_tb_routes", None)
    l1, g1 = _step(model, x, y)
    assert abs(l1.item() - l0.item()) <= 1e-5 * abs(l0.item())
    for a, b in zip(g0, g1):
        assert (a - b).norm().item() <= 2e-3 * a.norm().item() + 1e-6
