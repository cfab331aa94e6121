"""The full-resolution stride-2 layers of the U-Net on the direct kernels (csrc/conv_up.hip):
Conv3d(Cin <= 4 -> 16/32, stride 2) forward and ConvTranspose3d(Cin -> Cout <= 4, stride 2,
output_padding 1) forward and input gradient, against PyTorch (MIOpen) float32 and a float64 reference:
the error vs float64 within 4x max(PyTorch float32's, 1e-6 of the largest value)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def conv(gpu):
    from texbias import conv
    return conv


def close64(ours, ref32, ref64):
    scale = ref64.abs().max().item()
    e_ours = (ours.double() - ref64).abs().max().item()
    e_ref = (ref32.double() - ref64).abs().max().item()
    assert e_ours <= 4 * max(e_ref, 1e-6 * scale), (e_ours, e_ref, scale)


@pytest.mark.parametrize("cin,cout,shape", [(4, 16, (2, 12, 10, 32)), (3, 32, (1, 8, 6, 16)), (1, 16, (1, 6, 4, 8)),
                                            (4, 16, (1, 10, 14, 160)), (2, 32, (2, 4, 6, 24))])
def test_conv_s2_fewin(conv, cin, cout, shape):
    torch.manual_seed(0)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    ours = conv.Conv3d(cin, cout, 3, stride=2, padding=1).cuda()
    assert conv.s2_fewin_applies(x, ours.weight, ours.stride, ours.padding)
    ref = nn.Conv3d(cin, cout, 3, stride=2, padding=1).cuda()
    ref.load_state_dict(ours.state_dict())
    y = ours(x)
    yr = ref(x)
    y64 = F.conv3d(x.double(), ref.weight.double(), ref.bias.double(), stride=2, padding=1)
    close64(y, yr, y64)
    g = torch.randn_like(y)
    (gw, gb), (gwr, gbr) = torch.autograd.grad(y, (ours.weight, ours.bias), g), \
        torch.autograd.grad(yr, (ref.weight, ref.bias), g)
    w64 = ref.weight.double().detach().requires_grad_(True)
    gw64, = torch.autograd.grad(F.conv3d(x.double(), w64, None, stride=2, padding=1), w64, g.double())
    close64(gw, gwr, gw64)
    torch.testing.assert_close(gb, gbr, rtol=1e-4, atol=1e-4 * gbr.abs().max().item())


@pytest.mark.parametrize("cin,cout,shape", [(32, 3, (2, 6, 5, 20)), (16, 2, (1, 4, 6, 8)), (32, 4, (1, 5, 3, 12)),
                                            (32, 3, (1, 4, 4, 80)), (16, 1, (2, 3, 7, 4))])
def test_convT_fewout(conv, cin, cout, shape):
    torch.manual_seed(1)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda", requires_grad=True)
    ours = conv.ConvTranspose3d(cin, cout, 3, stride=2, padding=1, output_padding=1).cuda()
    assert conv.convT_fewout_applies(x, ours.weight, ours.stride, ours.padding, ours.output_padding)
    ref = nn.ConvTranspose3d(cin, cout, 3, stride=2, padding=1, output_padding=1).cuda()
    ref.load_state_dict(ours.state_dict())
    y = ours(x)
    yr = ref(x)
    x64 = x.detach().double().requires_grad_(True)
    w64 = ref.weight.detach().double().requires_grad_(True)
    y64 = F.conv_transpose3d(x64, w64, ref.bias.double(), stride=2, padding=1, output_padding=1)
    close64(y, yr, y64)
    g = torch.randn_like(y)
    gx, gw, gb = torch.autograd.grad(y, (x, ours.weight, ours.bias), g)
    gxr, gwr, gbr = torch.autograd.grad(yr, (x, ref.weight, ref.bias), g)
    gx64, gw64 = torch.autograd.grad(y64, (x64, w64), g.double())
    close64(gx, gxr, gx64)
    close64(gw, gwr, gw64)
    torch.testing.assert_close(gb, gbr, rtol=1e-4, atol=1e-4 * gbr.abs().max().item())


def test_full_resolution_layers(conv):
    """The bench shapes: Conv3d(4 -> 16, s2) on 2 x 4 x 240 x 240 x 160 and ConvTranspose3d(32 -> 3, s2)
    from 2 x 32 x 120 x 120 x 80, forward and input gradient against PyTorch float32 (relative to the
    largest value; the float64 comparison runs at the small shapes above)."""
    torch.manual_seed(2)
    x = torch.randn((2, 4, 240, 240, 160), device="cuda")
    c = conv.Conv3d(4, 16, 3, stride=2, padding=1).cuda()
    y = c(x)
    yr = F.conv3d(x, c.weight, c.bias, stride=2, padding=1)
    assert (y - yr).abs().max().item() <= 2e-5 * yr.abs().max().item()
    xt = torch.randn((2, 32, 120, 120, 80), device="cuda", requires_grad=True)
    t = conv.ConvTranspose3d(32, 3, 3, stride=2, padding=1, output_padding=1).cuda()
    yt = t(xt)
    ytr = F.conv_transpose3d(xt, t.weight, t.bias, stride=2, padding=1, output_padding=1)
    assert (yt - ytr).abs().max().item() <= 2e-5 * ytr.abs().max().item()
    g = torch.randn_like(yt)
    gx, = torch.autograd.grad(yt, xt, g)
    gxr, = torch.autograd.grad(ytr, xt, g)
    assert (gx - gxr).abs().max().item() <= 2e-5 * gxr.abs().max().item()


@pytest.mark.parametrize("shape", [(2, 6, 5, 32), (1, 9, 7, 80), (1, 3, 4, 16), (2, 12, 10, 48)])
def test_conv16_mfma(conv, shape):
    """Conv3d(16 -> 16, stride 1) forward and input gradient on k_conv3d_fwd16 (weight gradient: z-march)."""
    torch.manual_seed(3)
    x = torch.randn((shape[0], 16) + shape[1:], device="cuda", requires_grad=True)
    ours = conv.Conv3d(16, 16, 3, padding=1).cuda()
    assert conv.conv16_applies(x, ours.weight, ours.stride, ours.padding)
    ref = nn.Conv3d(16, 16, 3, padding=1).cuda()
    ref.load_state_dict(ours.state_dict())
    y, yr = ours(x), ref(x)
    x64 = x.detach().double().requires_grad_(True)
    w64 = ref.weight.detach().double().requires_grad_(True)
    y64 = F.conv3d(x64, w64, ref.bias.double(), padding=1)
    close64(y, yr, y64)
    g = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, (x, ours.weight), g)
    gxr, gwr = torch.autograd.grad(yr, (x, ref.weight), g)
    gx64, gw64 = torch.autograd.grad(y64, (x64, w64), g.double())
    close64(gx, gxr, gx64)
    close64(gw, gwr, gw64)


@pytest.mark.parametrize("shape", [(1, 3, 4, 8), (2, 5, 6, 40), (1, 4, 3, 16), (2, 60, 60, 40)])
def test_convT64_mfma(conv, shape):
    """ConvTranspose3d(64 -> 16, stride 2) forward on k_convT_mfma64 (sub-pixel, f32 matrix cores) vs
    ATen and float64; the C3 up1 shape is the last case."""
    torch.manual_seed(4)
    x = torch.randn((shape[0], 64) + shape[1:], device="cuda", requires_grad=True)
    ours = conv.ConvTranspose3d(64, 16, 3, stride=2, padding=1, output_padding=1).cuda()
    assert conv.convT64_applies(x, ours.weight, ours.stride, ours.padding, ours.output_padding)
    ref = nn.ConvTranspose3d(64, 16, 3, stride=2, padding=1, output_padding=1).cuda()
    ref.load_state_dict(ours.state_dict())
    y, yr = ours(x), ref(x)
    x64 = x.detach().double().requires_grad_(True)
    w64 = ref.weight.detach().double().requires_grad_(True)
    y64 = F.conv_transpose3d(x64, w64, ref.bias.double(), stride=2, padding=1, output_padding=1)
    close64(y, yr, y64)
    if shape[1] > 10:
        return  # the gradients are _ConvFn's (ATen input gradient, z-march weight gradient), tested elsewhere
    g = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, (x, ours.weight), g)
    gxr, gwr = torch.autograd.grad(yr, (x, ref.weight), g)
    gx64, gw64 = torch.autograd.grad(y64, (x64, w64), g.double())
    close64(gx, gxr, gx64)
    close64(gw, gwr, gw64)


@pytest.mark.parametrize("C,shape", [(32, (1, 5, 4, 40)), (32, (2, 3, 7, 12)), (64, (1, 4, 5, 20)), (64, (2, 3, 3, 8)),
                                     (32, (2, 60, 60, 40)), (64, (2, 30, 30, 20)), (32, (1, 4, 3, 64)),
                                     (64, (1, 3, 4, 48))])
def test_conv_mfma(conv, C, shape):
    """Conv3d(C -> C, stride 1), C = 32 / 64: forward and input gradient on k_conv3d_mfma_s1 (weight
    gradient: z-march) vs ATen and float64; the C3 shapes of the 32- and 64-channel units included."""
    torch.manual_seed(5)
    x = torch.randn((shape[0], C) + shape[1:], device="cuda", requires_grad=True)
    ours = conv.Conv3d(C, C, 3, padding=1).cuda()
    assert conv.conv_mfma_applies(x, ours.weight, ours.stride, ours.padding)
    ref = nn.Conv3d(C, C, 3, padding=1).cuda()
    ref.load_state_dict(ours.state_dict())
    y, yr = ours(x), ref(x)
    x64 = x.detach().double().requires_grad_(True)
    w64 = ref.weight.detach().double().requires_grad_(True)
    y64 = F.conv3d(x64, w64, ref.bias.double(), padding=1)
    close64(y, yr, y64)
    g = torch.randn_like(y)
    gx, gw = torch.autograd.grad(y, (x, ours.weight), g)
    gxr, gwr = torch.autograd.grad(yr, (x, ref.weight), g)
    gx64, gw64 = torch.autograd.grad(y64, (x64, w64), g.double())
    close64(gx, gxr, gx64)
    close64(gw, gwr, gw64)


@pytest.mark.parametrize("shape", [(1, 6, 8, 16), (2, 10, 6, 24), (2, 120, 120, 80)])
def test_s2_dgrad_mfma(conv, shape):
    """Conv3d(16 -> 32, stride 2): its input gradient on k_convT_mfma64 with 32 input channels vs ATen
    and float64 (the C3 down1 shape last)."""
    torch.manual_seed(6)
    x = torch.randn((shape[0], 16) + shape[1:], device="cuda", requires_grad=True)
    ours = conv.Conv3d(16, 32, 3, stride=2, padding=1).cuda()
    ref = nn.Conv3d(16, 32, 3, stride=2, padding=1).cuda()
    ref.load_state_dict(ours.state_dict())
    y, yr = ours(x), ref(x)
    g = torch.randn_like(y)
    assert conv.s2_dgrad_applies(g, x, ours.weight, ours.stride, ours.padding)
    gx, = torch.autograd.grad(y, (x,), g)
    gxr, = torch.autograd.grad(yr, (x,), g)
    x64 = x.detach().double().requires_grad_(True)
    y64 = F.conv3d(x64, ref.weight.double(), ref.bias.double(), stride=2, padding=1)
    gx64, = torch.autograd.grad(y64, (x64,), g.double())
    close64(gx, gxr, gx64)


@pytest.mark.parametrize("C,shape", [(16, (2, 6, 5, 32)), (32, (2, 5, 6, 12)), (64, (2, 4, 5, 8))])
def test_dgrad_strided_add(conv, C, shape):
    """The input-gradient kernels with the residual sum in their store, the add read in place from a
    channel slice of a wider tensor (tb_conv3d_{fwd16,mfma}_dgrad_f32 with add_sn) vs float64."""
    torch.manual_seed(8)
    g = torch.randn((shape[0], C) + shape[1:], device="cuda")
    w = torch.randn((C, C, 3, 3, 3), device="cuda") * (1.0 / (27 * C) ** 0.5)
    wide = torch.randn((shape[0], 2 * C) + shape[1:], device="cuda")
    add = wide[:, C:]
    dx = conv.conv_fwd16_dgrad(g, w, add) if C == 16 else conv.conv_mfma_dgrad(g, w, add)
    ref = F.conv_transpose3d(g.double(), w.double(), None, padding=1) + add.double()
    assert (dx.double() - ref).abs().max().item() <= 2e-5 * ref.abs().max().item()
