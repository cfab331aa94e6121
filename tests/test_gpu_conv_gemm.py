"""The implicit-GEMM convolutions (csrc/conv_gemm.hip, tb_conv3d_gemm_f32) against PyTorch float32 and a
float64 reference: Conv3d 3x3x3 / 1x1x1 at stride 1 and 2, the input gradient of a stride-1 Conv3d
(flipped, transposed weight), ConvTranspose3d(stride 2, padding 1, output_padding 1) in sub-pixel form
and -- with a stride-2 Conv3d's weight -- that layer's input gradient; the bias, the summed-in ``add``
and an output that is a channel slice of a larger buffer.  Error vs float64 within 4x max(PyTorch
float32's own error, 1e-6 of the largest value) (the bar of tests/test_gpu_conv_up.py)."""
import pytest
import torch
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


CONV = [(16, 32, (2, 12, 10, 8), 2, 3), (32, 64, (1, 6, 8, 10), 2, 3), (64, 128, (2, 6, 6, 4), 2, 3),
        (128, 128, (1, 5, 5, 4), 1, 3), (128, 256, (2, 3, 5, 4), 1, 3), (256, 256, (1, 3, 3, 2), 1, 3),
        (128, 256, (2, 5, 5, 4), 1, 1), (8, 16, (1, 7, 5, 9), 1, 3), (24, 40, (2, 5, 7, 6), 2, 3),
        (8, 24, (1, 9, 3, 5), 1, 3)]


@pytest.mark.parametrize("cin,cout,shape,s,k", CONV)
def test_conv_forward(conv, cin, cout, shape, s, k):
    torch.manual_seed(0)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    w = torch.randn((cout, cin, k, k, k), device="cuda") * (1.0 / (cin * k ** 3) ** 0.5)
    b = torch.randn(cout, device="cuda")
    p = (k - 1) // 2
    y = conv.conv_gemm(x, w, b, "conv", s, k)
    yr = F.conv3d(x, w, b, stride=s, padding=p)
    y64 = F.conv3d(x.double(), w.double(), b.double(), stride=s, padding=p)
    assert y.shape == yr.shape
    close64(y, yr, y64)


@pytest.mark.parametrize("cin,cout,shape,s,k", [c for c in CONV if c[3] == 1])
def test_conv_dgrad_s1(conv, cin, cout, shape, s, k):
    """dX of Conv3d(cin -> cout, stride 1) from dY: mode "dgrad" with the layer's weight."""
    torch.manual_seed(1)
    p = (k - 1) // 2
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda", dtype=torch.float64, requires_grad=True)
    w = torch.randn((cout, cin, k, k, k), device="cuda", dtype=torch.float64) * (1.0 / (cin * k ** 3) ** 0.5)
    y = F.conv3d(x, w, None, stride=1, padding=p)
    g = torch.randn_like(y)
    gx64, = torch.autograd.grad(y, x, g)
    gxr = torch.ops.aten.convolution_backward(g.float(), x.detach().float(), w.float(), None, [1] * 3, [p] * 3,
                                              [1] * 3, False, [0] * 3, 1, [True, False, False])[0]
    gx = conv.conv_gemm(g.float(), w.float(), None, "dgrad", 1, k)
    assert gx.shape == x.shape
    close64(gx, gxr, gx64)


@pytest.mark.parametrize("cin,cout,shape", [(384, 64, (2, 5, 5, 4)), (128, 32, (1, 6, 4, 6)), (64, 16, (2, 3, 4, 4)),
                                            (32, 12, (1, 5, 3, 7)), (8, 40, (2, 2, 3, 5)), (16, 4, (1, 3, 3, 4))])
def test_convT_forward(conv, cin, cout, shape):
    torch.manual_seed(2)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    w = torch.randn((cin, cout, 3, 3, 3), device="cuda") * (1.0 / (cin * 27) ** 0.5)
    b = torch.randn(cout, device="cuda")
    y = conv.conv_gemm(x, w, b, "convT", 2, 3)
    yr = F.conv_transpose3d(x, w, b, stride=2, padding=1, output_padding=1)
    y64 = F.conv_transpose3d(x.double(), w.double(), b.double(), stride=2, padding=1, output_padding=1)
    assert y.shape == yr.shape
    close64(y, yr, y64)


@pytest.mark.parametrize("cin,cout,shape", [(16, 32, (2, 12, 10, 8)), (32, 64, (1, 6, 8, 10)), (64, 128, (2, 6, 6, 4)),
                                            (12, 24, (1, 4, 6, 2))])
def test_conv_s2_dgrad(conv, cin, cout, shape):
    """dX of Conv3d(cin -> cout, stride 2) on even extents = mode "convT" on dY with the layer's weight."""
    torch.manual_seed(3)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda", dtype=torch.float64, requires_grad=True)
    w = torch.randn((cout, cin, 3, 3, 3), device="cuda", dtype=torch.float64) * (1.0 / (cin * 27) ** 0.5)
    y = F.conv3d(x, w, None, stride=2, padding=1)
    g = torch.randn_like(y)
    gx64, = torch.autograd.grad(y, x, g)
    gxr = torch.ops.aten.convolution_backward(g.float(), x.detach().float(), w.float(), None, [2] * 3, [1] * 3,
                                              [1] * 3, False, [0] * 3, 1, [True, False, False])[0]
    gx = conv.conv_gemm(g.float(), w.float(), None, "convT", 2, 3)
    assert gx.shape == x.shape
    close64(gx, gxr, gx64)


def test_add_and_channel_slice(conv):
    """``add`` summed in (aliasing the output: dX += ...) and the output written into a channel slice of a
    wider buffer (the SkipConnection concatenation) with its batch stride."""
    torch.manual_seed(4)
    x = torch.randn((2, 32, 6, 8, 4), device="cuda")
    w = torch.randn((48, 32, 3, 3, 3), device="cuda") * 0.05
    buf = torch.randn((2, 80, 3, 4, 2), device="cuda")
    keep = buf.clone()
    out = buf[:, 16:64]
    add = torch.randn((2, 48, 3, 4, 2), device="cuda")
    conv.conv_gemm(x, w, None, "conv", 2, 3, add=add, out=out)
    ref = F.conv3d(x, w, None, stride=2, padding=1) + add
    torch.testing.assert_close(buf[:, 16:64], ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(buf[:, :16], keep[:, :16], rtol=0, atol=0)
    torch.testing.assert_close(buf[:, 64:], keep[:, 64:], rtol=0, atol=0)
    # add aliasing the output (in-place accumulation)
    acc = torch.randn((2, 48, 3, 4, 2), device="cuda")
    acc0 = acc.clone()
    conv.conv_gemm(x, w, None, "conv", 2, 3, add=acc, out=acc)
    torch.testing.assert_close(acc, F.conv3d(x, w, None, stride=2, padding=1) + acc0, rtol=1e-5, atol=1e-5)


C3 = [("conv", 16, 32, (120, 120, 80), 2, 3), ("conv", 32, 64, (60, 60, 40), 2, 3),
      ("conv", 64, 128, (30, 30, 20), 2, 3), ("conv", 128, 128, (15, 15, 10), 1, 3),
      ("conv", 128, 256, (15, 15, 10), 1, 3), ("conv", 256, 256, (15, 15, 10), 1, 3),
      ("conv", 128, 256, (15, 15, 10), 1, 1), ("convT", 384, 64, (15, 15, 10), 2, 3),
      ("convT", 128, 32, (30, 30, 20), 2, 3)]


@pytest.mark.parametrize("mode,cin,cout,sp,s,k", C3)
def test_c3_layer_shapes(conv, mode, cin, cout, sp, s, k):
    """The U-Net's layers at the bench shape (batch 2, C3) against PyTorch float32, relative to the largest
    value (split-k and the 8 sub-pixel classes at their production tilings)."""
    torch.manual_seed(5)
    x = torch.randn((2, cin) + sp, device="cuda")
    if mode == "conv":
        w = torch.randn((cout, cin, k, k, k), device="cuda") * (1.0 / (cin * k ** 3) ** 0.5)
        y = conv.conv_gemm(x, w, None, "conv", s, k)
        yr = F.conv3d(x, w, None, stride=s, padding=(k - 1) // 2)
    else:
        w = torch.randn((cin, cout, 3, 3, 3), device="cuda") * (1.0 / (cin * 27) ** 0.5)
        y = conv.conv_gemm(x, w, None, "convT", 2, 3)
        yr = F.conv_transpose3d(x, w, None, stride=2, padding=1, output_padding=1)
    assert (y - yr).abs().max().item() <= 2e-5 * yr.abs().max().item()


def test_unsupported_channels_raise(conv):
    """Cin % 8 != 0 is refused (the k order needs 8 channels per tap row group), not computed wrongly."""
    from texbias._lib import TexbiasError
    x = torch.randn((1, 4, 6, 6, 6), device="cuda")
    w = torch.randn((16, 4, 3, 3, 3), device="cuda")
    with pytest.raises(TexbiasError):
        conv.conv_gemm(x, w, None, "conv", 1, 3)


@pytest.mark.parametrize("kind,c,sp", [("small", 3, (12, 10, 20)), ("fwd16", 16, (6, 5, 32)), ("mfma", 32, (6, 7, 8)),
                                       ("mfma", 64, (4, 5, 12)), ("gemm", 128, (3, 5, 4))])
def test_residual_add_epilogues(conv, kind, c, sp):
    """The identity-residual unit's sums in the conv kernels' stores: forward conv(x) + x and input
    gradient dconv(dY) + dY (tb_conv3d_{small,fwd16,mfma}_add_f32, the GEMM's ``add``)."""
    torch.manual_seed(6)
    x = torch.randn((2, c) + sp, device="cuda")
    w = torch.randn((c, c, 3, 3, 3), device="cuda") * (1.0 / (27 * c) ** 0.5)
    b = torch.randn(c, device="cuda")
    m = conv.Conv3d(c, c, 3, padding=1).cuda()
    with torch.no_grad():
        m.weight.copy_(w)
        m.bias.copy_(b)
    r = conv.route_of(m, x)
    assert r.kind == kind, r.kind
    y = r.forward(x, w, b, add=x)
    yr = F.conv3d(x, w, b, padding=1) + x
    assert (y - yr).abs().max().item() <= 2e-5 * yr.abs().max().item()
    g = torch.randn_like(y)
    gx = r.input_grad(g, x, w, add=g)
    gxr = torch.ops.aten.convolution_backward(g, x, w, None, [1] * 3, [1] * 3, [1] * 3, False, [0] * 3, 1,
                                              [True, False, False])[0] + g
    assert (gx - gxr).abs().max().item() <= 2e-5 * gxr.abs().max().item()


@pytest.mark.parametrize("cin,cout,shape", [(128, 32, (1, 6, 4, 6)), (128, 32, (2, 30, 30, 20)), (64, 16, (2, 3, 5, 4))])
def test_convT_input_grad_route(conv, cin, cout, shape, monkeypatch):
    """ConvTranspose3d whose forward stays on MIOpen (the sub-pixel GEMM form is off by default): with
    conv.GEMM_TDX its input gradient runs on the GEMM kernel as a stride-2 Conv3d of dY (Route.dx
    "gemm"), vs ATen and float64;
    the C3 up2 shape (128 -> 32 at 30 x 30 x 20) included."""
    monkeypatch.setattr(conv, "GEMM_TDX", True)
    torch.manual_seed(7)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda", requires_grad=True)
    m = conv.ConvTranspose3d(cin, cout, 3, stride=2, padding=1, output_padding=1).cuda()
    r = conv.Route(x, m.weight, m.stride, m.padding, m.output_padding, True)
    assert r.dx == "gemm"
    y = m(x)
    g = torch.randn_like(y)
    gx, = torch.autograd.grad(y, (x,), g)
    x64 = x.detach().double().requires_grad_(True)
    y64 = F.conv_transpose3d(x64, m.weight.detach().double(), m.bias.detach().double(), stride=2, padding=1,
                             output_padding=1)
    gx64, = torch.autograd.grad(y64, (x64,), g.double())
    gxr = torch.ops.aten.convolution_backward(g, x.detach(), m.weight.detach(), None, [2] * 3, [1] * 3, [1] * 3, True,
                                              [1] * 3, 1, [True, False, False])[0]
    close64(gx, gxr, gx64)
