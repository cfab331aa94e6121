"""The split-K MFMA weight-gradient kernel (tb_conv3d_wgrad_f32) against PyTorch's own
Conv3d / ConvTranspose3d gradients on small shapes (float32; summation order differs)."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def conv(gpu):
    from texbias import conv as C
    return C


def _grads(mod, x):
    x = x.clone().requires_grad_(True)
    y = mod(x)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    return y.detach(), x.grad, mod.weight.grad, mod.bias.grad


@pytest.mark.parametrize("cin,cout,stride,shape,fast", [
    (4, 16, 2, (2, 24, 20, 36), True), (16, 16, 1, (2, 12, 10, 40), True), (3, 3, 1, (1, 16, 16, 33), True),
    (20, 5, 1, (2, 10, 12, 18), True), (32, 24, 2, (1, 16, 16, 70), True), (16, 8, 1, (1, 17, 3, 5), True),
    (24, 40, 1, (1, 9, 7, 100), True),
    # rows too wide for a 16-channel tile in the LDS budget: ATen's weight gradient, same results
    (24, 40, 1, (1, 9, 7, 130), False), (8, 6, 1, (1, 5, 3, 250), False)])
def test_conv3d_wgrad(conv, cin, cout, stride, shape, fast, monkeypatch):
    monkeypatch.setattr(conv, "MIN_K_PER_OUTPUT", 1)
    torch.manual_seed(0)
    ref = nn.Conv3d(cin, cout, 3, stride=stride, padding=1).cuda()
    ours = conv.Conv3d(cin, cout, 3, stride=stride, padding=1).cuda()
    ours.load_state_dict(ref.state_dict())
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    out_sp = [(n + 2 - 3) // stride + 1 for n in shape[1:]]
    assert conv.fast_wgrad_applies(x, ours.weight, out_sp, ours.stride, ours.padding, False) == fast
    torch.manual_seed(1)
    yr, gxr, gwr, gbr = _grads(ref, x)
    torch.manual_seed(1)
    yo, gxo, gwo, gbo = _grads(ours, x)
    torch.testing.assert_close(yo, yr)
    torch.testing.assert_close(gxo, gxr)
    torch.testing.assert_close(gbo, gbr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gwo, gwr, rtol=1e-4, atol=1e-3 * gwr.abs().max().item())


@pytest.mark.parametrize("cin,cout,shape", [(16, 16, (2, 12, 10, 40)), (32, 32, (1, 9, 13, 20)), (24, 40, (1, 7, 6, 16)),
                                             (16, 16, (1, 3, 5, 8)), (16, 8, (2, 30, 6, 80)), (64, 64, (2, 5, 7, 12)),
                                             # few channels: k_conv3d_wgrad_zf1 (rows (m, tz, ty), columns (c, tx))
                                             (3, 3, (2, 12, 10, 40)), (3, 3, (1, 9, 7, 240)), (5, 2, (1, 6, 5, 16)),
                                             (1, 1, (2, 5, 3, 8)), (4, 3, (1, 17, 11, 100))])
def test_conv3d_wgrad_zmarch(conv, cin, cout, shape, monkeypatch):
    """Stride-1 layers of >= 8 channels and rows of 4k <= 80 floats take the z-marching kernel
    (k_conv3d_wgrad_zm: one staged input plane meets a ring of three G planes), those of <= 3 output and
    <= 5 input channels its few-channel form (k_conv3d_wgrad_zf1); partial channel tiles, a row block
    past H, z segments of unequal length."""
    monkeypatch.setattr(conv, "MIN_K_PER_OUTPUT", 1)
    torch.manual_seed(0)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    g = torch.randn((shape[0], cout) + shape[1:], device="cuda")
    w = torch.zeros((cout, cin, 3, 3, 3), device="cuda", requires_grad=True)
    ref, = torch.autograd.grad(torch.nn.functional.conv3d(x, w, padding=1), w, g)
    ours = conv.wgrad(g, x, w.shape, 1, 1)
    x64, g64 = x.double(), g.double()
    w64 = torch.zeros((cout, cin, 3, 3, 3), device="cuda", dtype=torch.float64, requires_grad=True)
    r64, = torch.autograd.grad(torch.nn.functional.conv3d(x64, w64, padding=1), w64, g64)
    scale = r64.abs().max().item()
    assert (ours.double() - r64).abs().max().item() <= 4 * max((ref.double() - r64).abs().max().item(), 1e-6 * scale)


@pytest.mark.parametrize("cin,cout,shape", [(16, 32, (2, 12, 10, 40)), (8, 24, (1, 8, 6, 16)), (20, 40, (1, 10, 14, 80)),
                                             (16, 64, (2, 6, 4, 8)),
                                             # few input channels: k_conv3d_wgrad_zf2 ((c, tx) columns, YB rows)
                                             (4, 16, (2, 12, 10, 40)), (3, 8, (1, 8, 6, 16)), (4, 16, (1, 6, 22, 160)),
                                             (5, 40, (2, 6, 10, 24)), (1, 20, (1, 4, 6, 8))])
def test_conv3d_wgrad_zmarch_stride2(conv, cin, cout, shape):
    """Stride-2 layers of >= 8 input channels and output rows of 4k <= 40 take the output-plane
    marching kernel (k_conv3d_wgrad_zm2: a 5-slot ring of input planes, two m-tiles per block), those of
    <= 5 input channels and output rows of 4k <= 80 its few-channel form (k_conv3d_wgrad_zf2); partial
    m / c tiles, row blocks past H."""
    torch.manual_seed(0)
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    osp = tuple(n // 2 for n in shape[1:])
    g = torch.randn((shape[0], cout) + osp, device="cuda")
    w = torch.zeros((cout, cin, 3, 3, 3), device="cuda", requires_grad=True)
    ref, = torch.autograd.grad(torch.nn.functional.conv3d(x, w, stride=2, padding=1), w, g)
    ours = conv.wgrad(g, x, w.shape, 2, 1)
    w64 = torch.zeros((cout, cin, 3, 3, 3), device="cuda", dtype=torch.float64, requires_grad=True)
    r64, = torch.autograd.grad(torch.nn.functional.conv3d(x.double(), w64, stride=2, padding=1), w64, g.double())
    scale = r64.abs().max().item()
    assert (ours.double() - r64).abs().max().item() <= 4 * max((ref.double() - r64).abs().max().item(), 1e-6 * scale)


@pytest.mark.parametrize("cin,cout,shape", [(32, 3, (2, 12, 10, 20)), (64, 16, (1, 12, 10, 16))])
def test_convtranspose3d_wgrad(conv, cin, cout, shape, monkeypatch):
    monkeypatch.setattr(conv, "MIN_K_PER_OUTPUT", 1)
    torch.manual_seed(0)
    ref = nn.ConvTranspose3d(cin, cout, 3, stride=2, padding=1, output_padding=1).cuda()
    ours = conv.ConvTranspose3d(cin, cout, 3, stride=2, padding=1, output_padding=1).cuda()
    ours.load_state_dict(ref.state_dict())
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    assert conv.fast_wgrad_applies(x, ours.weight, None, ours.stride, ours.padding, True)
    torch.manual_seed(1)
    yr, gxr, gwr, gbr = _grads(ref, x)
    torch.manual_seed(1)
    yo, gxo, gwo, gbo = _grads(ours, x)
    torch.testing.assert_close(yo, yr)
    torch.testing.assert_close(gxo, gxr)
    torch.testing.assert_close(gwo, gwr, rtol=1e-4, atol=1e-3 * gwr.abs().max().item())


def test_unet_uses_fast_path_and_trains(conv):
    from texbias.train import TrainStep, reference_model
    torch.manual_seed(0)
    step = TrainStep(reference_model(4, 3), torch.device("cuda"))
    x = torch.randn((2, 4, 32, 32, 32), device="cuda")
    lab = (torch.rand((2, 3, 32, 32, 32), device="cuda") > 0.7).float()
    l0 = step(x, lab).item()
    for _ in range(5):
        l1 = step(x, lab).item()
    assert l1 < l0


@pytest.mark.parametrize("cin,cout,shape", [(3, 3, (2, 12, 10, 40)), (4, 2, (1, 7, 9, 160)), (1, 4, (2, 5, 13, 17))])
def test_small_conv_direct(conv, cin, cout, shape):
    """Direct few-channel conv (tb_conv3d_small_f32): forward, input, weight and bias gradients vs
    PyTorch's Conv3d (float32)."""
    torch.manual_seed(0)
    ref = nn.Conv3d(cin, cout, 3, padding=1).cuda()
    ours = conv.Conv3d(cin, cout, 3, padding=1).cuda()
    ours.load_state_dict(ref.state_dict())
    x = torch.randn((shape[0], cin) + shape[1:], device="cuda")
    assert conv.small_conv_applies(x, ours.weight, ours.stride, ours.padding)
    torch.manual_seed(1)
    yr, gxr, gwr, gbr = _grads(ref, x)
    torch.manual_seed(1)
    yo, gxo, gwo, gbo = _grads(ours, x)
    torch.testing.assert_close(yo, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gxo, gxr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gbo, gbr, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(gwo, gwr, rtol=1e-4, atol=1e-3 * gwr.abs().max().item())


@pytest.mark.parametrize("M,Cc,N,gsp,xsp,stride", [
    (16, 16, 2, (12, 10, 40), (12, 10, 40), 1), (32, 32, 1, (9, 13, 20), (9, 13, 20), 1),
    (24, 40, 1, (7, 6, 16), (7, 6, 16), 1), (64, 64, 2, (5, 7, 12), (5, 7, 12), 1), (16, 16, 2, (20, 24, 80), (20, 24, 80), 1),
    (32, 16, 2, (6, 8, 12), (12, 16, 24), 2), (64, 32, 1, (5, 7, 20), (10, 14, 40), 2),       # k_conv3d_wgrad_zm2
    (3, 3, 2, (10, 12, 40), (10, 12, 40), 1), (2, 5, 1, (7, 9, 16), (7, 9, 16), 1),          # k_conv3d_wgrad_zf1
    (32, 4, 2, (6, 8, 12), (12, 16, 24), 2), (16, 3, 1, (5, 6, 20), (10, 12, 40), 2)])        # k_conv3d_wgrad_zf2
def test_wgrad_partial_tiles_match_atomics(conv, M, Cc, N, gsp, xsp, stride):
    """tb_conv3d_wgrad_ws_f32 (per-workgroup partial tiles + an ordered reduction) against
    tb_conv3d_wgrad_f32 (float atomics) on every z-marching route: the same sums in another order
    (max |d| <= 1e-5 max |dW|), bitwise repeatable, and a too-small workspace falls back to the atomics."""
    from texbias._lib import lib
    torch.manual_seed(5)
    G = torch.randn((N, M) + gsp, device="cuda")
    X = torch.randn((N, Cc) + xsp, device="cuda")
    dims = (N, M, Cc) + gsp + xsp + (stride, 1)
    nb = int(lib().tb_conv3d_wgrad_ws_bytes(*dims))
    assert nb > 0
    st = torch.cuda.current_stream().cuda_stream
    ref = torch.empty((M, Cc, 27), device="cuda")
    assert lib().tb_conv3d_wgrad_f32(G.data_ptr(), X.data_ptr(), ref.data_ptr(), *dims, st) == 0
    outs = []
    for _ in range(2):
        ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
        out = torch.empty_like(ref)
        assert lib().tb_conv3d_wgrad_ws_f32(G.data_ptr(), X.data_ptr(), out.data_ptr(), *dims, ws.data_ptr(), nb, st) == 0
        outs.append(out)
    small = torch.empty_like(ref)
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    assert lib().tb_conv3d_wgrad_ws_f32(G.data_ptr(), X.data_ptr(), small.data_ptr(), *dims, ws.data_ptr(), nb - 4,
                                        st) == 0
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (outs[0] - ref).abs().max().item() <= 1e-5 * scale
    assert torch.equal(outs[0], outs[1])
    assert (small - ref).abs().max().item() <= 1e-5 * scale
