"""The filters as PyTorch custom operators (texbias/ops.py): schema / fake-tensor checks, torch.compile
without a graph break through the filter, autograd of the Gibbs layer, and HIP-graph capture of the
fused filter chain together with the U-Net train step (bench.py's step).

Tolerances: compiled / captured results equal eager ones bit for bit (same kernels, same inputs).
"""
import numpy as np
import pytest
import torch

from texbias import kprog as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops(gpu):
    from texbias import ops as o
    return o


def _prog(spatial, b=0):
    geo = K.geometry(spatial)
    return [K.disk_op(5.0, False), K.spike_op((3 + b, 7, 9), geo, 9.0, phase=0.4), K.wrap_op(0.5)]


def test_opcheck_kspace_filter(ops):
    x = torch.randn((2, 4, 32, 30, 16), device="cuda")
    progs = ops.pack_programs([_prog((32, 30, 16), b) for b in range(2)])
    torch.library.opcheck(torch.ops.texbias.kspace_filter.default, (x, 3, progs, 4, 5),
                          test_utils=("test_schema", "test_faketensor"))
    y, mm = torch.ops.texbias.kspace_filter(x, 3, progs, 4, 5)
    assert y.shape == (2, 4, 32, 30, 21) and mm.shape == (2, 2) and mm.dtype == torch.int32


def test_compile_fullgraph_no_break(ops):
    """dynamo traces through the filter ops with their fake implementations (fullgraph=True would
    raise on a graph break); the compiled function returns the eager bits."""
    torch.manual_seed(0)
    x = torch.randn((2, 4, 32, 30, 16), device="cuda")
    progs = ops.pack_programs([_prog((32, 30, 16), b) for b in range(2)])
    thr = torch.tensor([[0.025, 0.05], [0.05, 0.1]], dtype=torch.float32)

    def f(x):
        y, mm = torch.ops.texbias.kspace_filter(x, 3, progs, 4, 5)
        z = y.clone()
        torch.ops.texbias.salt_and_pepper_(z[..., :16], mm, thr, 1234, 0, 4)
        return z * 2.0 + 1.0

    ref = f(x)
    exp = torch._dynamo.explain(f)(x)
    assert exp.graph_break_count == 0 and exp.graph_count == 1
    torch._dynamo.reset()
    got = torch.compile(f, fullgraph=True, backend="aot_eager")(x)
    torch.testing.assert_close(got, ref, rtol=0, atol=0)


def test_gibbs_layer_op_autograd(ops):
    """d/dx of the layer = the same (self-adjoint) filter on the gradient; d/d alpha = 0."""
    import stylization_layers as SL
    torch.manual_seed(1)
    layer = SL.GibbsNoiseLayer(0.3).cuda()
    x = torch.randn((2, 1, 16, 16, 8), device="cuda", requires_grad=True)
    g = torch.randn((2, 1, 16, 16, 8), device="cuda")
    y = layer(x)
    (y * g).sum().backward()
    ref = torch.ops.texbias.gibbs_layer(g, layer.alpha)
    torch.testing.assert_close(x.grad, ref, rtol=0, atol=0)
    # adjoint identity <A x, g> = <x, A g>
    lhs = (y.detach().double() * g.double()).sum()
    rhs = (x.detach().double() * ref.double()).sum()
    assert abs(lhs - rhs).item() / abs(lhs).item() < 1e-5
    compiled = torch.compile(lambda t: layer(t) * 3.0, fullgraph=True, backend="aot_eager")
    torch.testing.assert_close(compiled(x.detach()), y.detach() * 3.0, rtol=0, atol=0)


def test_graph_capture_chain_and_train_step(ops):
    """FusedChain (fixed draws, fixed Philox seed) + U-Net train step captured once in a HIP graph
    and replayed: the replay reproduces the eager step's filtered input bit for bit and trains."""
    import filters_and_operators as F
    from texbias.pipeline import FusedChain
    from texbias.synth import brats_labels, brats_like
    from texbias.train import TrainStep, reference_model
    torch.manual_seed(2)
    dev = torch.device("cuda")
    B, C, sp = 2, 4, (32, 32, 16)
    x = brats_like(B, C, sp, seed=3, device=dev)
    lab = brats_labels(B, sp, seed=3, device=dev, pad_to=16)
    disk = F.RandFourierDiskMaskd(keys="image", r=6.5, inside_off=False, prob=1.0)
    planes = F.RandPlaneWaves_ellipsoid("image", 10.0, 10.0, 5.0, intensity_value=9.0, prob=1.0)
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.05)
    chain = FusedChain([disk, planes, wrap, sap])
    plans = chain.plan(B, sp)
    step = TrainStep(reference_model(C, 3), dev, capturable=True)
    # eager reference of the filter stage
    y_ref = chain(x, plans=plans, seed=77).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm up: plans, workspaces, MIOpen solver choice, optimizer state
        for _ in range(3):
            step(chain(x, plans=plans, seed=77), lab)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    step.opt.zero_grad(set_to_none=True)
    with torch.cuda.graph(g):
        y_static = chain(x, plans=plans, seed=77)
        loss_static = step(y_static, lab)
    losses = []
    for _ in range(4):
        g.replay()
        torch.cuda.synchronize()
        losses.append(loss_static.item())
    torch.testing.assert_close(y_static, y_ref, rtol=0, atol=0)
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]


def test_graph_capture_gibbs_unet_survives_gibbs_gd(ops):
    """A captured Gibbs_UNet forward keeps reading the layer's live alpha: gibbs_gd updates the
    buffer in place (its device address never changes), so a replay after the update equals an
    eager forward at the new alpha, bit for bit."""
    import stylization_layers as SL
    from texbias.losses import DiceLoss
    from texbias.train import gibbs_gd
    torch.manual_seed(3)
    net = SL.Gibbs_UNet().cuda().eval()
    x = torch.randn((2, 1, 32, 32, 16), device="cuda")
    lab = (torch.rand((2, 1, 32, 32, 16), device="cuda") > 0.7).float()
    ptr0 = net.gibbs.alpha.data_ptr()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s), torch.no_grad():
        for _ in range(2):
            net(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.no_grad(), torch.cuda.graph(g):
        y_static = net(x)
    a0 = net.gibbs.alpha.clone()
    _, a1 = gibbs_gd(x, lab, net, DiceLoss(sigmoid=True, squared_pred=True), h=0.1, learning_rate=1.0)
    assert net.gibbs.alpha.data_ptr() == ptr0
    assert not torch.equal(a0, a1)
    g.replay()
    with torch.no_grad():
        y_eager = net(x)
    torch.testing.assert_close(y_static, y_eager, rtol=0, atol=0)
