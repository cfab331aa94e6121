"""Adam on the texbias kernel (texbias.optim.Adam -> tb_adam_f32) against ATen's fused Adam and its
single-tensor Adam on the same parameters and gradient sequence: the reference's configuration
(lr 1e-4, weight_decay 1e-5, amsgrad; stylized_gibbs12p5.py:203-205) and the other branches, over
tensors of the U-Net's kinds (conv weights, biases, the 1-element PReLU weights), a tensor longer than
one launch chunk, an odd size and an unaligned packed view.  Tolerance: 2 float32 ulps of the parameter
plus 1e-5 of the updates' size (the same expressions as ATen's fused Adam; float32 rounding only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(gpu, seed):
    """Leaf tensors requiring grad; the last is an unaligned view into a larger storage (as the packed
    [unit0; residual] weights of a strided ResidualUnit are)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    shapes = [(16, 4, 3, 3, 3), (16,), (1,), (3, 5, 7), (64, 32, 3, 3, 3), (300001,)]
    ps = [torch.randn(s, generator=g).to(gpu).requires_grad_(True) for s in shapes]
    packed = torch.randn(1 + 16 * 27, generator=g).to(gpu)
    view = packed[1:].view(16, 27).requires_grad_(True)
    assert view.data_ptr() % 16 != 0
    return ps + [view]


@pytest.mark.parametrize("lr,wd,ams", [(1e-4, 1e-5, True), (1e-3, 0.0, False), (3e-3, 1e-2, True)])
def test_adam_matches_aten(gpu, lr, wd, ams):
    from texbias.optim import Adam
    ref_fused, ref_single, mine = _params(gpu, 0), _params(gpu, 0), _params(gpu, 0)
    o_f = torch.optim.Adam(ref_fused, lr=lr, weight_decay=wd, amsgrad=ams, fused=True)
    o_s = torch.optim.Adam(ref_single, lr=lr, weight_decay=wd, amsgrad=ams, foreach=False)
    o_m = Adam(mine, lr=lr, weight_decay=wd, amsgrad=ams)
    g = torch.Generator(device="cpu").manual_seed(1)
    for _ in range(6):
        grads = [torch.randn(p.shape, generator=g).to(gpu) * 0.1 for p in mine]
        for ps, opt in ((ref_fused, o_f), (ref_single, o_s), (mine, o_m)):
            for p, gr in zip(ps, grads):
                p.grad = gr.clone()
            opt.step()
    for a, b, c in zip(mine, ref_fused, ref_single):
        # 2 ulps of the parameter plus 1e-5 of the six updates' size (lr each, at most)
        tol = 2 * torch.finfo(torch.float32).eps * b.detach().abs() + 1e-5 * 6 * lr
        assert ((a - b).abs() <= tol).all(), (a - b).abs().max().item()
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-7)
    for pm, pf in zip(mine, ref_fused):
        sm, sf = o_m.state[pm], o_f.state[pf]
        assert float(sm["step"]) == float(sf["step"]) == 6.0
        # moments: float32 rounding of the running sums (m crosses zero: absolute, on the moment's scale)
        for k in ("exp_avg", "exp_avg_sq") + (("max_exp_avg_sq",) if ams else ()):
            torch.testing.assert_close(sm[k], sf[k], rtol=1e-6, atol=1e-6 * sf[k].abs().max().item())


def test_adam_state_dict_and_graph(gpu):
    """state_dict round trip into a fresh optimizer continues identically; the step replays in a HIP graph."""
    from texbias.optim import Adam
    ps, qs = _params(gpu, 3), _params(gpu, 3)
    o1, o2 = Adam(ps, lr=1e-3, weight_decay=1e-5, amsgrad=True), Adam(qs, lr=1e-3, weight_decay=1e-5, amsgrad=True)
    for p, q in zip(ps, qs):
        p.grad = torch.full_like(p, 0.01)
        q.grad = torch.full_like(q, 0.01)
    o1.step()
    o2.step()
    o3 = Adam(qs, lr=1e-3, weight_decay=1e-5, amsgrad=True)
    o3.load_state_dict(o2.state_dict())
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            o3.step()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        o1.step()
        graph.replay()
    torch.cuda.synchronize()
    for p, q in zip(ps, qs):
        assert torch.equal(p, q)
    assert float(o3.state[qs[0]]["step"]) == 4.0  # 1 eager step + 3 replays (capture records, runs nothing)


def test_trainstep_uses_texbias_adam(gpu):
    from texbias import optim
    from texbias.train import TrainStep
    from texbias.unet import UNet
    ts = TrainStep(UNet(3, 1, 1, (4, 8), (2,), num_res_units=1), gpu)
    assert isinstance(ts.opt, optim.Adam) and ts.opt.defaults["amsgrad"] and ts.opt.defaults["weight_decay"] == 1e-5
