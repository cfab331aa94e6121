"""GPU parity of the separable wrap route (csrc/kern_wrap.hip): WrapArtifact
(filters_and_operators.py:503-515) as 2-tap H/W combines and a D circulant, against the full-spectrum
passes (same program, tb_set_wrap_plans(0)), the reference's golden fixtures and the numpy oracle.

Tolerances: wrap route vs full passes max|d| / max|y| <= 2e-6; vs golden / oracle <= 1e-5
(north_star); zero padding exact; per-sample min/max keys bit-exact against the output.
"""
import numpy as np
import pytest
import torch

from _golden import load_cases, relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt(gpu):
    from texbias import runtime
    return runtime


def both(rt, x, progs, C, pad=0):
    """(wrap route, full passes, kernel name of the wrap launch, keys wrap, keys full)"""
    B = len(progs)
    mm_w = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    mm_f = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    rt.set_pass_timing(True)
    yw = rt.kspace_filter(x, 3, progs, C, pad=pad, minmax=mm_w)
    _, _, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    try:
        rt.set_wrap_plans(False)
        yf = rt.kspace_filter(x, 3, progs, C, pad=pad, minmax=mm_f)
    finally:
        rt.set_wrap_plans(True)
    torch.cuda.synchronize()
    return yw, yf, names, mm_w, mm_f


def check_keys(rt, y, mm, D):
    v = y[..., :D].reshape(y.shape[0], -1)
    m = rt.keys_to_float(mm)
    np.testing.assert_array_equal(m[:, 0], v.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(m[:, 1], v.max(1).values.cpu().numpy())


@pytest.mark.parametrize("name,case", sorted(load_cases("wrap").items()))
def test_wrap_route_golden(rt, name, case):
    """The reference's own wrap fixtures (odd D = 15 with W/2 = 15 odd, and 16^3 all even)."""
    meta, a = case
    x = torch.from_numpy(np.ascontiguousarray(a["x"])).cuda()[None]
    yw, yf, names, mm_w, _ = both(rt, x, [[K.wrap_op(meta["alpha"])]], x.shape[1])
    H, W, D = x.shape[2:]
    if H % 2 == 0 and W % 2 == 0:   # the separable route needs the 2-tap H / W combines
        assert names[2] == ("k_wrap_dgemm" if D % 2 else "k_wrap_even")
    else:
        assert names[2] in ("k_slab_inv", "k_slab_inv_ct")
    assert relerr(yw[0].cpu().numpy(), a["y"]) < 1e-5
    assert (yw - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    check_keys(rt, yw, mm_w, x.shape[-1])


SHAPES = [(2, 4, 240, 240, 155), (2, 3, 32, 30, 15), (1, 2, 24, 18, 31), (2, 4, 128, 128, 128),
          (2, 2, 16, 12, 10), (1, 3, 20, 22, 193), (3, 1, 6, 10, 7)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("alpha", [0.0, 0.25, 0.5, 0.75, 1.0])
def test_wrap_route_matches_full(rt, shape, alpha):
    """Wrap route == full passes for every alpha the drivers use, with the U-Net padding (odd D up to
    the 256-column tiling: D = 193 runs the 16-tile kernel)."""
    torch.manual_seed(3)
    x = torch.randn(shape, device="cuda") * 3.0 + 1.0
    D = shape[-1]
    pad = 5 if D == 155 else 3
    yw, yf, names, mm_w, mm_f = both(rt, x, [[K.wrap_op(alpha)]] * shape[0], shape[1], pad=pad)
    assert names[2] == ("k_wrap_dgemm" if D % 2 else "k_wrap_even")
    assert (yw - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    assert torch.all(yw[..., D:] == 0)
    check_keys(rt, yw, mm_w, D)


@pytest.mark.parametrize("shape", [(2, 4, 240, 240, 155), (1, 4, 128, 128, 64)])
def test_wrap_route_oracle_c3(rt, shape):
    """Full BraTS size against the numpy oracle (the reference's own FFT arithmetic), per channel."""
    torch.manual_seed(8)
    x = torch.randn(shape, device="cuda")
    mm = torch.empty((shape[0], 2), dtype=torch.int32, device="cuda")
    y = rt.kspace_filter(x, 3, [[K.wrap_op(0.5)]] * shape[0], shape[1], pad=5, minmax=mm)
    torch.cuda.synchronize()
    for b, c in ((0, 0), (shape[0] - 1, shape[1] - 1)):
        ref = O.wrap_artifact(x[b, c:c + 1].cpu().numpy(), 0.5)[0]
        assert relerr(y[b, c, ..., :shape[-1]].cpu().numpy(), ref) < 1e-5


def test_wrap_route_mixed_batch(rt):
    """Per-sample alphas (runs split where the D table changes), an empty program in between, two
    wraps in one program (alphas multiply), an in-place call and strided (non-contiguous) rows."""
    torch.manual_seed(4)
    shape = (5, 3, 32, 30, 15)
    x = torch.randn(shape, device="cuda")
    progs = [[K.wrap_op(0.5)], [K.wrap_op(0.25)], [], [K.wrap_op(0.5), K.wrap_op(0.5)], [K.wrap_op(0.25)]]
    yw, yf, _, mm_w, _ = both(rt, x, progs, 3, pad=1)
    assert (yw - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    check_keys(rt, yw, mm_w, 15)
    xh = x.cpu().numpy()
    for b, al in ((0, 0.5), (1, 0.25), (3, 0.25)):
        assert relerr(yw[b, ..., :15].cpu().numpy(), O.wrap_artifact(xh[b], al)) < 1e-5
    np.testing.assert_array_equal(yw[2, ..., :15].cpu().numpy(), xh[2])
    # strided rows: a view of every other W row of a wider tensor (xs[2] != D -> scalar loads)
    big = torch.randn(2, 3, 32, 60, 15, device="cuda")
    xv = big[:, :, :, ::2, :]
    yv = rt.kspace_filter(xv, 3, [[K.wrap_op(0.5)]] * 2, 3)
    torch.cuda.synchronize()
    ref = O.wrap_artifact(xv[1].contiguous().cpu().numpy(), 0.5)
    assert relerr(yv[1].cpu().numpy(), ref) < 1e-5
    # in place
    z = x[:2].clone()
    z0 = z.cpu().numpy()
    rt.kspace_filter(z, 3, [[K.wrap_op(0.75)]] * 2, 3, out=z)
    torch.cuda.synchronize()
    assert relerr(z[0].cpu().numpy(), O.wrap_artifact(z0[0], 0.75)) < 1e-5


def test_wrap_route_mixed_alpha_even_d_one_launch(rt):
    """Even D: k_wrap_even carries per-sample 2-tap weights, so a batch with different alphas per
    sample runs as ONE launch (odd D still splits where the circulant table changes)."""
    torch.manual_seed(5)
    shape = (4, 2, 16, 12, 10)
    x = torch.randn(shape, device="cuda")
    alphas = [0.0, 0.25, 0.5, 0.75]
    progs = [[K.wrap_op(a)] for a in alphas]
    rt.set_pass_timing(True)
    yw = rt.kspace_filter(x, 3, progs, 2, pad=2)
    _, cnt, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    torch.cuda.synchronize()
    assert names[2] == "k_wrap_even" and cnt[2] == 1
    xh = x.cpu().numpy()
    for b, al in enumerate(alphas):
        assert relerr(yw[b, ..., :10].cpu().numpy(), O.wrap_artifact(xh[b], al)) < 1e-5
    assert torch.all(yw[..., 10:] == 0)
