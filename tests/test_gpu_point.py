"""GPU parity of the closed-form route for spike-only programs (csrc/kern_point.hip): plane waves
(RandPlaneWaves_ellipsoid, filters_and_operators.py:370-393) and KSpaceSpikeNoise spikes (:906-983)
against the full-spectrum passes (same program, tb_set_point_plans(0)) and the numpy oracle.

Tolerances: closed form vs full passes and vs the float64 exact result (O.spikes_exact: the same
replacements in a float64 spectrum) max|d| / max|y| <= 2e-6; vs oracle <= 1e-5 (north_star), or
1.5x the reference's own polar round-trip floor where that is larger (its float32 log / angle / exp of
EVERY coefficient moves a raw 240x240x155 volume by 1.4e-5 of max|x| against float64 -- no exact
method can be closer to it than that; ``O.polar_roundtrip``); zero padding and min/max keys
bit-exact against the output.
"""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt(gpu):
    from texbias import runtime
    return runtime


def spike(idx, spatial, li, phase=None, chan=-1, grouped=False):
    op = K.spike_op(idx, K.geometry(spatial), li, phase=phase, chan=chan)
    if grouped:
        op.reserved = 1
    return op


def both(rt, x, progs, C, pad=0):
    """(closed form, full passes, kernel names of the closed-form launch, mm closed, mm full)"""
    B = len(progs)
    mm_p = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    mm_f = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    rt.set_pass_timing(True)
    yp = rt.kspace_filter(x, 3, progs, C, pad=pad, minmax=mm_p)
    _, _, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    try:
        rt.set_point_plans(False)
        yf = rt.kspace_filter(x, 3, progs, C, pad=pad, minmax=mm_f)
    finally:
        rt.set_point_plans(True)
    torch.cuda.synchronize()
    return yp, yf, names, mm_p, mm_f


def check_keys(rt, y, mm, D):
    v = y[..., :D].reshape(y.shape[0], -1)
    m = rt.keys_to_float(mm)
    np.testing.assert_array_equal(m[:, 0], v.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(m[:, 1], v.max(1).values.cpu().numpy())


SHAPES = [(2, 4, 32, 30, 16), (2, 3, 24, 20, 15), (1, 2, 31, 17, 30), (2, 4, 128, 128, 64), (2, 4, 240, 240, 155)]


@pytest.mark.parametrize("shape", SHAPES)
def test_planes_closed_form(rt, shape):
    """RandPlaneWaves_ellipsoid alone (the 30_plane_waves_filters drivers): one spike, all channels,
    own phase kept; padded output."""
    torch.manual_seed(3)
    x = torch.randn(shape, device="cuda")
    sp = shape[2:]
    idxs = [tuple(int(n * f) for n, f in zip(sp, (0.8, 0.3, 0.65))), tuple(int(n * 0.15) + 1 for n in sp)]
    progs = [[spike(idxs[b % 2], sp, 12.0 + b)] for b in range(shape[0])]
    yp, yf, names, mmp, mmf = both(rt, x, progs, shape[1], pad=5)
    assert names[0].startswith("k_point_dft") and names[2] == "k_point_apply"
    assert torch.all(yp[..., sp[-1]:] == 0)
    assert (yp - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    check_keys(rt, yp, mmp, sp[-1])
    for b in range(shape[0]):
        xb = x[b].cpu().numpy()
        ref = O.plane_waves(xb, idxs[b % 2], 12.0 + b)
        tol = max(1e-5, 1.5 * relerr(O.polar_roundtrip(xb), xb))
        assert relerr(yp[b, ..., : sp[-1]].cpu().numpy(), ref) < tol


@pytest.mark.parametrize("where", ["dc", "nyquist", "kd0", "override"])
def test_planes_special_frequencies(rt, where):
    """Self-conjugate frequencies (DC; Nyquist on every even axis), the kd = 0 plane, a phase override."""
    shape = (2, 3, 24, 20, 16)
    sp = shape[2:]
    torch.manual_seed(4)
    x = torch.randn(shape, device="cuda")
    phase = None
    if where == "dc":
        idx = tuple(n // 2 for n in sp)             # unshifted (0, 0, 0)
    elif where == "nyquist":
        idx = (0, 0, 0)                              # unshifted (n/2, n/2, n/2)
    elif where == "kd0":
        idx = (3, 17, sp[2] // 2)
    else:
        idx, phase = (5, 7, 3), 0.7
    progs = [[spike(idx, sp, 9.0, phase=phase)] for _ in range(2)]
    yp, yf, names, mmp, _ = both(rt, x, progs, 3)
    assert names[0].startswith("k_point_dft")
    assert (yp - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    check_keys(rt, yp, mmp, sp[-1])
    ref = O.plane_waves(x[1].cpu().numpy(), idx, 9.0, phase=None if phase is None else [phase] * 3)
    assert relerr(yp[1].cpu().numpy(), ref) < 1e-5


def test_kspace_spike_groups_and_channels(rt):
    """KSpaceSpikeNoise with several full (c, h, w, d) locations in one call (grouped spikes, some
    channels without any -> copied), next to a plane-wave sample in the same launch."""
    shape = (2, 4, 32, 30, 16)
    sp = shape[2:]
    torch.manual_seed(5)
    x = torch.randn(shape, device="cuda")
    locs = [(0, 3, 4, 5), (2, 20, 9, 11), (0, 7, 25, 2)]
    vals = [11.0, 12.5, 10.0]
    p0 = [spike(l[1:], sp, v, chan=l[0], grouped=i > 0) for i, (l, v) in enumerate(zip(locs, vals))]
    p1 = [spike((9, 9, 9), sp, 13.0)]
    yp, yf, names, mmp, _ = both(rt, x, [p0, p1], 4, pad=3)
    assert names[0].startswith("k_point_dft")
    assert (yp - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    check_keys(rt, yp, mmp, sp[-1])
    ref = O.kspace_spike(x[0].cpu().numpy(), locs, vals)
    assert relerr(yp[0, ..., : sp[-1]].cpu().numpy(), ref) < 1e-5
    torch.testing.assert_close(yp[0, 1, ..., : sp[-1]], x[0, 1], rtol=0, atol=0)  # channel 1: no spike
    torch.testing.assert_close(yp[0, 3, ..., : sp[-1]], x[0, 3], rtol=0, atol=0)


def test_touching_spikes_take_full_route(rt):
    """Two spikes on conjugate frequencies of one channel are not independent: full passes."""
    shape = (1, 2, 24, 20, 16)
    sp = shape[2:]
    x = torch.randn(shape, device="cuda")
    a = (5, 7, 3)
    conj = tuple((2 * (n // 2) - i) % n for i, n in zip(a, sp))  # shifted index of -f
    prog = [[spike(a, sp, 9.0), spike(conj, sp, 8.0)]]
    rt.set_pass_timing(True)
    rt.kspace_filter(x, 3, prog, 2)
    _, _, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    assert not names[0].startswith("k_point_dft")


def test_planes_in_place_strided(rt):
    """Output aliasing a strided input view (the drop-in writes into the padded U-Net buffer)."""
    shape = (2, 2, 24, 20, 15)
    sp = shape[2:]
    torch.manual_seed(6)
    buf = torch.randn((2, 2, 24, 20, 20), device="cuda")
    view = buf[..., :15]
    x0 = view.clone()
    progs = [[spike((4, 6, 7), sp, 10.0)]] * 2
    rt.kspace_filter(view, 3, progs, 2, out=view)
    torch.cuda.synchronize()
    ref = O.plane_waves(x0[1].cpu().numpy(), (4, 6, 7), 10.0)
    assert relerr(view[1].cpu().numpy(), ref) < 1e-5



def test_planes_closed_form_entry(rt):
    """tb_planes_closed_form_f32 (SURVEY §8b's planes entry) == tb_kspace_filter_f32's own routing of a
    spike-only program, bit for bit; other programs are refused."""
    torch.manual_seed(12)
    shape = (2, 4, 240, 240, 155)
    x = torch.randn(shape, device="cuda")
    progs = [[spike((55, 55, 30), shape[2:], 15.0)], [spike((3, 200, 70), shape[2:], 12.0)]]
    mm_a = torch.empty((2, 2), dtype=torch.int32, device="cuda")
    mm_b = torch.empty((2, 2), dtype=torch.int32, device="cuda")
    ya = rt.planes_closed_form(x, 3, progs, 4, pad=5, minmax=mm_a)
    yb = rt.kspace_filter(x, 3, progs, 4, pad=5, minmax=mm_b)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb) and torch.equal(mm_a, mm_b)
    with pytest.raises(rt.TexbiasError):
        rt.planes_closed_form(x, 3, [[K.wrap_op(0.5)]] * 2, 4)


@pytest.mark.parametrize("shape", [(2, 4, 240, 240, 155), (2, 3, 24, 20, 15), (1, 2, 31, 17, 30)])
def test_closed_form_vs_float64_exact(rt, shape):
    """The closed form against the float64 exact result of the same program (no polar round trip):
    plane waves on sample 0, grouped per-channel spikes with a phase override on sample 1."""
    torch.manual_seed(13)
    x = torch.randn(shape, device="cuda")
    sp = shape[2:]
    C = shape[1]
    s0 = [(tuple(int(n * f) for n, f in zip(sp, (0.8, 0.3, 0.65))), 13.0, None)]
    s1 = [((0, 3, 4, 5), 11.0, None), ((C - 1, sp[0] - 4, 9, 2), 12.5, 0.3), ((0, 7, sp[1] - 2, sp[2] // 2), 10.0, None)]
    sets = [s0, s1][: shape[0]]
    progs = []
    for ss in sets:
        progs.append([spike(idx[-3:], sp, v, phase=ph, chan=idx[0] if len(idx) == 4 else -1,
                            grouped=len(idx) == 4 and i > 0) for i, (idx, v, ph) in enumerate(ss)])
    mm = torch.empty((shape[0], 2), dtype=torch.int32, device="cuda")
    rt.set_pass_timing(True)
    y = rt.kspace_filter(x, 3, progs, C, pad=2, minmax=mm)
    _, _, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    torch.cuda.synchronize()
    assert names[0].startswith("k_point_dft")
    for b, ss in enumerate(sets):
        ref = O.spikes_exact(x[b].double().cpu().numpy(), ss)
        yb = y[b, ..., : sp[-1]].double().cpu().numpy()
        err = np.abs(yb - ref).max() / np.abs(ref).max()
        print(f"{shape} sample {b}: closed form vs float64 exact {err:.2e}")
        assert err < 2e-6
