"""GPU parity of the half-unit full-spectrum route (slab_ct.h HalfPlan, kspace_ct.h b_mid_split): passes A
and C per (slab, row parity) over a split spectrum, pass B finishing the W transform -- the route of
Fourier.shift_fourier / inv_shift_fourier (filters_and_operators.py:594-632) for 240 x 240 x 155
programs that the band / closed-form / wrap routes do not take (RandGibbsNoised augmentation, the
device-alpha GibbsNoiseLayer, high-pass disks, mixed programs).

Tolerances: half units vs the whole-slab run-time-planned passes (tb_set_half_units(0)) max|d| / max|y| <= 2e-6;
vs the numpy oracle <= 1e-5 (north_star); zero padding exact; per-sample min/max keys bit-exact
against the output.
"""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu

SHAPE = (2, 4, 240, 240, 155)


@pytest.fixture(scope="module")
def rt(gpu):
    from texbias import runtime
    return runtime


def both(rt, x, progs, C, pad=0, out=None):
    """(half route, whole-slab route, kernel names of the half launch, keys half, keys whole)"""
    B = len(progs)
    mm_h = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    mm_w = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    try:
        rt.set_band_plans(False)   # the full-spectrum passes for every program
        rt.set_point_plans(False)
        rt.set_wrap_plans(False)
        rt.set_pass_timing(True)
        yh = rt.kspace_filter(x, 3, progs, C, pad=pad, minmax=mm_h, out=out)
        _, _, _, names = rt.pass_stats()
        rt.set_pass_timing(False)
        rt.set_half_units(False)
        yw = rt.kspace_filter(x, 3, progs, C, pad=pad, minmax=mm_w)
    finally:
        rt.set_half_units(True)
        rt.set_band_plans(True)
        rt.set_point_plans(True)
        rt.set_wrap_plans(True)
    torch.cuda.synchronize()
    return yh, yw, names, mm_h, mm_w


def check_keys(rt, y, mm, D):
    v = y[..., :D].reshape(y.shape[0], -1)
    m = rt.keys_to_float(mm)
    np.testing.assert_array_equal(m[:, 0], v.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(m[:, 1], v.max(1).values.cpu().numpy())


def test_half_route_mixed_program(rt):
    """Disk + plane-wave spike + wrap (the generic middle phase), padded output: half == whole slab,
    == oracle on one channel of each sample, pads zero, keys exact."""
    torch.manual_seed(21)
    x = torch.randn(SHAPE, device="cuda")
    geo = K.geometry(SHAPE[2:])
    idx = (9, 17, 23)
    progs = [[K.disk_op(40.0 + 10 * b, False), K.spike_op(idx, geo, 12.0, phase=0.4 + b), K.wrap_op(0.5)]
             for b in range(2)]
    yh, yw, names, mm_h, _ = both(rt, x, progs, 4, pad=5)
    assert names[:3] == ["k_slab_fwd_half", "k_kspace_half", "k_slab_inv_half"]
    assert torch.all(yh[..., 155:] == 0)
    assert (yh - yw).abs().max().item() / yw.abs().max().item() < 2e-6
    for b, c in ((0, 1), (1, 3)):
        x0 = x[b, c].cpu().numpy()[None]
        ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x0, 40.0 + 10 * b), idx, 12.0, phase=[0.4 + b]), 0.5)[0]
        assert relerr(yh[b, c, ..., :155].cpu().numpy(), ref) < 1e-5
    check_keys(rt, yh, mm_h, 155)


@pytest.mark.parametrize("alpha", [0.0, 0.25, 0.4])
def test_half_route_gibbs(rt, alpha):
    """RandGibbsNoised augmentation (alpha ~ U(0, 0.4), baseline_domain_augment_alpha0p4.py:118) on the
    mask-only middle phase: == oracle, == whole slab."""
    torch.manual_seed(22)
    x = torch.randn(SHAPE, device="cuda")
    progs = [[K.gibbs_op(alpha, SHAPE[2:])]] * 2
    yh, yw, names, mm_h, _ = both(rt, x, progs, 4)
    assert names[1] == "k_kspace_half"
    assert (yh - yw).abs().max().item() / yw.abs().max().item() < 2e-6
    ref = O.gibbs_noise(x[1].cpu().numpy(), alpha)
    assert relerr(yh[1].cpu().numpy(), ref) < 1e-5
    check_keys(rt, yh, mm_h, 155)


def test_half_route_highpass_in_place_strided(rt):
    """High-pass disk (inside_off=True: not a band program) on a strided input view (row pitch 160),
    written in place: == oracle, == the whole-slab passes on a contiguous copy; the columns past 155
    untouched."""
    torch.manual_seed(23)
    base = torch.randn((2, 4, 240, 240, 160), device="cuda")
    tail = base[..., 155:].clone()
    x = base[..., :155]
    x_copy = x.contiguous()
    progs = [[K.disk_op(30.0, True)], [K.disk_op(45.0, True)]]
    mm_h = torch.empty((2, 2), dtype=torch.int32, device="cuda")
    try:
        rt.set_band_plans(False)
        yh = rt.kspace_filter(x, 3, progs, 4, out=x, minmax=mm_h)
        rt.set_half_units(False)
        yw = rt.kspace_filter(x_copy, 3, progs, 4)
    finally:
        rt.set_half_units(True)
        rt.set_band_plans(True)
    torch.cuda.synchronize()
    assert yh.data_ptr() == x.data_ptr()
    assert torch.equal(base[..., 155:], tail)
    assert (yh - yw).abs().max().item() / yw.abs().max().item() < 2e-6
    for b, r in ((0, 30.0), (1, 45.0)):
        ref = O.fourier_disk(x_copy[b].cpu().numpy(), r, inside_off=True)
        assert relerr(yh[b].cpu().numpy(), ref) < 1e-5
    check_keys(rt, yh, mm_h, 155)
