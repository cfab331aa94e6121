"""GPU parity of the direct-DFT fallback (csrc/kern_generic.hip) against the numpy oracle.

The reference's torch.fft.fftn takes any size (source_code/filters_and_operators.py:594-632).
The mixed-radix passes take prime factors up to 31 and a (W, D) slab whose half spectrum fits in
LDS; any other plan runs its full-spectrum route on the fallback (O(n) work per coefficient and
axis), and its low-pass programs still on the band passes.  The shapes here have axes of 37, 41,
43, 53 and 59 and a 512 x 300 slab.  They are not in the reference's fixtures: the checks are
against the oracle (itself pinned by those fixtures in test_oracle_golden.py).

Tolerance: max|y - y_ref| / max|y_ref| <= 1e-5 (north_star); min/max keys equal the output's.
"""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu
TOL = 1e-5
SHAPES = [(2, 37, 41, 43), (1, 8, 53, 59), (1, 4, 512, 300)]


@pytest.fixture(scope="module")
def rt(gpu):
    from texbias import runtime
    return runtime


@pytest.fixture
def no_band(rt):
    rt.set_band_plans(False)
    yield
    rt.set_band_plans(True)


def run(rt, x, prog, pad=0):
    chans = x.shape[0]
    xb = torch.from_numpy(np.ascontiguousarray(x)).cuda().reshape((1,) + x.shape)
    mm = torch.empty((1, 2), dtype=torch.int32, device="cuda")
    y = rt.kspace_filter(xb, 3, [prog], chans, pad=pad, minmax=mm)
    torch.cuda.synchronize()
    return y.cpu().numpy().reshape(x.shape[:-1] + (x.shape[-1] + pad,)), rt.keys_to_float(mm)[0]


def data(shape, seed=3):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


@pytest.mark.parametrize("shape", SHAPES)
def test_generic_identity_roundtrip(rt, shape):
    x = data(shape)
    y, mm = run(rt, x, [K.wrap_op(1.0)], pad=3)
    assert relerr(y[..., :shape[-1]], x) < TOL
    assert not y[..., shape[-1]:].any()
    assert abs(mm[0] - x.min()) < 1e-5 and abs(mm[1] - x.max()) < 1e-5


@pytest.mark.parametrize("shape", SHAPES[:2])
def test_generic_highpass_wrap_spike(rt, shape):
    """A program the band passes refuse (high-pass disk first), so it runs on the fallback."""
    x = data(shape)
    geo = K.geometry(shape[1:])
    idx = (shape[1] // 2 + 3, shape[2] // 2 - 5, shape[3] // 2 + 7)
    prog = [K.disk_op(6.0, True), K.spike_op(idx, geo, 9.0), K.wrap_op(0.5)]
    y, mm = run(rt, x, prog)
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x, 6.0, inside_off=True), idx, 9.0), 0.5)
    assert relerr(y, ref) < TOL
    assert abs(mm[0] - y.min()) < 1e-6 and abs(mm[1] - y.max()) < 1e-6


@pytest.mark.parametrize("shape", SHAPES)
def test_generic_lowpass_fallback_and_band(rt, shape, no_band):
    """Gibbs truncation on the fallback (band plans off), then a narrow one (alpha 0.85, a box the
    band passes take) with band plans on: the band passes need no factorisation."""
    x = data(shape)
    y, _ = run(rt, x, [K.gibbs_op(0.5, shape[1:])])
    assert relerr(y, O.gibbs_noise(x, 0.5)) < TOL
    rt.set_band_plans(True)
    yb, _ = run(rt, x, [K.gibbs_op(0.85, shape[1:])])
    assert relerr(yb, O.gibbs_noise(x, 0.85)) < TOL


@pytest.mark.parametrize("shape", SHAPES[:2])
def test_generic_logabs_sums(rt, shape):
    x = data(shape)
    xb = torch.from_numpy(x).cuda().reshape((1,) + shape)
    s = rt.logabs_sums(xb, 3, [[]], shape[0]).cpu().numpy()
    la = np.log(np.abs(O.shift_fourier(x, 3)) + np.float32(1e-10)).astype(np.float64)
    ref = la.reshape(shape[0], -1).sum(axis=1)
    assert np.allclose(s, ref, rtol=1e-5, atol=1e-3 * np.sqrt(la[0].size))
