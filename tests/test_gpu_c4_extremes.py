"""GPU parity of ``FusedChain`` at full C3 size (2 x 4 x 240 x 240 x 155, pad 5) for the extremes of
bench.py's ``--random-filters`` draws (BASELINE config 4, bench.py ``randomize_filters``):
r ~ U(10, 25.1), plane-wave I ~ U(10, 17), wrap alpha in {0, .25, .5, .75}, S&P p ~ U(.05, .35).

The chain is the reference's (10_scripts/127_.../..._3modalities.py:171-174; the random-parameter
drivers, e.g. 10_scripts/20_Gibbs_filters/stylized_gibbs10-25.py, draw r per worker).  r = 25.1
gives a pass-A' box of NDk 26 / KW 25 and the two-tile (VT = 2) pass C'; alpha = 0 zeroes every
coefficient with an odd shifted index.  Checked per case: every (sample, channel) pair against
the numpy oracle (one oracle pass per sample) with the phase hook, the S&P class map from an explicit u (bit-exact), the pass-C'
per-sample min/max, and that the band passes (k_band_fwd / k_band_inv) are the ones that ran.

Tolerances: filtered values max|y - y_ref| / max|y_ref| <= 1e-5 (north_star); class map exact.
"""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5
PAD = 5
SPATIAL = (240, 240, 155)

# (r, I, wrap alpha, p): every extreme of each draw appears at least once
CASES = [
    (10.0, 10.0, 0.0, 0.05),
    (25.1, 17.0, 0.75, 0.35),
    (25.1, 10.0, 0.0, 0.35),
    (10.0, 17.0, 0.75, 0.05),
]


@pytest.fixture(scope="module")
def env(gpu):
    import filters_and_operators as F
    from texbias import runtime as rt
    from texbias.pipeline import FusedChain
    return F, rt, FusedChain


@pytest.mark.parametrize("r,I,alpha,p", CASES)
def test_random_filter_extremes_full_c3(env, r, I, alpha, p, heartbeat):
    F, rt, FusedChain = env
    torch.manual_seed(11)
    B, C = 2, 4
    x = torch.randn((B, C) + SPATIAL, device="cuda")
    disk = F.RandFourierDiskMaskd(keys="image", r=12.5, inside_off=False, prob=1.0)
    planes = F.RandPlaneWaves_ellipsoid("image", 55.0, 55.0, 30.0, intensity_value=15.0, prob=1.0)
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.05)
    for j, t in enumerate((disk, planes, sap)):
        t.set_random_state(20 + j)
    planes.ellipsoid.set_random_state(27)
    # exactly what bench.py's randomize_filters() sets
    disk.r = float(r)
    planes.intensity_value = float(I)
    wrap.transform.alpha = float(alpha)
    sap.p = float(p)
    chain = FusedChain([disk, planes, wrap, sap])
    phases = [[0.3 - 0.2 * (b * C + c) for c in range(C)] for b in range(B)]
    idx = []
    plans = []
    for b in range(B):   # one sample at a time, so the ellipsoid draw of each is recorded
        plans += chain.plan(1, SPATIAL, [phases[b]])
        idx.append(tuple(planes.idx))
    u = torch.rand((B, C) + SPATIAL, device="cuda")
    cls = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    rt.set_pass_timing(True)
    y = chain(x, pad=PAD, plans=plans, u=u, cls=cls)
    torch.cuda.synchronize()
    _, cnt, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    assert "band_fwd" in names[0] and "band_inv" in names[2], names
    assert y.shape == (B, C, 240, 240, 160) and torch.all(y[..., 155:] == 0)
    mm = chain.last_minmax
    yh, ch, uh = y[..., :155].cpu().numpy(), cls.cpu().numpy(), u.cpu().numpy()
    for b in range(B):   # one oracle pass per sample, every channel checked
        ref3 = O.wrap_artifact(O.plane_waves(O.fourier_disk(x[b].cpu().numpy(), float(r)), idx[b], float(I),
                                             phase=np.float32(phases[b])), float(alpha))
        np.testing.assert_allclose(mm[b], [ref3.min(), ref3.max()], rtol=0, atol=1e-5 * np.abs(ref3).max())
        for c in range(C):
            _, cref = O.salt_and_pepper(ref3[c][None], float(p), uh[b, c][None])
            np.testing.assert_array_equal(ch[b, c], cref[0])
            # S&P values are the sample's (all-channel) min/max halves
            zc = ref3[c].copy()
            zc[cref[0] == 1] = np.float32(mm[b][0]) / 2
            zc[cref[0] == 2] = np.float32(mm[b][1]) / 2
            assert relerr(yh[b, c], zc) < TOL, (b, c)
