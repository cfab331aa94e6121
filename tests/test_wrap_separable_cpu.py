"""CPU check of the separable wrap decomposition the GPU route uses (csrc/wrap.h): WrapArtifact's mask
(filters_and_operators.py:503-515) factors into symmetric 1-D masks, so the filter is a 2-tap roll
combine on even axes and a real circulant k = delta + (alpha - 1) q on odd axes.  Restated here in
float64 numpy and checked against the reference's golden wrap fixtures (1e-5) and the oracle."""
import numpy as np
import pytest

from _golden import load_cases, relerr
from oracle import filters_oracle as O


def q_table(n):
    f = np.arange(n)
    odd = ((f + n // 2) % n) & 1
    j = np.arange(n)
    return (odd[None, :] * np.cos(2 * np.pi * ((j[:, None] * f[None, :]) % n) / n)).sum(1) / n


def axis_filter(x, axis, alpha):
    n = x.shape[axis]
    if n % 2 == 0:
        s = -1.0 if (n // 2) % 2 else 1.0
        return 0.5 * (1 + alpha) * x + s * 0.5 * (1 - alpha) * np.roll(x, n // 2, axis=axis)
    k = (np.arange(n) == 0).astype(np.float64) + (alpha - 1.0) * q_table(n)
    K = k[(np.arange(n)[:, None] - np.arange(n)[None, :]) % n]  # y[o] = sum_i k[o - i] x[i]
    return np.moveaxis(np.tensordot(K, np.moveaxis(x, axis, 0), axes=(1, 0)), 0, axis)


def separable_wrap(x, alpha):
    y = np.asarray(x, np.float64)
    for ax in range(1, y.ndim):
        y = axis_filter(y, ax, alpha)
    return y


@pytest.mark.parametrize("name,case", sorted(load_cases("wrap").items()))
def test_separable_matches_golden(name, case):
    meta, a = case
    assert relerr(separable_wrap(a["x"], meta["alpha"]), a["y"]) < 1e-5


@pytest.mark.parametrize("shape", [(2, 8, 6, 7), (1, 4, 10, 9), (3, 6, 6, 6), (2, 12, 14, 15)])
@pytest.mark.parametrize("alpha", [0.0, 0.3, 0.75, 1.0])
def test_separable_matches_oracle(shape, alpha):
    x = np.random.default_rng(1).standard_normal(shape).astype(np.float32)
    assert relerr(separable_wrap(x, alpha), O.wrap_artifact(x, alpha)) < 1e-5


def test_circulant_is_real_symmetric():
    for n in (7, 15, 155):
        k = (np.arange(n) == 0) + (0.5 - 1.0) * q_table(n)
        np.testing.assert_allclose(k[1:], k[1:][::-1], atol=1e-15)
