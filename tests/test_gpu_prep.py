"""GPU BraTS preprocessing (tb_brats_prep_f32 via texbias.prep.BratsPrep) against the numpy oracle
(oracle/prep_oracle.py): crop + flips + NormalizeIntensity(nonzero, channel_wise) + scale + shift
within max|d| <= 1e-5 (float32, FMA-folded affine vs the step-by-step oracle; statistics in float64
vs numpy's float32 mean/std), label classes bit-exact (the label glue is pinned to the reference,
tests/test_prep_cpu.py); and the prepared batch fed through FusedChain."""
import numpy as np
import pytest
import torch

from oracle import prep_oracle as PO

pytestmark = pytest.mark.gpu


def _raw(B, C, sp, seed):
    rng = np.random.default_rng(seed)
    img = (rng.standard_normal((B, C) + sp) * 3.0 + 1.5).astype(np.float32)
    zz, yy, xx = np.meshgrid(*[np.linspace(-1, 1, n) for n in sp], indexing="ij")
    brain = (zz / 0.8) ** 2 + (yy / 0.9) ** 2 + (xx / 0.7) ** 2 < 1.0
    img *= brain[None, None]
    lab = (rng.integers(0, 5, size=(B,) + sp) * brain[None]).astype(np.float32)
    return img, lab


@pytest.mark.parametrize("flip_axes", [(), (0,), (1, 2), (0, 1, 2)])
def test_prep_matches_oracle(gpu, flip_axes):
    from texbias.prep import BratsPrep
    B, C, sp, roi = 3, 4, (40, 36, 30), (32, 24, 16)
    img, lab = _raw(B, C, sp, 1)
    img[1, 2] = 0.0                                   # an empty channel: no statistics, shift only
    img[2, 1][img[2, 1] != 0] = 2.5                   # a constant channel: std 0 -> divide by 1
    prep = BratsPrep(roi_size=roi, flip_axis=flip_axes if flip_axes else None, flip_prob=1.0, scale_prob=1.0,
                     shift_prob=1.0).set_random_state(3)
    params = prep.draw(B, sp)
    x, y = prep(torch.from_numpy(img).cuda(), torch.from_numpy(lab).cuda(), params=params)
    for b, q in enumerate(params):
        xr, yr = PO.prep(img[b], lab[b], (q.h0, q.w0, q.d0), roi, flip_axes=flip_axes, scale=q.scale, shift=q.shift)
        np.testing.assert_allclose(x[b].cpu().numpy(), xr, rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(y[b].cpu().numpy(), yr)


def test_prep_draws_and_no_label(gpu):
    from texbias.prep import BratsPrep
    B, C, sp, roi = 4, 4, (48, 40, 36), (32, 32, 16)
    img, _ = _raw(B, C, sp, 2)
    prep = BratsPrep(roi_size=roi).set_random_state(11)
    params = prep.draw(B, sp)
    x, y = prep(torch.from_numpy(img).cuda(), None, params=params)
    assert y is None and x.shape == (B, C) + roi
    for b, q in enumerate(params):
        axes = (0,) if q.flip else ()
        xr, _ = PO.prep(img[b], None, (q.h0, q.w0, q.d0), roi, flip_axes=axes,
                        scale=q.scale if q.scale != 1.0 else None, shift=q.shift if q.shift != 0.0 else None)
        np.testing.assert_allclose(x[b].cpu().numpy(), xr, rtol=1e-5, atol=1e-5)


def test_prep_feeds_fused_chain(gpu):
    """The reference's training input: raw -> prep (128x128x64 crops) -> the C3 filter chain."""
    from texbias.pipeline import reference_c3_chain
    from texbias.prep import BratsPrep
    B, C, sp = 2, 4, (160, 150, 78)
    img, lab = _raw(B, C, sp, 3)
    prep = BratsPrep().set_random_state(0)
    x, y = prep(torch.from_numpy(img).cuda(), torch.from_numpy(lab).cuda())
    assert x.shape == (B, C, 128, 128, 64) and y.shape == (B, 3, 128, 128, 64)
    chain, _ = reference_c3_chain(0)
    out = chain(x)
    assert out.shape == x.shape and torch.isfinite(out).all()
