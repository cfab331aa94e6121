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


RESAMPLE_CASES = [
    # (raw shape, affine, pixdim, roi, center crop)
    ((60, 54, 40), np.diag([-1.0, -1.0, 1.0, 1.0]), (1.5, 1.5, 2.0), (32, 32, 16), True),    # BraTS LPS -> RAS
    ((60, 54, 40), np.diag([-1.0, -1.0, 1.0, 1.0]), (1.5, 1.5, 2.0), (24, 32, 16), False),   # random crop + flips
    ((44, 50, 36), np.array([[0.0, -0.75, 0.0, 3.0], [1.0, 0.0, 0.0, -2.0], [0.0, 0.0, 1.25, 7.0],
                             [0.0, 0.0, 0.0, 1.0]]), (1.5, 1.5, 2.5), (16, 24, 16), True),  # permuted axes
]


@pytest.mark.parametrize("case", range(len(RESAMPLE_CASES)))
def test_prep_spacing_orientation_matches_oracle(gpu, case):
    """Spacingd(pixdim, bilinear/nearest) -> Orientationd(RAS) -> crop -> flip -> normalise -> scale
    -> shift as one affine gather on the GPU (texbias.affine + tb_brats_prep_f32 resample mode)
    against the step-by-step oracle: image 1e-5, label classes bit-exact (nearest, half to even)."""
    from texbias.prep import BratsPrep
    sp, aff, pixdim, roi, center = RESAMPLE_CASES[case]
    B, C = 2, 4
    img, lab = _raw(B, C, sp, 10 + case)
    prep = BratsPrep(roi_size=roi, pixdim=pixdim, axcodes="RAS", center_crop=center,
                     flip_axis=(0, 2), flip_prob=0.0 if center else 1.0, scale_prob=1.0,
                     shift_prob=1.0).set_random_state(case)
    affs = [aff, aff]
    M, shp = prep.spatial_map(sp, aff)
    params = prep.draw(B, sp, affs)
    x, y = prep(torch.from_numpy(img).cuda(), torch.from_numpy(lab).cuda(), params=params, affines=affs)
    for b, q in enumerate(params):
        G = np.array(list(q.m)).reshape(3, 4)
        # the crop corner the host drew: the map's translation at output voxel 0, back through M
        corner = np.rint(np.linalg.solve(M[:3, :3], G[:, 3] - M[:3, 3])).astype(int)
        if not center:   # flips (0, 2) drawn with prob 1: the corner is at the window's far end there
            corner[[0, 2]] -= np.array(roi)[[0, 2]] - 1
        xr, yr = PO.prep_resampled(img[b], lab[b], aff, pixdim, tuple(corner), roi,
                                   flip_axes=() if center else (0, 2), scale=q.scale, shift=q.shift)
        assert xr.shape == (C,) + roi
        np.testing.assert_allclose(x[b].cpu().numpy(), xr, rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(y[b].cpu().numpy(), yr)


def test_prep_spacing_identity_at_matching_pixdim(gpu):
    """A volume already at the target voxel size: Spacing is the identity (MONAI copies), so the
    resample path equals the crop-only path bit for bit."""
    from texbias.prep import BratsPrep
    B, C, sp, roi = 2, 4, (40, 36, 30), (32, 24, 16)
    img, lab = _raw(B, C, sp, 21)
    aff = np.diag([1.5, 1.5, 2.0, 1.0])
    rs = BratsPrep(roi_size=roi, pixdim=(1.5, 1.5, 2.0), axcodes="RAS", flip_prob=1.0).set_random_state(4)
    plain = BratsPrep(roi_size=roi, flip_prob=1.0).set_random_state(4)
    pr = rs.draw(B, sp, [aff, aff])
    pp = plain.draw(B, sp)
    assert all(q.resample == 1 for q in pr)
    xi, li = torch.from_numpy(img).cuda(), torch.from_numpy(lab).cuda()
    x1, y1 = rs(xi, li, params=pr)
    x2, y2 = plain(xi, li, params=pp)
    assert torch.equal(x1, x2) and torch.equal(y1, y2)


def test_brats_val_shapes(gpu):
    """The validation Compose's spatial part on a BraTS-sized raw volume (240 x 240 x 155 at 1 mm,
    LPS): Spacing (1.5, 1.5, 2.0) -> 160 x 160 x 78, RAS, CenterSpatialCrop 128 x 128 x 64."""
    from texbias.prep import BratsPrep
    prep = BratsPrep(pixdim=(1.5, 1.5, 2.0), axcodes="RAS", center_crop=True, flip_prob=0.0, scale_prob=0.0,
                     shift_prob=0.0)
    M, shp = prep.spatial_map((240, 240, 155), np.diag([-1.0, -1.0, 1.0, 1.0]))
    assert shp == (160, 160, 78)
    img, lab = _raw(1, 4, (240, 240, 155), 5)
    x, y = prep(torch.from_numpy(img).cuda(), torch.from_numpy(lab).cuda(), affines=[np.diag([-1.0, -1.0, 1.0, 1.0])])
    assert x.shape == (1, 4, 128, 128, 64) and y.shape == (1, 3, 128, 128, 64)
    xr, yr = PO.prep_resampled(img[0], lab[0], np.diag([-1.0, -1.0, 1.0, 1.0]), (1.5, 1.5, 2.0), (16, 16, 7),
                               (128, 128, 64))
    np.testing.assert_allclose(x[0].cpu().numpy(), xr, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(y[0].cpu().numpy(), yr)
