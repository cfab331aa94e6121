"""BraTS preprocessing, host side: the label-glue oracle against the reference's own output
(tests/golden/golden_labels.npz, bit-exact) and BratsPrep's per-sample draws (MONAI 0.5 order)."""
import numpy as np
import pytest

from _golden import load_cases
from oracle import prep_oracle as PO
from texbias.prep import BratsPrep


def test_convert_brats_classes_matches_reference():
    cases = load_cases("labels")
    assert len(cases) == 2
    for name, (meta, arr) in cases.items():
        np.testing.assert_array_equal(PO.convert_brats_classes(arr["label"]), arr["out"])


def test_draws_bounds_and_replay():
    p = BratsPrep(roi_size=(128, 128, 64)).set_random_state(5)
    a = p.draw(64, (160, 150, 78))
    assert all(0 <= q.h0 <= 32 and 0 <= q.w0 <= 22 and 0 <= q.d0 <= 14 for q in a)
    assert {q.flip for q in a} == {0, 1}
    sc = np.array([q.scale for q in a])
    assert np.all((sc == 1.0) | ((sc >= 0.9) & (sc <= 1.1))) and 0 < np.mean(sc != 1.0) < 1
    sh = np.array([q.shift for q in a])
    assert np.all(np.abs(sh) <= 0.1) and 0 < np.mean(sh != 0.0) < 1
    b = BratsPrep(roi_size=(128, 128, 64)).set_random_state(5).draw(64, (160, 150, 78))
    assert [bytes(q) for q in a] == [bytes(q) for q in b]
    # the crop corner follows MONAI 0.5: randint(0, n - roi + 1) per axis, on the crop's own stream
    rs = np.random.RandomState(5)
    assert (a[0].h0, a[0].w0, a[0].d0) == (rs.randint(0, 33), rs.randint(0, 23), rs.randint(0, 15))
    with pytest.raises(ValueError):
        p.draw(1, (100, 150, 78))


def test_oracle_prep_composition():
    rng = np.random.default_rng(0)
    img = rng.standard_normal((2, 12, 10, 8)).astype(np.float32)
    img[:, :3] = 0.0
    lab = rng.integers(0, 4, size=(12, 10, 8)).astype(np.float32)
    x, y = PO.prep(img, lab, (2, 1, 0), (8, 8, 6), flip_axes=(0,), scale=1.05, shift=-0.02)
    assert x.shape == (2, 8, 8, 6) and y.shape == (3, 8, 8, 6)
    c = PO.crop(img, (2, 1, 0), (8, 8, 6))[:, ::-1]
    nz = c[0] != 0
    ref = np.where(nz, (c[0] - c[0][nz].mean()) / c[0][nz].std(), 0) * np.float32(1.05) + np.float32(-0.02)
    np.testing.assert_allclose(x[0], ref, rtol=1e-5, atol=1e-6)


def _gather_with_map(vol, G, roi, nearest=False):
    """Numpy emulation of the device's resample gather: output voxel o samples vol at G[:, :3] o + G[:, 3]."""
    from oracle import prep_oracle as PO
    o = np.meshgrid(*[np.arange(n, dtype=np.float64) for n in roi], indexing="ij")
    c = [G[a, 0] * o[0] + G[a, 1] * o[1] + G[a, 2] * o[2] + G[a, 3] for a in range(3)]
    f = PO._nearest_border if nearest else PO._trilinear_border
    return np.stack([f(vol[k], *c) for k in range(vol.shape[0])])


@pytest.mark.parametrize("aff,pixdim,sp,roi,center", [
    (np.diag([-1.0, -1.0, 1.0, 1.0]), (1.5, 1.5, 2.0), (60, 54, 40), (32, 32, 16), True),
    (np.diag([-1.0, -1.0, 1.0, 1.0]), (1.5, 1.5, 2.0), (60, 54, 40), (24, 32, 16), False),
    (np.array([[0.0, -0.75, 0.0, 3.0], [1.0, 0.0, 0.0, -2.0], [0.0, 0.0, 1.25, 7.0], [0, 0, 0, 1.0]]),
     (1.5, 1.5, 2.5), (44, 50, 36), (16, 24, 16), True),
    (np.diag([1.0, 1.0, 1.0, 1.0]), (1.0, 1.0, 1.0), (20, 22, 18), (16, 16, 8), False),
])
def test_composed_affine_map_matches_stepwise_oracle(aff, pixdim, sp, roi, center):
    """texbias.affine's one-map composition of Spacing -> Orientation -> crop -> flip (host logic of
    tb_brats_prep_f32's resample mode) equals the oracle's step-by-step arrays (image 1e-6, labels exact)."""
    from oracle import prep_oracle as PO
    from texbias.prep import BratsPrep
    rng = np.random.default_rng(0)
    img = rng.standard_normal((2,) + sp).astype(np.float32)
    lab = rng.integers(0, 5, size=sp).astype(np.float32)
    prep = BratsPrep(roi_size=roi, pixdim=pixdim, axcodes="RAS", center_crop=center, flip_axis=(0, 2),
                     flip_prob=0.0 if center else 1.0).set_random_state(1)
    M, shp = prep.spatial_map(sp, aff)
    q = prep.draw(1, sp, [aff])[0]
    G = np.array(list(q.m), dtype=np.float64).reshape(3, 4)
    cf = np.linalg.solve(M[:3, :3], G[:, 3] - M[:3, 3])
    corner = np.rint(cf).astype(int)
    flips = () if center else (0, 2)
    for a in flips:
        corner[a] -= roi[a] - 1
    ref = PO.flip(PO.crop(PO.spacing_orientation(img, aff, pixdim), corner, roi), flips)
    got = _gather_with_map(img, G, roi)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6)
    lref = PO.flip(PO.crop(PO.spacing_orientation(lab[None], aff, pixdim, nearest=True), corner, roi), flips)
    np.testing.assert_array_equal(_gather_with_map(lab[None], G, roi, nearest=True), lref)
