"""CPU oracle of the BraTS preprocessing the reference runs before its texture filters.

TEST INFRASTRUCTURE ONLY (imported by ``tests/``): the checker of ``tb_brats_prep_f32``.

Driver call site: 10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:151-170.

* ``convert_brats_classes`` restates ConvertToMultiChannelBasedOnBratsClassesd
  (source_code/filters_and_operators.py:61-87) -- **pinned** by tests/golden/golden_labels.npz,
  produced by the reference's own class.
* The MONAI 0.5 transforms (RandSpatialCropd, RandFlipd, NormalizeIntensityd(nonzero=True,
  channel_wise=True), RandScaleIntensityd, RandShiftIntensityd) are restated from MONAI 0.5's
  published semantics: slice at a corner drawn ``randint(0, n - roi + 1)`` per axis; ``np.flip``
  of each channel along the spatial axis; ``(x - mean) / std`` over the nonzero voxels of each
  channel (float32 ``np.mean`` / ``np.std``, std 0 -> 1); ``x * (1 + factor)``; ``x + offset``.
  MONAI is not installed here, so these are **parity unpinned** (no reference output to pin them).
* ``spacing_orientation`` restates Spacingd(pixdim, mode=("bilinear", "nearest")) ->
  Orientationd(axcodes="RAS") (…3modalities.py:156-161) step by step on arrays, for voxel-to-world
  affines that are signed, scaled axis permutations (the BraTS case): the Spacing grid has
  ``round((n - 1) |zoom| / pixdim + 1)`` voxels per axis and samples the input at
  ``o * pixdim / |zoom|`` (trilinear image, nearest label rounding half to even, border clamp --
  grid_sample's modes; a map within 1e-3 of the identity copies the data), then the axes are
  flipped where the affine points away from R/A/S and transposed into (R, A, S) order.  Written
  independently of the product's composed-affine host code (texbias/affine.py); **parity unpinned**
  (MONAI and nibabel are absent).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np


def convert_brats_classes(lab: np.ndarray) -> np.ndarray:
    """label map -> [TC, WT, ET] float32 (filters_and_operators.py:76-86)."""
    tc = np.logical_or(lab == 2, lab == 3)
    wt = np.logical_or(tc, lab == 1)
    et = lab == 2
    return np.stack([tc, wt, et], axis=0).astype(np.float32)


def crop(x: np.ndarray, corner: Sequence[int], roi: Sequence[int]) -> np.ndarray:
    """[C, *spatial] -> [C, *roi] at ``corner`` (MONAI 0.5 RandSpatialCrop with random_center)."""
    sl = (slice(None),) + tuple(slice(c, c + r) for c, r in zip(corner, roi))
    return x[sl]


def flip(x: np.ndarray, axes: Sequence[int]) -> np.ndarray:
    """Flip spatial axes (MONAI Flip: np.flip of every channel)."""
    for a in axes:
        x = np.flip(x, axis=1 + a)
    return np.ascontiguousarray(x)


def normalize_nonzero_channelwise(x: np.ndarray) -> np.ndarray:
    out = np.array(x, dtype=np.float32, copy=True)
    for c in range(out.shape[0]):
        ch = out[c]
        sl = ch != 0
        if not np.any(sl):
            continue
        mean = np.mean(ch[sl])
        std = np.std(ch[sl])
        if std == 0.0:
            std = 1.0
        ch[sl] = (ch[sl] - mean) / std
    return out.astype(np.float32)


def prep(img: np.ndarray, lab: Optional[np.ndarray], corner, roi, flip_axes=(), scale: Optional[float] = None,
         shift: Optional[float] = None, normalize: bool = True) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """The driver's order: labels to classes, crop, flip, normalise, scale, shift."""
    x = flip(crop(img, corner, roi), flip_axes)
    if normalize:
        x = normalize_nonzero_channelwise(x)
    if scale is not None:
        x = (x * np.float32(scale)).astype(np.float32)
    if shift is not None:
        x = (x + np.float32(shift)).astype(np.float32)
    y = None
    if lab is not None:
        y = flip(crop(convert_brats_classes(lab), corner, roi), flip_axes)
    return x, y


def _trilinear_border(v: np.ndarray, cx, cy, cz) -> np.ndarray:
    """v [H, W, D]; coordinate grids (float64) -> float32 samples, border clamp."""
    out = []
    idx = []
    for c, n in zip((cx, cy, cz), v.shape):
        c = np.clip(c, 0.0, n - 1.0)
        i0 = np.floor(c).astype(np.int64)
        i1 = np.minimum(i0 + 1, n - 1)
        idx.append((i0, i1, (c - i0).astype(np.float64)))
    (x0, x1, fx), (y0, y1, fy), (z0, z1, fz) = idx
    vv = v.astype(np.float64)
    c00 = vv[x0, y0, z0] * (1 - fz) + vv[x0, y0, z1] * fz
    c01 = vv[x0, y1, z0] * (1 - fz) + vv[x0, y1, z1] * fz
    c10 = vv[x1, y0, z0] * (1 - fz) + vv[x1, y0, z1] * fz
    c11 = vv[x1, y1, z0] * (1 - fz) + vv[x1, y1, z1] * fz
    c0 = c00 * (1 - fy) + c01 * fy
    c1 = c10 * (1 - fy) + c11 * fy
    out = c0 * (1 - fx) + c1 * fx
    return out.astype(np.float32)


def _nearest_border(v: np.ndarray, cx, cy, cz) -> np.ndarray:
    ii = [np.clip(np.rint(c).astype(np.int64), 0, n - 1) for c, n in zip((cx, cy, cz), v.shape)]
    return v[ii[0], ii[1], ii[2]]


def spacing_orientation(x: np.ndarray, affine: np.ndarray, pixdim: Sequence[float], nearest: bool = False,
                        ras: bool = True) -> np.ndarray:
    """[C, H, W, D] -> Spacing(pixdim) then Orientation("RAS") for a signed, scaled axis-permutation
    affine (each voxel axis along one world axis)."""
    R = np.asarray(affine, dtype=np.float64)[:3, :3]
    zoom = np.sqrt((R * R).sum(axis=0))              # voxel size of each voxel axis
    ratio = np.asarray(pixdim, dtype=np.float64) / zoom
    shape = x.shape[1:]
    if np.allclose(ratio, 1.0, atol=1e-3):
        y = x.copy()
    else:
        out = [int(np.round((n - 1) / r + 1.0)) for n, r in zip(shape, ratio)]
        g = np.meshgrid(*[np.arange(n, dtype=np.float64) * r for n, r in zip(out, ratio)], indexing="ij")
        f = _nearest_border if nearest else _trilinear_border
        y = np.stack([f(x[c], *g) for c in range(x.shape[0])])
    if not ras:
        return y
    world = np.argmax(np.abs(R), axis=0)             # world axis of each voxel axis
    sign = np.sign(R[world, np.arange(3)])
    for ax in range(3):
        if sign[ax] < 0:
            y = np.flip(y, axis=1 + ax)
    perm = [int(np.nonzero(world == a)[0][0]) for a in range(3)]   # output axis a <- voxel axis
    return np.ascontiguousarray(y.transpose([0] + [1 + p for p in perm]))


def prep_resampled(img: np.ndarray, lab: Optional[np.ndarray], affine: np.ndarray, pixdim, corner, roi,
                   flip_axes=(), scale: Optional[float] = None, shift: Optional[float] = None,
                   normalize: bool = True):
    """Validation/training order of the drivers: labels to classes, Spacingd, Orientationd, crop,
    flip, normalise, scale, shift (…3modalities.py:151-170, :179-190)."""
    x = spacing_orientation(img, affine, pixdim)
    x = flip(crop(x, corner, roi), flip_axes)
    if normalize:
        x = normalize_nonzero_channelwise(x)
    if scale is not None:
        x = (x * np.float32(scale)).astype(np.float32)
    if shift is not None:
        x = (x + np.float32(shift)).astype(np.float32)
    y = None
    if lab is not None:
        y = spacing_orientation(convert_brats_classes(lab), affine, pixdim, nearest=True)
        y = flip(crop(y, corner, roi), flip_axes)
    return x, y
