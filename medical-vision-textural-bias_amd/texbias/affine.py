"""Host-side geometry of Spacingd / Orientationd (MONAI 0.5) as voxel-index affine maps.

The reference's BraTS Compose resamples every sample before cropping
(10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:156-161 and :183-190):

    Spacingd(keys=["image", "label"], pixdim=(1.5, 1.5, 2.0), mode=("bilinear", "nearest"))
    Orientationd(keys=["image", "label"], axcodes="RAS")

MONAI 0.5 implements them with nibabel's orientation helpers and a ``grid_sample`` resampler.
Neither library is installed here; their published algorithms are restated below (nibabel's
``io_orientation`` / ``axcodes2ornt`` / ``ornt_transform`` / ``apply_orientation``, MONAI's
``zoom_affine`` / ``compute_shape_offset`` / ``Spacing`` identity shortcut).  Every spatial step
of the chain -- spacing, orientation, the crop, the flips -- maps output voxel indices to input
voxel coordinates affinely, so the whole chain is composed here into ONE 3 x 4 map per sample and
the device gathers each output voxel once (``tb_brats_prep_f32`` with ``resample``).
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np

LABELS = (("L", "R"), ("P", "A"), ("I", "S"))


def zoom_affine(affine: np.ndarray, scale: Sequence[float]) -> np.ndarray:
    """MONAI 0.5 ``zoom_affine(affine, scale, diagonal=False)``: keep the rotation, set the voxel
    sizes to |scale| (signs from the Cholesky factor's diagonal); translation zero."""
    affine = np.array(affine, dtype=float, copy=True)
    d = len(affine) - 1
    s = np.array(scale, dtype=float, copy=True)
    if len(s) < d:
        s = np.append(s, np.ones(d - len(s)))
    s = s[:d]
    s[s == 0] = 1.0
    rzs = affine[:-1, :-1]
    zs = np.linalg.cholesky(rzs.T @ rzs).T
    rotation = rzs @ np.linalg.inv(zs)
    new = np.eye(len(affine))
    new[:-1, :-1] = rotation @ np.diag(np.sign(np.diag(zs)) * np.abs(s))
    return new


def io_orientation(affine: np.ndarray) -> np.ndarray:
    """nibabel ``io_orientation``: per voxel axis, (world axis, +1/-1) of its closest direction."""
    affine = np.asarray(affine, dtype=float)
    q, p = affine.shape[0] - 1, affine.shape[1] - 1
    rzs = affine[:q, :p]
    zooms = np.sqrt(np.sum(rzs * rzs, axis=0))
    zooms[zooms == 0] = 1
    rs = rzs / zooms
    P, S, Qs = np.linalg.svd(rs, full_matrices=False)
    tol = S.max() * max(rs.shape) * np.finfo(np.float64).eps
    keep = S > tol
    R = np.dot(P[:, keep], Qs[keep])
    ornt = np.full((p, 2), np.nan)
    for in_ax in range(p):
        col = R[:, in_ax]
        if not np.allclose(col, 0):
            out_ax = int(np.argmax(np.abs(col)))
            ornt[in_ax, 0] = out_ax
            ornt[in_ax, 1] = -1 if col[out_ax] < 0 else 1
            R[out_ax, :] = 0
    return ornt


def axcodes2ornt(axcodes: str, labels=LABELS) -> np.ndarray:
    """nibabel ``axcodes2ornt``: "RAS" -> [[0, 1], [1, 1], [2, 1]]."""
    ornt = np.full((len(axcodes), 2), np.nan)
    for code_idx, code in enumerate(axcodes):
        for label_idx, (lo, hi) in enumerate(labels):
            if code == lo:
                ornt[code_idx] = [label_idx, -1]
            elif code == hi:
                ornt[code_idx] = [label_idx, 1]
    if np.isnan(ornt).any():
        raise ValueError(f"axcodes {axcodes!r} not in {labels}")
    return ornt


def ornt_transform(start: np.ndarray, end: np.ndarray) -> np.ndarray:
    """nibabel ``ornt_transform``: the orientation taking ``start`` to ``end``."""
    start, end = np.asarray(start), np.asarray(end)
    result = np.empty_like(start)
    for end_in, (end_out, end_flip) in enumerate(end):
        for start_in, (start_out, start_flip) in enumerate(start):
            if end_out == start_out:
                result[start_in, :] = [end_in, 1 if start_flip == end_flip else -1]
                break
        else:
            raise ValueError(f"unable to take orientation {start.tolist()} to {end.tolist()}")
    return result


def compute_shape_offset(shape: Sequence[int], in_affine: np.ndarray, out_affine: np.ndarray):
    """MONAI 0.5 ``compute_shape_offset``: the output grid covering the input's corner voxels."""
    shp = np.array(shape, dtype=float)
    sr = len(shp)
    corners = np.asarray(np.meshgrid(*[(0.0, d - 1.0) for d in shp], indexing="ij")).reshape((sr, -1))
    corners = np.concatenate((corners, np.ones_like(corners[:1])))
    corners = in_affine @ corners
    corners_out = np.linalg.inv(out_affine) @ corners
    corners_out = corners_out[:-1] / corners_out[-1]
    out_shape = np.round(np.ptp(corners_out, axis=1) + 1.0)
    if np.allclose(io_orientation(in_affine), io_orientation(out_affine)):
        offset = in_affine @ ([0] * sr + [1])
        offset = offset[:-1] / offset[-1]
    else:
        c = corners[:-1] / corners[-1]
        offset = np.min(c, 1)
    return out_shape.astype(int), offset


def spacing_map(shape: Sequence[int], affine: np.ndarray, pixdim: Sequence[float]):
    """Spacing (MONAI 0.5 ``Spacing.__call__``): (4 x 4 map output index -> input coordinate,
    output shape, output affine).  A map within 1e-3 of the identity is the identity (MONAI copies
    the data unresampled)."""
    affine = np.asarray(affine, dtype=float)
    out_d = np.array(pixdim, dtype=float)[: len(shape)]
    if out_d.size < len(shape):
        out_d = np.append(out_d, [1.0] * (len(shape) - out_d.size))
    if np.any(out_d <= 0):
        raise ValueError(f"pixdim must be positive, got {tuple(out_d)}")
    new_affine = zoom_affine(affine, out_d)
    out_shape, offset = compute_shape_offset(shape, affine, new_affine)
    new_affine[: len(shape), -1] = offset[: len(shape)]
    T = np.linalg.inv(affine) @ new_affine
    if np.allclose(T, np.eye(len(T)), atol=1e-3):
        return np.eye(len(T)), tuple(int(v) for v in shape), affine
    return T, tuple(int(v) for v in out_shape), new_affine


def orientation_map(shape: Sequence[int], affine: np.ndarray, axcodes: str = "RAS"):
    """Orientation (MONAI 0.5 ``Orientation.__call__`` = nibabel ``apply_orientation``: flip the
    input axes with direction -1, then transpose by argsort of the target axes): (4 x 4 map
    oriented index -> pre-orientation index, oriented shape)."""
    sr = len(shape)
    src = io_orientation(affine)
    dst = axcodes2ornt(axcodes[:sr])
    ornt = ornt_transform(src, dst)
    O = np.zeros((sr + 1, sr + 1))
    O[sr, sr] = 1.0
    out_shape = [0] * sr
    for ax in range(sr):
        a = int(ornt[ax, 0])
        out_shape[a] = int(shape[ax])
        if ornt[ax, 1] == -1:
            O[ax, a] = -1.0
            O[ax, sr] = shape[ax] - 1.0
        else:
            O[ax, a] = 1.0
    return O, tuple(out_shape)


def crop_flip_map(corner: Sequence[int], roi: Sequence[int], flip_axes: Sequence[int]) -> np.ndarray:
    """Crop at ``corner`` then mirror ``flip_axes`` inside the window: output -> oriented index."""
    n = len(roi)
    M = np.eye(n + 1)
    for a in range(n):
        if a in flip_axes:
            M[a, a] = -1.0
            M[a, n] = corner[a] + roi[a] - 1.0
        else:
            M[a, n] = float(corner[a])
    return M


def center_corner(shape: Sequence[int], roi: Sequence[int]) -> Tuple[int, ...]:
    """MONAI 0.5 ``CenterSpatialCrop``: window centred at ``n // 2`` (start ``n // 2 - roi // 2``)."""
    return tuple(max(int(n) // 2 - int(r) // 2, 0) for n, r in zip(shape, roi))
