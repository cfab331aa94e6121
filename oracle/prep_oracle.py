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
