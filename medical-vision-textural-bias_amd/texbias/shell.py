"""Candidate points of the plane-wave ellipsoid shell (filters_and_operators.py:294-352).

``ellipsoid.binary_mask_3d`` marks 0.95 < (i-ci)^2/a^2 + (j-cj)^2/b^2 + (k-ck)^2/c^2 < 1.05
(float32 arithmetic, centre floor(n/2), int64 squares divided by the float radius squared) and
``sample_ellipsoid`` indexes ``mask.nonzero()`` (row-major) with ``R.randint(0, len)``.  The list
depends only on (shape, a, b, c); it is built once on the host and cached, so a sampled index
is bit-identical to the reference's for the same RandomState.
"""
from __future__ import annotations

from functools import lru_cache
from typing import Sequence

import numpy as np


@lru_cache(maxsize=64)
def _coords(shape3, a, b, c) -> np.ndarray:
    terms = []
    for n, r in zip(shape3, (a, b, c)):
        off = np.arange(n, dtype=np.int64) - (n // 2)
        terms.append((off * off).astype(np.float32) / np.float32(r * r))
    q = terms[0][:, None, None] + terms[1][None, :, None]
    q = q + terms[2][None, None, :]
    hit = np.logical_and(q > np.float32(0.95), q < np.float32(1.05))
    co = np.stack(np.nonzero(hit), axis=1).astype(np.int64)
    co.setflags(write=False)
    return co


def shell_coords(shape3: Sequence[int], a: float, b: float, c: float) -> np.ndarray:
    shape3 = tuple(int(s) for s in shape3)
    if len(shape3) != 3:
        raise ValueError("the ellipsoid shell lives on a 3-D grid")
    return _coords(shape3, float(a), float(b), float(c))
