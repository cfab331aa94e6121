"""CPU oracle, second form: the reference's filter chain in torch CPU ops (its real arithmetic).

TEST / BASELINE INFRASTRUCTURE ONLY.  Imported by ``tests/`` and the ``cpu_baseline`` leg of
``bench.py`` (through ``oracle/cpu_bench.py``) -- the reference's CPU filter path, timed beside the
HIP kernels; never imported by the product package.

``filters_oracle.py`` restates the reference in numpy (for parity); this module restates the same
transforms with the torch calls the reference makes on CPU tensors (``torch.fft.fftn`` over the
three trailing axes, ``fftshift``, float32 masks built per call, ``abs().log()`` / ``angle()`` /
``exp`` for the spike, ``torch.rand`` for salt-and-pepper), so that its timing is the reference's
per-volume CPU cost -- including the per-call mask construction the reference does.

  disk       RandFourierDiskMaskd.__call__  source_code/filters_and_operators.py:236-252, mask :165-197
  planes     RandPlaneWaves_ellipsoid.__call__  :370-393, ellipsoid mask / sampling :294-352
  wrap       WrapArtifact.__call__  :503-515 (Fourier helpers :517-537)
  sap        SaltAndPepper.salt_and_pepper  :465-482 (p clamp :444)
"""
from __future__ import annotations

from math import floor
from typing import Sequence, Tuple

import numpy as np
import torch

_AX = (-3, -2, -1)


def _fwd(x: torch.Tensor) -> torch.Tensor:
    return torch.fft.fftshift(torch.fft.fftn(x, dim=_AX), dim=_AX)


def _inv(k: torch.Tensor) -> torch.Tensor:
    return torch.fft.ifftn(torch.fft.ifftshift(k, dim=_AX), dim=_AX, norm="backward")


def _centred_sq(n: int) -> torch.Tensor:
    return (torch.arange(0, n) - floor(n / 2)) ** 2


def disk_mask(shape: Sequence[int], r, inside_off: bool = False) -> torch.Tensor:
    """float32 0/1 mask of k's full shape; int64 squared distances compared with r**2 (:184-187)."""
    D, H, W = shape[-3:]
    sel = (_centred_sq(D)[:, None, None] + _centred_sq(H)[None, :, None] + _centred_sq(W)[None, None, :]) < r ** 2
    m = torch.zeros(tuple(shape)).reshape(-1, D, H, W)
    m[sel.unsqueeze(0).repeat_interleave(m.size(0), 0)] = 1
    if inside_off:
        m = 1 - m
    return m.reshape(tuple(shape))


def disk(x: torch.Tensor, r, inside_off: bool = False) -> torch.Tensor:
    k = _fwd(x)
    return _inv(k * disk_mask(k.shape, r, inside_off)).real


def ellipsoid_coords(shape: Sequence[int], a: float, b: float, c: float) -> torch.Tensor:
    """Shell 0.95 < q < 1.05 of the ellipsoid around the centre, as ``nonzero()`` coordinates of the
    float32 mask the reference builds for every call (:294-325, :347-348)."""
    D, H, W = shape[-3:]
    q = (_centred_sq(D)[:, None, None] / a ** 2 + _centred_sq(H)[None, :, None] / b ** 2
         + _centred_sq(W)[None, None, :] / c ** 2)
    sel = torch.logical_and(q > .95, q < 1.05)
    m = torch.zeros(tuple(shape)).reshape(-1, D, H, W)
    m[sel.unsqueeze(0).repeat_interleave(m.size(0), 0)] = 1
    return m.reshape(tuple(shape)).nonzero()


def planes(x: torch.Tensor, a: float, b: float, c: float, intensity: float,
           rs: np.random.RandomState) -> Tuple[torch.Tensor, Tuple[int, int, int]]:
    """log|k| := intensity at one sampled shell point in every channel, phase kept (:381-392)."""
    k = _fwd(x)
    la = k.abs().log()
    ang = k.angle()
    coords = ellipsoid_coords(la[0].shape, a, b, c)
    idx = tuple(int(v) for v in coords[rs.randint(0, len(coords))].numpy())
    la[:, idx[0], idx[1], idx[2]] = intensity
    return _inv(la.exp() * torch.exp(1j * ang)).real, idx


def wrap(x: torch.Tensor, alpha: float) -> torch.Tensor:
    """Every odd index of the shifted spectrum scaled by alpha, once per axis (:509-511)."""
    k = _fwd(x)
    for ax in (1, 2, 3):
        sl = [slice(None)] * 4
        sl[ax] = slice(1, k.size(ax), 2)
        k[tuple(sl)] = k[tuple(sl)] * alpha
    return _inv(k).real


def sap(x: torch.Tensor, p: float, gen: torch.Generator = None) -> torch.Tensor:
    p = min(max(0, p), 1.)
    u = torch.rand(x.size(), generator=gen)
    x = x.clone()
    mx, mn = x.max() / 2, x.min() / 2
    x[u <= p / 2] = mn
    x[torch.logical_and(u > p / 2, u <= p)] = mx
    keep = torch.logical_and(u > p, u != 1.)
    x[keep] = x[keep]
    return x


def chain_c3(x: torch.Tensor, rs: np.random.RandomState, gen: torch.Generator = None) -> torch.Tensor:
    """C3: disk(12.5) -> planes(55, 55, 30, I=15) -> wrap(0.5) -> S&P(0.05)
    (10_scripts/127_.../..._3modalities.py:171-174)."""
    y = disk(x, 12.5)
    y, _ = planes(y, 55.0, 55.0, 30.0, 15.0, rs)
    y = wrap(y, 0.5)
    return sap(y, 0.05, gen)


def chain_c2(x: torch.Tensor, rs: np.random.RandomState = None, gen: torch.Generator = None) -> torch.Tensor:
    """C2: Gibbs truncation only -- RandFourierDiskMaskd(r=12.5)."""
    return disk(x, 12.5)
