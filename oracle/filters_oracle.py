"""CPU oracle: a numpy restatement of the reference's k-space / spatial filters.

TEST INFRASTRUCTURE ONLY.  Imported by ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` -- as the CHECKER, never as the
thing measured or shipped.  The product path (``medical-vision-textural-bias_amd``)
never imports this module and fails loudly when its HIP library is missing.

Each function restates one reference function op for op, in the reference's
precision (complex64 spectra, float32 images; numpy >= 2 keeps single
precision through ``np.fft``), and cites the file:line it follows.  It is
pinned against fixtures produced by the reference itself
(``tests/golden/make_golden.py`` -> ``tests/golden/golden_*.npz``); see
``tests/test_oracle_golden.py``.

Conventions shared with the reference:
* spatial axes are the trailing ``n_dims`` axes; k-space is ``fftshift``-ed;
* ``.real`` after every inverse transform (G7 in SURVEY.md appendix A).
"""
from __future__ import annotations

from math import floor
from typing import Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "shift_fourier", "inv_shift_fourier", "disk_mask", "fourier_disk", "ellipsoid_shell",
    "ellipsoid_sample", "plane_waves", "wrap_artifact", "salt_and_pepper", "gibbs_mask",
    "gibbs_noise", "kspace_spike", "kspace_default_intensity", "gibbs_layer_mask", "gibbs_layer", "chain",
]


def _axes(n_dims: int) -> Tuple[int, ...]:
    return tuple(range(-n_dims, 0))


# filters_and_operators.py:594-632 (Fourier), dup. stylization_layers.py:16-52,
# inline copies filters_and_operators.py:263-279, 397-414, 517-537.
def shift_fourier(x: np.ndarray, n_dims: int) -> np.ndarray:
    ax = _axes(n_dims)
    return np.fft.fftshift(np.fft.fftn(np.asarray(x, np.float32), axes=ax), axes=ax).astype(np.complex64)


def inv_shift_fourier(k: np.ndarray, n_dims: int) -> np.ndarray:
    ax = _axes(n_dims)
    return np.fft.ifftn(np.fft.ifftshift(k, axes=ax), axes=ax).real.astype(np.float32)


# filters_and_operators.py:136-197 (disk_mask.binary_mask_2d / binary_mask_3d)
def disk_mask(shape: Sequence[int], r, dim: int, inside_off: bool) -> np.ndarray:
    """Binary disk/sphere on the last ``dim`` axes; centre floor(n/2); strict '<'.

    The reference compares an int64 sum of squares with ``r**2``: a Python
    float radius promotes the comparison to float32 (torch default dtype), an
    int radius keeps it integer (``:151-152, 184-187``)."""
    sp = shape[-dim:]
    s = np.zeros(sp, np.int64)
    for a, n in enumerate(sp):
        g = (np.arange(n, dtype=np.int64) - floor(n / 2)) ** 2
        s = s + g.reshape([-1 if i == a else 1 for i in range(dim)])
    if isinstance(r, (int, np.integer)) and not isinstance(r, bool):
        sel = s < int(r) ** 2
    else:
        sel = s.astype(np.float32) < np.float32(float(r) ** 2)
    m = sel.astype(np.float32)
    if inside_off:
        m = np.float32(1) - m
    return np.broadcast_to(m, tuple(shape)).astype(np.float32)


# filters_and_operators.py:236-252, 263-279 (RandFourierDiskMaskd.__call__, dim=3 hard-wired :248)
def fourier_disk(x: np.ndarray, r, inside_off: bool = False) -> np.ndarray:
    k = shift_fourier(x, 3)
    k = k * disk_mask(k.shape, r, 3, inside_off)
    return inv_shift_fourier(k.astype(np.complex64), 3)


# filters_and_operators.py:294-325 (ellipsoid.binary_mask_3d): shell 0.95 < q < 1.05 in float32
def ellipsoid_shell(shape3: Sequence[int], a: float, b: float, c: float) -> np.ndarray:
    """Row-major list of shell coordinates (what ``mask.nonzero()`` returns, :348)."""
    ax = [np.arange(n, dtype=np.int64) - floor(n / 2) for n in shape3]
    t = [np.float32(v * v) / np.float32(d * d) for v, d in zip(ax, (a, b, c))]
    q = (t[0][:, None, None] + t[1][None, :, None]) + t[2][None, None, :]
    sel = (q > np.float32(0.95)) & (q < np.float32(1.05))
    return np.argwhere(sel)


# filters_and_operators.py:342-352 (ellipsoid.sample_ellipsoid)
def ellipsoid_sample(coords: np.ndarray, rs: np.random.RandomState) -> Tuple[int, int, int]:
    i = rs.randint(0, len(coords))
    return tuple(int(v) for v in coords[i])


# filters_and_operators.py:370-414 (RandPlaneWaves_ellipsoid.__call__)
def plane_waves(x: np.ndarray, idx: Sequence[int], intensity: float,
                phase: Optional[np.ndarray] = None) -> np.ndarray:
    """Set log|k| = intensity at ``idx`` (all channels), keep phase, invert.

    ``phase`` (per channel) overrides ``angle(k[idx])`` -- the hook used when the
    coefficient is rounding noise (after a low-pass), where no two FFT
    implementations agree on its angle."""
    k = shift_fourier(x, 3)
    with np.errstate(divide="ignore"):
        la = np.log(np.abs(k)).astype(np.float32)     # no eps (:383)
    ph = np.angle(k).astype(np.float32)
    sl = (slice(None), idx[0], idx[1], idx[2])
    la[sl] = np.float32(intensity)
    if phase is not None:
        ph[sl] = np.asarray(phase, np.float32)
    k2 = (np.exp(la) * np.exp(1j * ph)).astype(np.complex64)
    return inv_shift_fourier(k2, 3)


def spikes_exact(x: np.ndarray, sets) -> np.ndarray:
    """The float64 exact result of a spike program: the same coefficient replacements as
    plane_waves / kspace_spike (:370-393, :966-983 -- |k| := exp(val) at each location, phase kept or
    overridden), in a float64 spectrum with every other coefficient left untouched (no float32 polar
    round trip).  ``sets``: (idx, val, phase) with idx spatial (all channels) or (c, h, w, d);
    phase None keeps angle(k).  The closed-form route's own target (it adds each spike's plane wave
    to x), to ~1e-15."""
    ax = _axes(3)
    k = np.fft.fftshift(np.fft.fftn(np.asarray(x, np.float64), axes=ax), axes=ax)
    for idx, val, phase in sets:
        sel = tuple(idx) if len(idx) == 4 else (slice(None),) + tuple(idx)
        ph = np.angle(k[sel]) if phase is None else np.float64(np.float32(phase))
        k[sel] = np.exp(np.float64(np.float32(val))) * np.exp(1j * ph)
    return np.fft.ifftn(np.fft.ifftshift(k, axes=ax), axes=ax).real


def polar_roundtrip(x: np.ndarray) -> np.ndarray:
    """The reference's float32 polar round trip of every coefficient with nothing changed
    (filters_and_operators.py:383-391: log|k|, angle, exp(log) * exp(i angle), inverse `.real`): its
    distance from x is the rounding floor of any plane-wave / spike output of that path (1.4e-5 of
    max|x| for a raw 240x240x155 volume; after a low-pass almost every coefficient is exactly 0)."""
    k = shift_fourier(x, 3)
    with np.errstate(divide="ignore"):
        la = np.log(np.abs(k)).astype(np.float32)
    ph = np.angle(k).astype(np.float32)
    return inv_shift_fourier((np.exp(la) * np.exp(1j * ph)).astype(np.complex64), 3)


# filters_and_operators.py:503-515 (WrapArtifact.__call__): odd shifted indices scaled by alpha per axis
def wrap_artifact(x: np.ndarray, alpha: float) -> np.ndarray:
    k = shift_fourier(x, 3)
    a = np.float32(alpha)
    k[:, 1::2, :, :] *= a
    k[:, :, 1::2, :] *= a
    k[:, :, :, 1::2] *= a
    return inv_shift_fourier(k, 3)


# filters_and_operators.py:465-482 (SaltAndPepper.salt_and_pepper); p clamp :444
def salt_and_pepper(x: np.ndarray, p: float, u: np.ndarray):
    """Returns (y, cls) with cls 0 keep / 1 pepper(MIN) / 2 salt(MAX), given u in [0,1)."""
    p = min(max(0.0, p), 1.0)
    x = np.asarray(x, np.float32)
    mx, mn = np.float32(x.max()) / np.float32(2), np.float32(x.min()) / np.float32(2)
    lo, hi = np.float32(p / 2), np.float32(p)
    cls = np.zeros(x.shape, np.int8)
    cls[u <= lo] = 1
    cls[(u > lo) & (u <= hi)] = 2
    y = x.copy()
    y[cls == 1] = mn
    y[cls == 2] = mx
    return y, cls


# filters_and_operators.py:678-705 (GibbsNoise._apply_mask): float64 geometry, centre (n-1)/2, '<='
def gibbs_mask(spatial: Sequence[int], alpha: float) -> np.ndarray:
    r = (1 - alpha) * np.max(spatial) * np.sqrt(2) / 2.0
    center = (np.array(spatial) - 1) / 2
    coords = np.ogrid[tuple(slice(0, i) for i in spatial)]
    d2 = sum((c - z) ** 2 for c, z in zip(coords, center))
    return np.sqrt(d2) <= r


# filters_and_operators.py:663-675 (GibbsNoise.__call__)
def gibbs_noise(x: np.ndarray, alpha: float) -> np.ndarray:
    n = x.ndim - 1
    k = shift_fourier(x, n)
    k = k * gibbs_mask(x.shape[1:], alpha)[None]
    return inv_shift_fourier(k.astype(np.complex64), n)


# filters_and_operators.py:906-945 (KSpaceSpikeNoise.__call__) + _set_spike :966-983
def kspace_spike(x: np.ndarray, loc, k_intensity=None) -> np.ndarray:
    """``loc``: one spatial tuple (all channels) or a sequence of full tuples.

    With ``k_intensity=None`` the per-CHANNEL default 2.5*mean(log|k|) (:933) is
    zipped against the LOCATIONS in order (:937), exactly as the reference does."""
    n = x.ndim - 1
    k = shift_fourier(x, n)
    la = np.log(np.abs(k) + np.float32(1e-10)).astype(np.float32)
    ph = np.angle(k).astype(np.float32)
    if k_intensity is None:
        k_intensity = kspace_default_intensity(x)
    multi = isinstance(loc[0], (tuple, list))
    locs = list(loc) if multi else [tuple(loc)]
    vals = list(k_intensity) if multi else [k_intensity]
    for idx, val in zip(locs, vals):
        idx = tuple(idx)
        if len(idx) == la.ndim:
            la[idx] = val
        else:
            if not np.isscalar(val) and np.ndim(val) != 0:
                raise TypeError("can't assign a tuple to a torch.FloatTensor")  # reference :981 failure
            la[(slice(None),) + idx] = val
    k2 = (np.exp(la) * np.exp(1j * ph)).astype(np.complex64)
    return inv_shift_fourier(k2, n)


# filters_and_operators.py:926-933 (default k_intensity) and :1125-1131 (default range centre)
def kspace_default_intensity(x: np.ndarray) -> tuple:
    n = x.ndim - 1
    la = np.log(np.abs(shift_fourier(x, n)) + np.float32(1e-10))
    return tuple(la.mean(axis=_axes(n), dtype=np.float64).astype(np.float32) * np.float32(2.5))


# stylization_layers.py:91-116 (GibbsNoiseLayer._apply_mask): float32 geometry, mask = !(d/(a*max d) > 1)
def gibbs_layer_mask(spatial: Sequence[int], alpha: float) -> np.ndarray:
    center = (np.array(spatial, np.float32) - np.float32(1)) / np.float32(2)
    grids = np.meshgrid(*[np.arange(n, dtype=np.float32) for n in spatial], indexing="ij")
    s = np.float32(0)
    for g, c in zip(grids, center):
        s = s + (g - c) ** 2
    dist = np.sqrt(s.astype(np.float32))
    an = np.float32(alpha) * dist.max()
    with np.errstate(divide="ignore", invalid="ignore"):
        nd = dist / an
    return ~(nd > 1)


def gibbs_layer(x: np.ndarray, alpha: float) -> np.ndarray:
    """stylization_layers.py:79-89: FFT over ALL non-batch axes (n_dims = x.ndim-1)."""
    n = x.ndim - 1
    k = shift_fourier(x, n)
    k = k * gibbs_layer_mask(x.shape[1:], alpha)[None]
    return inv_shift_fourier(k.astype(np.complex64), n)


def chain(x: np.ndarray, r, idx, intensity: float, alpha: float, p: float, u: np.ndarray,
          phase: Optional[np.ndarray] = None):
    """The drivers' chain (e.g. 127_.../..._3modalities.py:171-174):
    disk -> plane waves -> wrap -> salt & pepper.  Returns all stage outputs."""
    y1 = fourier_disk(x, r, False)
    y2 = plane_waves(y1, idx, intensity, phase)
    y3 = wrap_artifact(y2, alpha)
    y, cls = salt_and_pepper(y3, p, u)
    return y1, y2, y3, y, cls


# 50_reconstruction/reconGan/utils2.py:34-74 (RandZF): full spectrum, k[u <= p] = 0, inverse .real.
# The mask is given (``keep`` in the fftshift-ed layout of k); ``zf_keep_mask`` replays the device
# stream of TB_OP_ZF (include/texbias.h) for the parity tests.
def rand_zf(x: np.ndarray, keep: np.ndarray) -> np.ndarray:
    n = x.ndim - 1
    k = shift_fourier(x, n)
    k = np.where(keep, k, np.complex64(0)).astype(np.complex64)
    return inv_shift_fourier(k, n)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def zf_keep_mask(shape: Sequence[int], p: float, seed: int) -> np.ndarray:
    """bool [C, *spatial] in the fftshift-ed layout: coefficient kept iff u > p."""
    key = _splitmix64(np.array([seed], dtype=np.uint64))[0]
    idx = np.arange(int(np.prod(shape)), dtype=np.uint64).reshape(tuple(shape))  # unshifted frequencies
    u = (_splitmix64(idx ^ key) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    keep = u > np.float32(min(max(0.0, p), 1.0))
    return np.fft.fftshift(keep, axes=tuple(range(1, len(shape))))
