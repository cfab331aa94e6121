"""Host-side construction of k-space op programs (the parameters of tb_kspace_filter_f32).

Everything the reference computes from Python scalars before touching the
spectrum is evaluated here once per call, in the reference's own precision, so
that the device only does integer / float32 compares that are bit-identical to
the reference's masks:

* disk_mask (filters_and_operators.py:145-152, 176-187): int64 sum of squares vs
  ``r**2`` -- float32 compare for a float radius, int64 for an int radius;
* GibbsNoise._apply_mask (:686-698): float64 ``sqrt(d2) <= r`` turned into an
  exact integer threshold on ``4*d2``;
* GibbsNoiseLayer._apply_mask (stylization_layers.py:99-109): float32
  ``alpha * max(dist)``;
* spikes: the reference's fftshift-ed index -> unshifted frequency; the
  magnitude ``exp(intensity)`` as torch computes it in float32.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._abi import (TB_MAX_OPS, TB_OP_DISK, TB_OP_GIBBS, TB_OP_LAYER, TB_OP_SPIKE, TB_OP_WRAP, TB_OP_ZF, TbOp)


@dataclass(frozen=True)
class Geometry:
    """Mapping of a tensor's spatial axes onto the library's (H, W, D).

    ``spatial``: the reference's spatial shape (all transformed axes, size-1
    included).  ``kept``: indices (into ``spatial``) of the non-trivial axes;
    they become (H, W, D) = (k0, k1, k2), (k0, 1, k1) or (1, 1, k0).
    """

    spatial: Tuple[int, ...]
    kept: Tuple[int, ...]

    @property
    def hwd(self) -> Tuple[int, int, int]:
        n = [self.spatial[i] for i in self.kept]
        if len(n) == 3:
            return n[0], n[1], n[2]
        if len(n) == 2:
            return n[0], 1, n[1]
        if len(n) == 1:
            return 1, 1, n[0]
        return 1, 1, 1

    @property
    def numel(self) -> int:
        return int(np.prod(self.spatial))

    def to_hwd(self, per_axis: Sequence[int]) -> Tuple[int, int, int]:
        """Map a per-spatial-axis tuple (e.g. an unshifted frequency) to (h, w, d)."""
        v = [int(per_axis[i]) for i in self.kept]
        if len(v) == 3:
            return v[0], v[1], v[2]
        if len(v) == 2:
            return v[0], 0, v[1]
        if len(v) == 1:
            return 0, 0, v[0]
        return 0, 0, 0


def geometry(spatial: Sequence[int]) -> Geometry:
    spatial = tuple(int(s) for s in spatial)
    if any(s < 1 for s in spatial):
        raise ValueError(f"empty spatial shape {spatial}")
    kept = tuple(i for i, s in enumerate(spatial) if s > 1)
    if len(kept) > 3:
        raise ValueError(f"at most 3 non-singleton transformed axes are supported, got shape {spatial}")
    return Geometry(spatial, kept)


def _op(kind: int, chan: int = -1) -> TbOp:
    op = TbOp()
    op.kind = kind
    op.chan = chan
    return op


# --------------------------------------------------------------------- disk
def disk_op(r, inside_off: bool) -> TbOp:
    """RandFourierDiskMaskd / disk_mask (filters_and_operators.py:111-206)."""
    op = _op(TB_OP_DISK)
    if isinstance(r, (int, np.integer)) and not isinstance(r, bool):
        op.i[0] = 1
        op.l = int(r) * int(r)
    else:
        op.i[0] = 0
        r2 = float(r) ** 2
        op.f[0] = np.float32(r2) if math.isfinite(r2) else np.float32(np.inf)
    op.i[1] = 1 if inside_off else 0
    return op


# -------------------------------------------------------------------- Gibbs
def gibbs_threshold4(spatial: Sequence[int], alpha: float) -> int:
    """Largest integer t with fl64(sqrt(t/4)) <= r, r = (1-alpha)*max(shape)*sqrt(2)/2.

    The reference's mask is ``sqrt(d2) <= r`` in float64 with d2 = sum (i-(n-1)/2)^2
    (a quarter-integer, exact); so d2 is in the mask iff 4*d2 <= t."""
    r = (1 - alpha) * np.max(spatial) * np.sqrt(2) / 2.0
    if not r >= 0:  # r < 0 or NaN: nothing is inside
        return -1
    hi = int(sum((n - 1) ** 2 for n in spatial))  # max possible 4*d2
    if np.sqrt(hi / 4.0) <= r:
        return hi
    lo = -1  # invariant: sqrt(lo/4) <= r (lo=-1 sentinel), sqrt(hi/4) > r
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if np.sqrt(np.float64(mid) / 4.0) <= r:
            lo = mid
        else:
            hi = mid
    return lo


def gibbs_op(alpha: float, spatial: Sequence[int]) -> TbOp:
    """GibbsNoise._apply_mask (filters_and_operators.py:678-705); alpha in [0,1] asserted by the caller."""
    op = _op(TB_OP_GIBBS)
    op.l = gibbs_threshold4(spatial, alpha)
    return op


def layer_alpha_norm(alpha: float, spatial: Sequence[int]) -> np.float32:
    """alpha * max(dist) in float32 (stylization_layers.py:101-106); max dist is the corner."""
    s = np.float32(0)
    for n in spatial:
        c = (np.float32(n) - np.float32(1)) / np.float32(2)
        s = np.float32(s + c * c)
    return np.float32(np.float32(alpha) * np.sqrt(np.float32(s)))


def layer_op(alpha: float, spatial: Sequence[int], alpha_ptr: int = 0) -> TbOp:
    """GibbsNoiseLayer mask.  With ``alpha_ptr`` (device address of a float32 alpha) the kernel
    reads alpha itself, so a layer whose alpha lives on the device never syncs the host."""
    op = _op(TB_OP_LAYER)
    if alpha_ptr:
        op.l = int(alpha_ptr)
        op.f[1] = layer_alpha_norm(1.0, spatial)   # = max dist
    else:
        op.f[0] = layer_alpha_norm(alpha, spatial)
    return op


# --------------------------------------------------------------------- wrap
def wrap_op(alpha: float) -> TbOp:
    """WrapArtifact (filters_and_operators.py:509-511)."""
    op = _op(TB_OP_WRAP)
    op.f[0] = np.float32(alpha)
    return op


# ---------------------------------------------------------------------- ZF
_M64 = (1 << 64) - 1


def splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def zf_op(p: float, seed: int, spatial3: Sequence[int]) -> TbOp:
    """RandZF (50_reconstruction/reconGan/utils2.py:34-74): each k-space coefficient zeroed with
    probability p (u <= p), u from a counter-based hash of (seed, channel, frequency) -- see
    TB_OP_ZF in include/texbias.h.  ``spatial3`` = the (H, W, D) geometry of the transform."""
    op = _op(TB_OP_ZF)
    op.f[0] = np.float32(min(max(0.0, float(p)), 1.0))
    op.i[1], op.i[2] = int(spatial3[1]), int(spatial3[2])
    k = splitmix64(int(seed) & _M64)
    op.l = k - (1 << 64) if k >= (1 << 63) else k   # int64 field, same bits
    return op


# ------------------------------------------------------------------- spikes
def unshift(idx: Sequence[int], spatial: Sequence[int]) -> Tuple[int, ...]:
    """fftshift-ed index s -> unshifted frequency k = (s - n//2) mod n."""
    return tuple((int(s) - n // 2) % n for s, n in zip(idx, spatial))


def spike_op(idx_shifted: Sequence[int], geo: Geometry, log_intensity: float,
             phase: Optional[float] = None, chan: int = -1) -> TbOp:
    """Set |k| = exp(log_intensity) at the fftshift-ed spatial index (phase kept or overridden).

    RandPlaneWaves_ellipsoid (filters_and_operators.py:383-390; all channels) and
    KSpaceSpikeNoise._set_spike (:966-983; one channel or all)."""
    if len(idx_shifted) != len(geo.spatial):
        raise ValueError("spike index rank does not match the transformed axes")
    for s, n in zip(idx_shifted, geo.spatial):
        if not 0 <= int(s) < n:
            raise IndexError(f"spike index {tuple(idx_shifted)} out of bounds for {geo.spatial}")
    k = unshift(idx_shifted, geo.spatial)
    kh, kw, kd = geo.to_hwd(k)
    op = _op(TB_OP_SPIKE, chan)
    op.i[0], op.i[1], op.i[2] = kh, kw, kd
    op.f[0] = np.exp(np.float32(log_intensity))  # torch float32 exp of the stored log value
    if phase is None:
        op.f[1] = np.float32(np.nan)
    else:
        op.f[1] = np.float32(phase)
        op.f[2] = np.cos(np.float32(phase))
        op.f[3] = np.sin(np.float32(phase))
    return op


Program = List[TbOp]


def _copy(op: TbOp) -> TbOp:
    c = TbOp()
    C_ = type(op)
    for name, _ in C_._fields_:
        v = getattr(op, name)
        setattr(c, name, v if not hasattr(v, "_length_") else type(v)(*v))
    return c


def _touch(a: TbOp, b: TbOp, hwd: Sequence[int]) -> bool:
    """Spikes ``a`` and ``b`` reach the same stored coefficient (equal or conjugate frequencies,
    overlapping channels)."""
    if a.kind != TB_OP_SPIKE or b.kind != TB_OP_SPIKE:
        return True
    if a.chan != -1 and b.chan != -1 and a.chan != b.chan:
        return False
    fa = tuple(int(v) for v in a.i)
    fb = tuple(int(v) for v in b.i)
    conj = tuple((n - v) % n for v, n in zip(fb, hwd))
    return fa == fb or fa == conj


def split_program(prog: Sequence[TbOp], hwd: Sequence[int], max_ops: int = TB_MAX_OPS) -> List[List[TbOp]]:
    """Cut a program longer than one launch holds (``TB_MAX_OPS``) into passes run one after the
    other, each FFT -> ops -> inverse FFT (.real), at points where that is exact:

    * between two reference calls (ops not joined by ``reserved``): the reference itself takes
      ``.real`` after every call, which a separate pass reproduces;
    * inside one call's group of spikes (KSpaceSpikeNoise with many locations, channel-wise
      draws): a later part reads the spectrum after the earlier part's pass, which differs from the
      pre-call spectrum only at the earlier part's own frequencies and their conjugates -- so the cut
      is exact when no spike of the later part touches those (same or conjugate frequency in an
      overlapping channel); otherwise ValueError.
    The first op of every later pass starts a new group."""
    if len(prog) <= max_ops:
        return [list(prog)]
    chunks: List[List[TbOp]] = [[]]
    group: List[Tuple[int, TbOp]] = []   # the current call's spikes so far, with their pass index
    for op in prog:
        cut = len(chunks[-1]) == max_ops
        if cut:
            chunks.append([])
        k = len(chunks) - 1
        if not op.reserved:
            group = []
        elif any(ki < k and _touch(g, op, hwd) for ki, g in group):
            raise ValueError("cannot split this spike group exactly: two of its spikes share a frequency "
                             "(or its conjugate) in one channel")
        o = op
        if cut and op.reserved:
            o = _copy(op)
            o.reserved = 0
        chunks[-1].append(o)
        group.append((k, op))
    return chunks
