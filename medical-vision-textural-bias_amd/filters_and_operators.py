"""Drop-in replacement of the reference's ``source_code/filters_and_operators.py``.

Same module name, class names, constructor arguments, RNG draws and error
behaviour as the reference; the arithmetic runs in the texbias HIP kernels
(``libtexbias.so``) on the MI355X.  A driver switches by pointing its
``SOURCE_CODE_PATH`` at this directory.

Tensors on the CPU are moved to the current HIP device for the filter and the
result is returned on the caller's device; there is no CPU implementation --
without a HIP device the filters raise.  For throughput use the batched
device-side stage ``texbias.pipeline.FusedChain`` after collation instead of
per-sample calls inside DataLoader workers.  The arithmetic goes through the
``torch.ops.texbias.*`` custom operators (``texbias/ops.py``).

Inside ``DataLoader`` worker processes (forked: no HIP context) the dictionary transforms defer:
they make their draws and record the sample's stage for one batched GPU pass in the main process
(``texbias.deferred``: ``deferred_collate`` + ``run_deferred`` / ``DeferredLoader``).

Reference line numbers are cited per class (``filters_and_operators.py:N``).
"""
from __future__ import annotations

import warnings
from math import floor
from typing import Any, Dict, Hashable, List, Mapping, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from texbias import deferred as _D
from texbias import kprog as _K
from texbias import ops as _ops  # registers torch.ops.texbias.*
from texbias import runtime as _rt
from texbias.shell import shell_coords as _shell_coords
from texbias.transform_base import (MapTransform, Randomizable, RandomizableTransform, Transform,
                                    ensure_tuple)

KeysCollection = Union[Hashable, Sequence[Hashable]]

__all__ = [
    "SelectChanneld", "ConvertToMultiChannelBasedOnBratsClassesd", "WholeTumorTCGA", "disk_mask",
    "RandFourierDiskMaskd", "ellipsoid", "RandPlaneWaves_ellipsoid", "SaltAndPepper", "WrapArtifact",
    "WrapArtifactd", "SegmentationSlicesd", "Fourier", "GibbsNoise", "RandGibbsNoise", "RandGibbsNoised",
    "KSpaceSpikeNoise", "RandKSpaceSpikeNoise", "RandKSpaceSpikeNoised", "MultimodalSlicesd",
]


# ------------------------------------------------------------------ helpers
def _device_of(t) -> torch.device:
    if isinstance(t, torch.Tensor) and t.device.type == "cuda":
        return t.device
    if torch.utils.data.get_worker_info() is not None:
        raise _rt.TexbiasError(
            "texbias filters cannot run inside a (forked) DataLoader worker: use the dictionary transforms, which "
            "defer there, with collate_fn=texbias.deferred.deferred_collate and texbias.deferred.DeferredLoader")
    if not torch.cuda.is_available():
        raise _rt.TexbiasError("texbias filters need a HIP device (there is no CPU implementation)")
    return torch.device("cuda", torch.cuda.current_device())


def _as_f32_tensor(img) -> torch.Tensor:
    """numpy -> torch.Tensor(img) exactly like the reference (float32 CPU tensor)."""
    if isinstance(img, np.ndarray):
        return torch.Tensor(img)
    return img


def _kspace(img: torch.Tensor, n_dims: int, program: Sequence, pad: int = 0) -> torch.Tensor:
    """One sample [*channels, *spatial]: run `program` over the trailing n_dims axes on the device,
    return a float32 tensor on the caller's device."""
    dev = _device_of(img)
    x = img.to(device=dev, dtype=torch.float32)
    lead = x.shape[: x.dim() - n_dims]
    chans = int(np.prod(lead)) if len(lead) else 1
    xb = x.reshape((1, chans) + tuple(x.shape[x.dim() - n_dims:]))
    geo = _K.geometry(tuple(x.shape[x.dim() - n_dims:]))
    y, _ = torch.ops.texbias.kspace_filter(xb, n_dims, _ops.pack_programs_split([list(program)], geo.hwd), chans, 0)
    y = y.reshape(tuple(x.shape))
    return y if img.device == dev else y.to(img.device)


# ---------------------------------------------------------- channel glue
class SelectChanneld(MapTransform):
    """Keep one channel per key, keeping a leading channel axis (:25-58)."""

    def __init__(self, keys, chan_num: Union[int, Sequence[int]], allow_missing_keys=False):
        self.chan_num = chan_num
        super().__init__(keys, allow_missing_keys)

    def __call__(self, data):
        d = dict(data)
        if isinstance(self.chan_num, Sequence):
            if len(self.chan_num) > 1:
                for i, key in zip(self.chan_num, self.key_iterator(d)):
                    if d[key].shape[0] <= i:
                        raise AssertionError(
                            f"Provided channel index {i} larger than max channel index for key = {key}")
                    self._select(d, key, i)
            else:
                for key in self.key_iterator(d):
                    self._select(d, key, self.chan_num[0])
        else:
            for key in self.key_iterator(d):
                self._select(d, key, self.chan_num)
        return d

    @staticmethod
    def _select(d, key, c) -> None:
        if _D.active() and _D.has_plan(d, key):  # a deferred filter is pending: select after it
            _D.record(d, key, ("sel", int(c)))
        else:
            d[key] = d[key][c][None, :]


class ConvertToMultiChannelBasedOnBratsClassesd(MapTransform):
    """BraTS labels {1 edema, 2 enhancing, 3 necrotic} -> channels (TC, WT, ET) (:61-87)."""

    def __call__(self, data):
        d = dict(data)
        for key in self.keys:
            lab = np.asarray(d[key])
            tc = (lab == 2) | (lab == 3)
            wt = tc | (lab == 1)
            et = lab == 2
            d[key] = np.stack([tc, wt, et], axis=0).astype(np.float32)
        return d


class WholeTumorTCGA(MapTransform):
    """Any non-zero TCGA label -> whole tumour, with a channel axis (:90-101)."""

    def __init__(self, keys, allow_missing_keys=False):
        MapTransform.__init__(self, keys, allow_missing_keys)

    def __call__(self, data):
        d = dict(data)
        for key in self.key_iterator(d):
            d[key] = (np.asarray(d[key]) != 0)[None, :].astype(np.float32)
        return d


# ---------------------------------------------------------------- disk mask
class disk_mask:
    """Binary disk (dim=2) / sphere (dim=3) on the trailing axes of a k-space tensor (:105-206).

    Centre floor(n/2) of the fftshift-ed grid, strict ``<``; ``inside_off`` inverts.  The mask
    is built by the ``tb_disk_mask_f32`` kernel on the device and kept on ``k_tensor``'s device.
    """

    def __init__(self, k_tensor: torch.Tensor, r: float = 2, dim: int = 2, inside_off=True):
        self.r = r
        self.dim = dim
        self.inside_off = inside_off
        self.last_dims = k_tensor.size(-1)
        if dim in (2, 3):
            dev = _device_of(k_tensor)
            m = _rt.disk_mask_tensor(tuple(k_tensor.shape), r, dim, inside_off, dev)
            self.binary_mask = m if k_tensor.device == dev else m.to(k_tensor.device)
        else:
            print("Only 2- and 3-dimensional images.")

    def binary_mask_2d(self, k_tensor) -> torch.Tensor:
        return _rt.disk_mask_tensor(tuple(k_tensor.shape), self.r, 2, self.inside_off, _device_of(k_tensor))

    def binary_mask_3d(self, k_tensor) -> torch.Tensor:
        return _rt.disk_mask_tensor(tuple(k_tensor.shape), self.r, 3, self.inside_off, _device_of(k_tensor))

    def apply(self, k_tensor: torch.Tensor) -> torch.Tensor:
        assert k_tensor.size(-1) == self.last_dims, f"Last dimension of input must be = {self.last_dims}"
        return k_tensor * self.binary_mask


class RandFourierDiskMaskd(RandomizableTransform, MapTransform):
    """Low-pass (``inside_off=False``) / high-pass disk mask in k-space -- "Gibbs truncation" (:210-279).

    ``r`` may be ``[lo, hi]``: it is sampled ONCE on the first call and then frozen (the
    reference overwrites ``self.r``, :260-261).  The sphere always spans the last 3 axes.
    """

    def __init__(self, keys: Union[str, List[str]], r: Union[float, List[float]] = float("Inf"),
                 inside_off: bool = False, prob: float = 0.5, allow_missing_keys: bool = False) -> None:
        assert prob <= 1 and prob >= 0, "prob must take values in [0,1]"
        self.r = r
        self.inside_off = inside_off
        MapTransform.__init__(self, keys, allow_missing_keys)
        RandomizableTransform.__init__(self, prob=prob)

    def program(self) -> List:
        return [_K.disk_op(self.r, self.inside_off)]

    def __call__(self, data):
        d = dict(data)
        self.randomize()
        if _D.active():
            for key in self.key_iterator(d):
                _D.record(d, key, ("k", self.program() if self._do_transform else []))
            return d
        if not self._do_transform:
            return d
        for key in self.key_iterator(d):
            d[key] = _kspace(_as_f32_tensor(d[key]), 3, self.program())
        return d

    def randomize(self, data=None) -> None:
        super().randomize(None)
        if type(self.r) == list:  # noqa: E721 - the reference tests the exact type
            self.r = self.R.uniform(self.r[0], self.r[1])

    def shift_fourier(self, x: torch.Tensor) -> torch.Tensor:
        return Fourier.shift_fourier(x, 3)

    def inv_shift_fourier(self, k: torch.Tensor) -> torch.Tensor:
        return Fourier.inv_shift_fourier_complex(k, 3)


# --------------------------------------------------------------- ellipsoid
class ellipsoid(Randomizable):
    """Shell 0.95 < sum((i-c)^2/a^2) < 1.05 (float32), centre floor(n/2) (:284-352).

    The candidate list (row-major, what ``mask.nonzero()`` yields) is computed once per
    (shape, a, b, c) and cached; sampling draws ``self.R.randint(0, len)`` exactly as the
    reference does, so seeded sequences reproduce.
    """

    def __init__(self, a: float, b: float, c: float):
        self.a, self.b, self.c = a, b, c

    def binary_mask_3d(self, k_tensor) -> torch.Tensor:
        shape = tuple(k_tensor.size())
        sp = shape[-3:]
        m = np.zeros(sp, np.float32)
        co = _shell_coords(sp, self.a, self.b, self.c)
        m[tuple(co.T)] = 1.0
        return torch.from_numpy(np.broadcast_to(m, shape).copy())

    def _get_3d_center(self, data):
        return (floor(data.size(-3) / 2), floor(data.size(-2) / 2), floor(data.size(-1) / 2))

    def _get_three_axes(self, data):
        return tuple(torch.arange(0, data.size(i)) for i in (-3, -2, -1))

    def sample_ellipsoid(self, k_tensor) -> Tuple[int, int, int]:
        shape = tuple(k_tensor.shape) if hasattr(k_tensor, "shape") else tuple(k_tensor)
        if len(shape) != 3:
            raise ValueError("sample_ellipsoid expects a 3-D grid")
        co = _shell_coords(shape, self.a, self.b, self.c)
        idx = self.R.randint(0, len(co))
        return tuple(int(v) for v in co[idx])

    def randomize(self, data=None):
        pass


class RandPlaneWaves_ellipsoid(RandomizableTransform, MapTransform):
    """Plane-wave artefact: |k| := exp(intensity_value) at one point of the ellipsoid shell,
    same point for all channels, phase kept (:355-414)."""

    def __init__(self, keys: Union[str, List[str]] = "image", a: float = 10, b: float = 10, c: float = 10,
                 intensity_value: float = 1, prob: float = 0.2, allow_missing_keys: bool = False):
        MapTransform.__init__(self, keys, allow_missing_keys)
        RandomizableTransform.__init__(self, prob=prob)
        self.ellipsoid = ellipsoid(a, b, c)
        self.intensity_value = intensity_value
        self.idx = None

    def program_for(self, spatial: Sequence[int], phase: Optional[Sequence[float]] = None) -> List:
        """Sample the shell point for a [C, *spatial] item and return its op program."""
        self.idx = self.ellipsoid.sample_ellipsoid(tuple(spatial))
        geo = _K.geometry(spatial)
        if phase is None:
            return [_K.spike_op(self.idx, geo, self.intensity_value)]
        return [_K.spike_op(self.idx, geo, self.intensity_value, phase=float(p), chan=c) for c, p in enumerate(phase)]

    def __call__(self, data, phase: Optional[Sequence[float]] = None):
        d = dict(data)
        self.randomize(None)
        if _D.active():
            for key in self.key_iterator(d):
                prog = self.program_for(tuple(d[key].shape[-3:]), phase) if self._do_transform else []
                for op in prog[1:]:
                    op.reserved = 1
                _D.record(d, key, ("k", prog))
            return d
        if not self._do_transform:
            return d
        for key in self.key_iterator(d):
            img = _as_f32_tensor(d[key])
            prog = self.program_for(tuple(img.shape[-3:]), phase)
            if phase is not None:
                for op in prog[1:]:
                    op.reserved = 1
            d[key] = _kspace(img, 3, prog)
        return d

    def shift_fourier(self, x: torch.Tensor) -> torch.Tensor:
        return Fourier.shift_fourier(x, 3)

    def inv_shift_fourier(self, k: torch.Tensor) -> torch.Tensor:
        return Fourier.inv_shift_fourier(k, 3)


# ----------------------------------------------------------- salt & pepper
def _sap_thresholds(p: float) -> Tuple[float, float]:
    """u <= p/2 -> MIN, p/2 < u <= p -> MAX, compared in float32 (:478-479)."""
    return float(np.float32(p / 2)), float(np.float32(p))


def _philox_seed() -> int:
    """Per-call Philox key drawn from torch's global CPU generator (the reference's
    ``torch.rand`` draws from it too, :472), so torch.manual_seed reproduces runs."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class SaltAndPepper(MapTransform, RandomizableTransform):
    """Salt-and-pepper: u ~ U[0,1) per voxel; u <= p/2 -> min/2, p/2 < u <= p -> max/2 of the
    whole (all-channel) input (:419-482)."""

    def __init__(self, p: float = 0, keys: Union[str, List[str]] = "image", prob: float = 1.0,
                 allow_missing_keys: bool = False):
        self.p = min(max(0, p), 1.0)
        if p < 0 or p > 1:
            warnings.warn(f"Setting p to {self.p}.")
        MapTransform.__init__(self, keys, allow_missing_keys)
        RandomizableTransform.__init__(self, prob=prob)

    def __call__(self, data):
        d = dict(data)
        self.randomize(None)
        if _D.active():   # the Philox key is drawn here, in the worker, as the eager call draws it
            for key in self.key_iterator(d):
                _D.record(d, key, ("sap", self.p, _philox_seed()) if self._do_transform else ("sap", None, None))
            return d
        if not self._do_transform:
            return d
        for key in self.key_iterator(d):
            d[key] = self.salt_and_pepper(d[key])
        return d

    def salt_and_pepper(self, x: torch.Tensor, u: Optional[torch.Tensor] = None,
                        return_classes: bool = False):
        """``u`` (same shape) replays an explicit uniform field (parity mode); otherwise a
        device Philox stream keyed from torch's global generator.  ``return_classes`` also
        returns the int8 class map (0 keep, 1 MIN, 2 MAX)."""
        x = _as_f32_tensor(x)
        dev = _device_of(x)
        xd = x.to(device=dev, dtype=torch.float32).contiguous()
        nd = xd.dim()
        mm = _rt.minmax_keys(xd, nd)
        out = xd.clone()
        cls = torch.empty(xd.shape, dtype=torch.int8, device=dev) if return_classes else None
        ud = u.to(device=dev, dtype=torch.float32).contiguous() if u is not None else None
        seed = _philox_seed() if u is None else 0
        same = ud is None and cls is None
        _rt.salt_and_pepper(out if same else xd, nd, [_sap_thresholds(self.p)], mm, out=out, u=ud, cls=cls,
                            seed=seed)
        y = out if x.device == dev else out.to(x.device)
        if return_classes:
            return y, (cls if x.device == dev else cls.to(x.device))
        return y


# ---------------------------------------------------------------- wrap-around
class WrapArtifact(Transform):
    """Wrap-around: k-space entries with an odd fftshift-ed index along each of the 3 spatial
    axes are scaled by alpha (alpha^m for m odd coordinates) (:488-537).  3-D only, as the
    reference's hard-wired 4-D indexing."""

    def __init__(self, alpha: float = 0.5):
        self.alpha = alpha

    def program(self) -> List:
        return [_K.wrap_op(self.alpha)]

    def __call__(self, img: torch.Tensor):
        img = _as_f32_tensor(img)
        if img.dim() < 4:
            raise IndexError(f"too many indices for tensor of dimension {img.dim()}")
        if img.dim() > 4:
            raise NotImplementedError("WrapArtifact: only (C, H, W, D) inputs (the reference's 4-D indexing)")
        return _kspace(img, 3, self.program())

    def _shift_fourier(self, x: torch.Tensor, n_dims: int) -> torch.Tensor:
        return Fourier.shift_fourier(x, n_dims)

    def _inv_shift_fourier(self, k: torch.Tensor, n_dims: int) -> torch.Tensor:
        return Fourier.inv_shift_fourier(k, n_dims)


class WrapArtifactd(MapTransform):
    """Dictionary version of :class:`WrapArtifact` (:540-560)."""

    def __init__(self, keys: KeysCollection, alpha: float = 0.5, allow_missing_keys: bool = False):
        MapTransform.__init__(self, keys, allow_missing_keys)
        self.transform = WrapArtifact(alpha)

    def __call__(self, data: Mapping[Hashable, torch.Tensor]):
        d = dict(data)
        for key in self.key_iterator(d):
            if _D.active():
                _D.record(d, key, ("k", self.transform.program()))
            else:
                d[key] = self.transform(d[key])
        return d


class SegmentationSlicesd(MapTransform, Randomizable):
    """Three consecutive slices around a depth c whose +-3 neighbours both contain label (:563-589)."""

    def __init__(self, keys, seed: Optional[int] = None, allow_missing_keys: bool = False):
        Randomizable.set_random_state(self, seed=seed)
        MapTransform.__init__(self, keys, allow_missing_keys)

    def randomize(self, data=None):
        pass

    def __call__(self, data):
        d = dict(data)
        lab = d["label"]
        while True:
            c = self.R.randint(3, 60)
            if lab[0, :, :, c - 3].max() == lab[0, :, :, c + 3].max() == 1:
                break
        for key in self.key_iterator(d):
            d[key] = d[key].squeeze(0)[:, :, c:c + 3].transpose(0, 2)
        return d


# ------------------------------------------------------------------- Fourier
class Fourier:
    """Full-spectrum helpers (:594-632).  Not on the filter hot path (the filters never
    materialise a full shifted complex spectrum); provided for API compatibility and run
    by torch.fft on the tensor's device."""

    @staticmethod
    def shift_fourier(x: torch.Tensor, n_dims: int) -> torch.Tensor:
        dims = tuple(range(-n_dims, 0))
        return torch.fft.fftshift(torch.fft.fftn(x, dim=dims), dim=dims)

    @staticmethod
    def inv_shift_fourier(k: torch.Tensor, n_dims: int) -> torch.Tensor:
        dims = tuple(range(-n_dims, 0))
        return torch.fft.ifftn(torch.fft.ifftshift(k, dim=dims), dim=dims).real

    @staticmethod
    def inv_shift_fourier_complex(k: torch.Tensor, n_dims: int) -> torch.Tensor:
        dims = tuple(range(-n_dims, 0))
        return torch.fft.ifftn(torch.fft.ifftshift(k, dim=dims), dim=dims, norm="backward")


# --------------------------------------------------------------- Gibbs noise
class GibbsNoise(Transform, Fourier):
    """MONAI-style Gibbs truncation: keep k-space within r = (1-alpha)*max(shape)*sqrt(2)/2 of the
    (n-1)/2 centre (float64 geometry), all channels (:635-705).  2-D or 3-D."""

    def __init__(self, alpha: float = 0.5, as_tensor_output: bool = True) -> None:
        if alpha > 1 or alpha < 0:
            raise AssertionError("alpha must take values in the interval [0,1].")
        self.alpha = alpha
        self.as_tensor_output = as_tensor_output

    def program(self, spatial: Sequence[int]) -> List:
        return [_K.gibbs_op(self.alpha, spatial)]

    def __call__(self, img: Union[np.ndarray, torch.Tensor]) -> Union[torch.Tensor, np.ndarray]:
        n_dims = len(img.shape[1:])
        img = _as_f32_tensor(img)
        out = _kspace(img, n_dims, self.program(tuple(img.shape[1:])))
        return out if self.as_tensor_output else out.cpu().detach().numpy()


class RandGibbsNoise(RandomizableTransform):
    """Random GibbsNoise: applied with probability ``prob``, alpha ~ U(alpha[0], alpha[1]) (:708-768)."""

    def __init__(self, prob: float = 0.1, alpha: Sequence[float] = (0.0, 1.0), as_tensor_output: bool = True) -> None:
        if len(alpha) != 2:
            raise AssertionError("alpha length must be 2.")
        if alpha[1] > 1 or alpha[0] < 0:
            raise AssertionError("alpha must take values in the interval [0,1]")
        if alpha[0] > alpha[1]:
            raise AssertionError("When alpha = [a,b] we need a < b.")
        self.alpha = alpha
        self.sampled_alpha = -1.0
        self.as_tensor_output = as_tensor_output
        RandomizableTransform.__init__(self, prob=prob)

    def __call__(self, img: Union[np.ndarray, torch.Tensor]) -> Union[torch.Tensor, np.ndarray]:
        self._randomize(None)
        if self._do_transform:
            return GibbsNoise(self.sampled_alpha, self.as_tensor_output)(img)
        if isinstance(img, np.ndarray) and self.as_tensor_output:
            return torch.Tensor(img)
        if isinstance(img, torch.Tensor) and not self.as_tensor_output:
            return img.detach().cpu().numpy()
        return img

    def _randomize(self, _: Any) -> None:
        super().randomize(None)
        self.sampled_alpha = self.R.uniform(self.alpha[0], self.alpha[1])


class RandGibbsNoised(RandomizableTransform, MapTransform):
    """Dictionary RandGibbsNoise; one alpha per call shared by all keys (:771-843)."""

    def __init__(self, keys: KeysCollection, prob: float = 0.1, alpha: Sequence[float] = (0.0, 1.0),
                 as_tensor_output: bool = True, allow_missing_keys: bool = False) -> None:
        MapTransform.__init__(self, keys, allow_missing_keys)
        RandomizableTransform.__init__(self, prob=prob)
        self.alpha = alpha
        self.sampled_alpha = -1.0
        self.as_tensor_output = as_tensor_output

    def __call__(self, data: Mapping[Hashable, Union[torch.Tensor, np.ndarray]]) -> Dict[Hashable, Any]:
        d = dict(data)
        self._randomize(None)
        if _D.active():
            for key in self.key_iterator(d):
                sp = tuple(d[key].shape[1:])
                _D.record(d, key, ("k", [_K.gibbs_op(self.sampled_alpha, sp)] if self._do_transform else []))
            return d
        transform = None
        for i, key in enumerate(self.key_iterator(d)):
            if self._do_transform:
                if i == 0:
                    transform = GibbsNoise(self.sampled_alpha, self.as_tensor_output)
                d[key] = transform(d[key])
            else:
                if isinstance(d[key], np.ndarray) and self.as_tensor_output:
                    d[key] = torch.Tensor(d[key])
                elif isinstance(d[key], torch.Tensor) and not self.as_tensor_output:
                    d[key] = self._to_numpy(d[key])
        return d

    def _randomize(self, _: Any) -> None:
        super().randomize(None)
        self.sampled_alpha = self.R.uniform(self.alpha[0], self.alpha[1])

    def _to_numpy(self, d: Union[torch.Tensor, np.ndarray]) -> np.ndarray:
        return d.cpu().detach().numpy() if isinstance(d, torch.Tensor) else d


# ------------------------------------------------------------ k-space spikes
def _is_seq(v) -> bool:
    return isinstance(v, Sequence) and not isinstance(v, (str, bytes))


def _default_intensities(img: torch.Tensor, n_dims: int) -> Tuple[float, ...]:
    """2.5 * mean(log(|FFT(img)| + 1e-10)) per channel (:927-933), reduced on the device."""
    dev = _device_of(img)
    x = img.to(device=dev, dtype=torch.float32)
    chans = x.shape[0]
    xb = x.reshape((1, chans) + tuple(x.shape[1:]))
    sums = _rt.logabs_sums(xb, n_dims, [[]], chans).cpu().numpy()
    n = float(np.prod(x.shape[1:]))
    return tuple(float(np.float32(s / n) * np.float32(2.5)) for s in sums)


class KSpaceSpikeNoise(Transform, Fourier):
    """Spikes in k-space: log|k| := value at given (fftshift-ed) locations, phase kept (:846-983).

    ``loc``: one spatial tuple (all channels), or a sequence of tuples, each (C, X, Y[, Z]) for one
    channel or spatial-only for all channels.  ``k_intensity=None`` uses 2.5*mean(log|k|) per
    channel, zipped against the locations in order exactly as the reference does (:936-938).
    """

    def __init__(self, loc: Union[Tuple, Sequence[Tuple]], k_intensity: Optional[Union[Sequence[float], float]] = None,
                 as_tensor_output: bool = True):
        self.loc = ensure_tuple(loc)
        self.as_tensor_output = as_tensor_output
        self.k_intensity = k_intensity
        if isinstance(k_intensity, Sequence):
            if not isinstance(loc[0], Sequence):
                raise AssertionError(
                    "If a sequence is passed to k_intensity, then a sequence of locations must be passed to loc")
            if len(k_intensity) != len(loc):
                raise AssertionError("There must be one intensity_factor value for each tuple of indices in loc.")
        if isinstance(self.loc[0], Sequence) and k_intensity is not None:
            if not isinstance(self.k_intensity, Sequence):
                raise AssertionError("There must be one intensity_factor value for each tuple of indices in loc.")

    def _check_indices(self, img) -> None:
        loc = list(self.loc)
        if not isinstance(loc[0], Sequence):
            loc = [loc]
        loc = [([0] + list(l)) if len(l) < len(img.shape) else list(l) for l in loc]
        for i in range(len(img.shape)):
            if img.shape[i] <= max(x[i] for x in loc):
                raise AssertionError(
                    f"The index value at position {i} of one of the tuples in loc = {self.loc} is out of bounds "
                    "for current image.")

    def program(self, img, k_intensity=None) -> List:
        """Op program for a [C, *spatial] image (validates like the reference)."""
        shape = tuple(img.shape)
        n_dims = len(shape) - 1
        geo = _K.geometry(shape[1:])
        if k_intensity is None:
            k_intensity = self.k_intensity
        if k_intensity is None:
            k_intensity = _default_intensities(_as_f32_tensor(img), n_dims)
        ops: List = []

        def spike(idx, val):
            idx = tuple(int(v) for v in idx)
            if len(idx) == len(shape):
                v = val[idx[0]] if _is_seq(val) else val
                ops.append(_K.spike_op(idx[1:], geo, float(v), chan=idx[0]))
            elif len(idx) == len(shape) - 1 and len(shape) in (3, 4):
                if _is_seq(val) or (isinstance(val, np.ndarray) and val.ndim):
                    raise TypeError(f"can't assign a {type(val).__name__} to a torch.FloatTensor")
                ops.append(_K.spike_op(idx, geo, float(val)))
            # any other rank: the reference silently sets nothing (:975-983)

        if isinstance(self.loc[0], Sequence):
            for idx, val in zip(self.loc, ensure_tuple(k_intensity)):
                spike(idx, val)
        else:
            spike(self.loc, k_intensity)
        # one call = one simultaneous group; a later duplicate location overwrites an earlier one
        seen: Dict[Tuple[int, int, int, int], int] = {}
        for j, op in enumerate(ops):
            seen[(op.chan, op.i[0], op.i[1], op.i[2])] = j
        ops = [op for j, op in enumerate(ops) if seen[(op.chan, op.i[0], op.i[1], op.i[2])] == j]
        for op in ops[1:]:
            op.reserved = 1
        return ops

    def __call__(self, img: Union[np.ndarray, torch.Tensor]) -> Union[torch.Tensor, np.ndarray]:
        self._check_indices(img)
        if len(img.shape) < 3:
            raise AssertionError("Image needs a channel direction.")
        if isinstance(self.loc[0], int) and len(img.shape) == 4 and len(self.loc) == 2:
            raise AssertionError("Input images of dimension 4 need location tuple to be length 3 or 4")
        if isinstance(self.loc[0], Sequence) and len(img.shape) == 4 and min(map(len, self.loc)) == 2:
            raise AssertionError("Input images of dimension 4 need location tuple to be length 3 or 4")
        n_dims = len(img.shape[1:])
        img = _as_f32_tensor(img)
        prog = self.program(img)
        out = _kspace(img, n_dims, prog) if prog else _kspace(img, n_dims, [])
        return out if self.as_tensor_output else out.cpu().detach().numpy()


class RandKSpaceSpikeNoise(RandomizableTransform, Fourier):
    """Random k-space spikes, per channel (``channel_wise``) or one location for all (:986-1131)."""

    def __init__(self, prob: float = 0.1, intensity_range: Optional[Sequence[Union[Sequence[float], float]]] = None,
                 channel_wise=True, as_tensor_output: bool = True):
        self.intensity_range = intensity_range
        self.channel_wise = channel_wise
        self.as_tensor_output = as_tensor_output
        self.sampled_k_intensity: List = []
        self.sampled_locs: List[Tuple] = []
        if intensity_range is not None:
            if isinstance(intensity_range[0], Sequence) and not channel_wise:
                raise AssertionError(
                    "When channel_wise = False, intensity_range should be a 2-tuple (low, high) or None.")
        super().__init__(prob)

    def __call__(self, img: Union[np.ndarray, torch.Tensor]) -> Union[torch.Tensor, np.ndarray]:
        if self.intensity_range is not None:
            if isinstance(self.intensity_range[0], Sequence) and len(self.intensity_range) != img.shape[0]:
                raise AssertionError(
                    "If intensity_range is a sequence of sequences, then there must be one (low, high) tuple for "
                    "each channel.")
        self.sampled_k_intensity = []
        self.sampled_locs = []
        if not isinstance(img, torch.Tensor):
            img = torch.Tensor(img)
        intensity_range = self._make_sequence(img)
        self._randomize(img, intensity_range)
        if self.sampled_locs:
            transform = KSpaceSpikeNoise(self.sampled_locs, self.sampled_k_intensity, self.as_tensor_output)
            return transform(img)
        return img if self.as_tensor_output else img.detach().numpy()

    def _randomize(self, img: torch.Tensor, intensity_range: Sequence[Sequence[float]]) -> None:
        if self.channel_wise:
            for i in range(img.shape[0]):
                super().randomize(None)
                if self._do_transform:
                    self.sampled_locs.append((i,) + tuple(self.R.randint(0, k) for k in img.shape[1:]))
                    self.sampled_k_intensity.append(self.R.uniform(intensity_range[i][0], intensity_range[i][1]))
        else:
            super().randomize(None)
            if self._do_transform:
                spatial = tuple(self.R.randint(0, k) for k in img.shape[1:])
                self.sampled_locs = [(i,) + spatial for i in range(img.shape[0])]
                if isinstance(intensity_range[0], Sequence):
                    self.sampled_k_intensity = [self.R.uniform(p[0], p[1]) for p in intensity_range]
                else:
                    self.sampled_k_intensity = [self.R.uniform(intensity_range[0], intensity_range[1])] * len(img)

    def _make_sequence(self, x: torch.Tensor) -> Sequence[Sequence[float]]:
        if self.intensity_range is not None:
            if not isinstance(self.intensity_range[0], Sequence):
                return (ensure_tuple(self.intensity_range),) * x.shape[0]
            return ensure_tuple(self.intensity_range)
        return self._set_default_range(x)

    def _set_default_range(self, img: torch.Tensor) -> Sequence[Sequence[float]]:
        means = _default_intensities(img, len(img.shape[1:]))
        return tuple((m * 0.95, m * 1.1) for m in means)


class RandKSpaceSpikeNoised(RandomizableTransform, MapTransform):
    """Dictionary RandKSpaceSpikeNoise with a global probability, one inner transform per key
    (:1134-1254)."""

    def __init__(self, keys: KeysCollection, global_prob: float = 1.0, prob: float = 0.1,
                 intensity_ranges: Optional[Mapping[Hashable, Sequence[Union[Sequence[float], float]]]] = None,
                 channel_wise: bool = True, common_sampling: bool = False, common_seed: int = 42,
                 as_tensor_output: bool = True, allow_missing_keys: bool = False):
        MapTransform.__init__(self, keys, allow_missing_keys)
        RandomizableTransform.__init__(self, global_prob)
        self.common_sampling = common_sampling
        self.common_seed = common_seed
        self.as_tensor_output = as_tensor_output
        self.transforms = {}
        for k in self.keys:
            rng = intensity_ranges[k] if isinstance(intensity_ranges, Mapping) else None
            self.transforms[k] = RandKSpaceSpikeNoise(prob, rng, channel_wise, self.as_tensor_output)

    def __call__(self, data):
        d = dict(data)
        super().randomize(None)
        if self.common_sampling:
            for k in self.keys:
                self.transforms[k].set_random_state(self.common_seed)
        if _D.active():
            from texbias.pipeline import spike_program
            for key, t in self.key_iterator(d, self.transforms):
                img = d[key]
                prog = spike_program(self.transforms[t], int(img.shape[0]), tuple(img.shape[1:])) \
                    if self._do_transform else []
                _D.record(d, key, ("k", prog))
            return d
        for key, t in self.key_iterator(d, self.transforms):
            if self._do_transform:
                d[key] = self.transforms[t](d[key])
            else:
                if isinstance(d[key], np.ndarray) and self.as_tensor_output:
                    d[key] = torch.Tensor(d[key])
                elif isinstance(d[key], torch.Tensor) and not self.as_tensor_output:
                    d[key] = self._to_numpy(d[key])
        return d

    def set_rand_state(self, seed: Optional[int] = None, state: Optional[np.random.RandomState] = None) -> None:
        self.set_random_state(seed, state)
        for key in self.keys:
            self.transforms[key].set_random_state(seed, state)

    def _to_numpy(self, d: Union[torch.Tensor, np.ndarray]) -> np.ndarray:
        return d.cpu().detach().numpy() if isinstance(d, torch.Tensor) else d


class MultimodalSlicesd(Randomizable, MapTransform):
    """One random image channel and one label channel per sample: the drivers' own glue class
    (10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
    stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:82-109), provided here so that a
    deferred Compose (texbias.deferred) can select AFTER the deferred filters: ``c =
    R.choice(img_chan_indices)`` once per call, image -> image[c], label -> label[label_idx]."""

    def __init__(self, keys, img_chan_indices: list = [0], label_idx: int = 0, seed: int = None,  # noqa: B006
                 allow_missing_keys: bool = False):
        Randomizable.set_random_state(self, seed=seed)
        MapTransform.__init__(self, keys, allow_missing_keys)
        self.img_chan_indices = img_chan_indices
        self.label_idx = label_idx

    def randomize(self, data=None):
        pass

    def __call__(self, data):
        d = dict(data)
        c = self.R.choice(self.img_chan_indices)
        for key in self.key_iterator(d):
            if key == "image":
                if _D.active() and _D.has_plan(d, key):
                    _D.record(d, key, ("sel", int(c)))
                else:
                    d[key] = d[key][c].unsqueeze(0)
            elif key == "label":
                d[key] = d[key][self.label_idx].unsqueeze(0)
        return d
