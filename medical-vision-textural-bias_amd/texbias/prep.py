"""GPU-side BraTS preprocessing in front of the texture filters.

The reference's training Compose (10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:151-170) runs, per sample in CPU
DataLoader workers:

    ConvertToMultiChannelBasedOnBratsClassesd("label")      filters_and_operators.py:61-87
    Spacingd(pixdim=(1.5, 1.5, 2.0), mode=("bilinear", "nearest"))   (``pixdim=``)
    Orientationd(axcodes="RAS")                                       (``axcodes=``)
    RandSpatialCropd(roi_size=[128, 128, 64], random_size=False)  (validation: CenterSpatialCropd,
                                                                   ``center_crop=True``, :186)
    RandFlipd(prob=0.5, spatial_axis=0)
    NormalizeIntensityd("image", nonzero=True, channel_wise=True)
    RandScaleIntensityd("image", factors=0.1, prob=0.5)
    RandShiftIntensityd("image", offsets=0.1, prob=0.5)

``BratsPrep`` draws these per sample on the host with MONAI 0.5's draw order (each transform its
own ``RandomState``: crop corner ``randint(0, n - roi + 1)`` per axis; flip ``rand() < prob``;
scale ``uniform(-f, f)`` then ``rand() < prob``; shift ``uniform(-o, o)`` then ``rand() < prob``)
and applies them to a batch of resident raw volumes in one ``tb_brats_prep_f32`` call: a
statistics pass over each crop window, then one gather pass writing the cropped, flipped,
normalised, scaled and shifted image and the 3-channel label. Its output is what ``FusedChain``
consumes.

With ``pixdim`` and/or ``axcodes`` the spatial steps (spacing, orientation, crop, flip) are
composed on the host into one affine map per sample (``texbias.affine``; each sample's NIfTI
``affine`` is an input) and the device samples the raw volume through it: trilinear for the image,
nearest (round half to even) for the label, border clamping -- grid_sample's modes in MONAI's
``Spacing``.  The crop window is drawn on the resampled, reoriented grid, as in the reference.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._abi import TbPrepParams
from ._lib import check, lib
from . import affine as A
from . import runtime as rt


class BratsPrep:
    def __init__(self, roi_size: Sequence[int] = (128, 128, 64), flip_prob: float = 0.5,
                 flip_axis: Optional[int] = 0, scale_factors: float = 0.1, scale_prob: float = 0.5,
                 shift_offsets: float = 0.1, shift_prob: float = 0.5, normalize: bool = True,
                 pixdim: Optional[Sequence[float]] = None, axcodes: Optional[str] = None, center_crop: bool = False):
        """``pixdim``: Spacingd's target voxel size (None: no resampling); ``axcodes``: Orientationd's
        target (None: keep); ``center_crop``: CenterSpatialCropd instead of RandSpatialCropd (no
        crop draw)."""
        self.pixdim = None if pixdim is None else tuple(float(v) for v in pixdim)
        self.axcodes = axcodes
        self.center_crop = bool(center_crop)
        if len(roi_size) != 3:
            raise ValueError("roi_size: three spatial extents")
        self.roi = tuple(int(v) for v in roi_size)
        self.flip_prob = float(flip_prob)
        self.flip_axes = () if flip_axis is None else ((flip_axis,) if isinstance(flip_axis, int) else tuple(flip_axis))
        if any(a not in (0, 1, 2) for a in self.flip_axes):
            raise ValueError("flip axes are spatial axes 0..2")
        f, o = float(scale_factors), float(shift_offsets)
        self.factors = (min(-f, f), max(-f, f))
        self.offsets = (min(-o, o), max(-o, o))
        self.scale_prob, self.shift_prob = float(scale_prob), float(shift_prob)
        self.normalize = bool(normalize)
        self.set_random_state(None)

    def set_random_state(self, seed: Optional[int] = None) -> "BratsPrep":
        """One stream per transform (crop, flip, scale, shift), seeded ``seed + k``."""
        mk = (lambda k: np.random.RandomState(None)) if seed is None else \
            (lambda k: np.random.RandomState((int(seed) + k) % (2 ** 32)))
        self.R_crop, self.R_flip, self.R_scale, self.R_shift = (mk(k) for k in range(4))
        return self

    @property
    def resamples(self) -> bool:
        return self.pixdim is not None or self.axcodes is not None

    def spatial_map(self, spatial: Sequence[int], affine: Optional[np.ndarray] = None):
        """(4 x 4 map from the resampled, reoriented grid's indices to raw input coordinates, that
        grid's shape) for one sample (Spacingd then Orientationd; identity when neither is set)."""
        aff = np.eye(4) if affine is None else np.asarray(affine, dtype=float)
        if aff.shape != (4, 4):
            raise ValueError("affine: a 4 x 4 voxel-to-world matrix")
        M, shp = np.eye(4), tuple(int(v) for v in spatial)
        if self.pixdim is not None:
            M, shp, aff = A.spacing_map(shp, aff, self.pixdim)
        if self.axcodes is not None:
            O, shp = A.orientation_map(shp, aff, self.axcodes)
            M = M @ O
        return M, shp

    def draw(self, B: int, spatial: Sequence[int], affines: Optional[Sequence[np.ndarray]] = None) -> List[TbPrepParams]:
        """Per-sample draws in Compose order (crop, flip, scale, shift).  With resampling, each
        sample's crop is drawn on its own resampled, reoriented grid (``affines``: one 4 x 4 each)."""
        if affines is not None and len(affines) != B:
            raise ValueError("one affine per sample")
        out = []
        for b in range(B):
            M, shp = (self.spatial_map(spatial, None if affines is None else affines[b]) if self.resamples
                      else (None, tuple(int(v) for v in spatial)))
            if any(r > n for r, n in zip(self.roi, shp)):
                raise ValueError(f"roi {self.roi} larger than the volume {shp}")
            if self.center_crop:
                corner = list(A.center_corner(shp, self.roi))
            else:
                corner = [self.R_crop.randint(0, n - r + 1) if n > r else 0 for n, r in zip(shp, self.roi)]
            do_flip = self.R_flip.rand() < self.flip_prob
            factor = self.R_scale.uniform(low=self.factors[0], high=self.factors[1])
            do_scale = self.R_scale.rand() < self.scale_prob
            offset = self.R_shift.uniform(low=self.offsets[0], high=self.offsets[1])
            do_shift = self.R_shift.rand() < self.shift_prob
            p = TbPrepParams()
            p.h0, p.w0, p.d0 = (int(v) for v in corner)
            p.flip = sum(1 << a for a in self.flip_axes) if do_flip else 0
            p.scale = float(np.float32(1.0 + factor)) if do_scale else 1.0
            p.shift = float(np.float32(offset)) if do_shift else 0.0
            p.normalize = 1 if self.normalize else 0
            if M is not None:
                G = M @ A.crop_flip_map(corner, self.roi, self.flip_axes if do_flip else ())
                p.resample = 1
                for a in range(3):
                    for c in range(4):
                        p.m[4 * a + c] = float(G[a, c])
            out.append(p)
        return out

    def __call__(self, img: torch.Tensor, lab: Optional[torch.Tensor] = None,
                 params: Optional[Sequence[TbPrepParams]] = None,
                 affines: Optional[Sequence[np.ndarray]] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """img [B, C, H0, W0, D0] float32 on a HIP device; lab [B, H0, W0, D0] (class ids) or None;
        ``affines``: each sample's 4 x 4 voxel-to-world matrix (resampling only; default identity).
        Returns (image [B, C, *roi], label [B, 3, *roi] or None)."""
        rt.require_hip(img, "BratsPrep")
        if img.dim() != 5:
            raise ValueError("BratsPrep expects [B, C, H, W, D]")
        img = img.contiguous()
        B, Cn = img.shape[:2]
        sp = tuple(img.shape[2:])
        if lab is not None:
            if tuple(lab.shape) != (B,) + sp:
                raise ValueError(f"label must be [B, H, W, D] = {(B,) + sp}")
            lab = lab.to(device=img.device, dtype=torch.float32).contiguous()
        params = list(params) if params is not None else self.draw(B, sp, affines)
        if len(params) != B:
            raise ValueError("one parameter record per sample")
        arr = (TbPrepParams * B)(*params)
        h, w, d = self.roi
        out = torch.empty((B, Cn, h, w, d), dtype=torch.float32, device=img.device)
        olab = torch.empty((B, 3, h, w, d), dtype=torch.float32, device=img.device) if lab is not None else None
        nws = int(lib().tb_brats_prep_workspace_bytes(min(B, 8), Cn))
        ws = rt.workspace_prep(img.device, nws)
        with torch.cuda.device(img.device):
            check(lib().tb_brats_prep_f32(img.data_ptr(), lab.data_ptr() if lab is not None else None, B, Cn, *sp,
                                          C.cast(arr, C.c_void_p), h, w, d, out.data_ptr(),
                                          olab.data_ptr() if olab is not None else None, ws.data_ptr(), nws,
                                          rt._stream(img.device)), "tb_brats_prep_f32")
        return out, olab
