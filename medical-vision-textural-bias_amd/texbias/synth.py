"""Synthetic BraTS-like volumes and labels, generated on the device (no dataset in this image).

Volumes mirror the reference's preprocessed inputs (NormalizeIntensityd(nonzero=True,
channel_wise=True), e.g. 127_.../..._3modalities.py:167): zero background outside an
ellipsoidal "brain" (~55 % of the voxels), inside a smooth random field plus white noise,
z-scored per channel over the brain.  Labels are nested random blobs in the (TC, WT, ET)
channel convention of ConvertToMultiChannelBasedOnBratsClassesd.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch
import torch.nn.functional as F


def _brain_mask(spatial: Sequence[int], device) -> torch.Tensor:
    # a size-1 axis (2-D slices as [1, H, W]) sits at the centre
    axes = [torch.linspace(-1, 1, n, device=device) if n > 1 else torch.zeros(1, device=device) for n in spatial]
    g = torch.meshgrid(*axes, indexing="ij")
    r2 = sum((a / s) ** 2 for a, s in zip(g, (0.85, 0.8, 0.9)))
    return r2 < 1.0


def brats_like(batch: int, channels: int, spatial: Sequence[int], seed: int, device) -> torch.Tensor:
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    spatial = tuple(int(s) for s in spatial)
    low = tuple(max(2, s // 12) for s in spatial)
    coarse = torch.randn((batch, channels) + low, generator=gen, device=device)
    field = F.interpolate(coarse, size=spatial, mode="trilinear", align_corners=False)
    field = field / field.std() + 0.5 * torch.randn((batch, channels) + spatial, generator=gen, device=device)
    brain = _brain_mask(spatial, device)
    m = brain.float()
    n = m.sum()
    mean = (field * m).sum(dim=(2, 3, 4), keepdim=True) / n
    var = (((field - mean) * m) ** 2).sum(dim=(2, 3, 4), keepdim=True) / n
    return (((field - mean) / var.sqrt()) * m).contiguous()


def brats_labels(batch: int, spatial: Sequence[int], seed: int, device, pad_to: int = 0) -> torch.Tensor:
    """[B, 3, *spatial] float32 labels (TC, WT, ET) with WT >= TC >= ET; optional zero pad of D."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed + 7919)
    spatial = tuple(int(s) for s in spatial)
    low = tuple(max(2, s // 16) for s in spatial)
    blob = F.interpolate(torch.randn((batch, 1) + low, generator=gen, device=device), size=spatial,
                         mode="trilinear", align_corners=False)[:, 0]
    brain = _brain_mask(spatial, device)
    wt = (blob > 1.0) & brain
    tc = (blob > 1.4) & brain
    et = (blob > 1.8) & brain
    lab = torch.stack([tc, wt, et], dim=1).float()
    if pad_to and pad_to > spatial[-1]:
        lab = F.pad(lab, (0, pad_to - spatial[-1]))
    return lab.contiguous()
