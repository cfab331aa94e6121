"""Drop-in replacement of the reference's ``source_code/stylization_layers.py``.

In-model texture filters in front of the 3-D U-Net, running the texbias HIP kernels:

* ``GibbsNoiseLayer`` (stylization_layers.py:55-116): k-space low-pass with the mask
  ``dist / (alpha * max dist) <= 1`` (centre (n-1)/2, float32 geometry) over ALL non-batch axes.
  ``alpha`` is a registered buffer (the reference keeps a plain tensor that is in neither
  ``state_dict`` nor ``parameters()``); the kernel reads it from device memory, so a
  finite-difference update of ``alpha`` (Gibbs_GD) never forces a host sync.  Its gradient w.r.t.
  alpha is zero as in the reference; w.r.t. the input the filter is self-adjoint, so the backward
  pass is the same filter applied to the incoming gradient.
* ``spike_layer`` / ``Spikes_UNet`` (:143-174): a fresh ``RandKSpaceSpikeNoise(prob=1,
  intensity_range=(I, I), channel_wise=False)`` per forward (one location shared by the batch,
  drawn from the class-level RandomState).
* ``Gibbs_UNet`` (:119-139): ignores its ``alpha`` argument and uses 0.5, as the reference does.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from filters_and_operators import Fourier as _Fourier
from filters_and_operators import RandKSpaceSpikeNoise
from texbias import ops as _ops  # noqa: F401 - registers torch.ops.texbias.*
from texbias import runtime as _rt
from texbias.unet import UNet

__all__ = ["Fourier", "GibbsNoiseLayer", "Gibbs_UNet", "spike_layer", "Spikes_UNet", "UNet"]


class Fourier(_Fourier):
    """Full-spectrum helpers (:16-52), shared with filters_and_operators."""


class GibbsNoiseLayer(nn.Module, Fourier):
    """Gibbs-truncation layer; alpha = 1 is the identity (mask covers the whole grid)."""

    def __init__(self, alpha=None) -> None:
        nn.Module.__init__(self)
        if alpha is None:
            a = torch.rand(1)
        else:
            a = torch.tensor([min(max(alpha, 0.0), 1.0)], dtype=torch.float32)
        self.register_buffer("alpha", a)
        if torch.cuda.is_available():
            self.alpha = self.alpha.to(torch.device("cuda", torch.cuda.current_device()))

    @property
    def device(self) -> torch.device:
        return self.alpha.device

    def forward(self, img: torch.Tensor) -> torch.Tensor:
        if img.device.type != "cuda":
            raise _rt.TexbiasError("GibbsNoiseLayer runs on a HIP device; move the model and input to cuda")
        return torch.ops.texbias.gibbs_layer(img, self.alpha)


class Gibbs_UNet(nn.Module):
    """ResUnet with a Gibbs layer (alpha fixed at 0.5 as in the reference, :125)."""

    def __init__(self, alpha=None):
        super().__init__()
        self.gibbs = GibbsNoiseLayer(0.5)
        self.ResUnet = UNet(dimensions=3, in_channels=1, out_channels=1, channels=(16, 32, 64, 128, 256),
                            strides=(2, 2, 2, 2), num_res_units=2)

    def forward(self, img):
        return self.ResUnet(self.gibbs(img))


class spike_layer(nn.Module):
    """k-space spike at one random location shared by the batch, log-intensity ``intensity``."""

    def __init__(self, intensity):
        super().__init__()
        self.intensity = torch.tensor(intensity)

    def forward(self, x):
        v = float(self.intensity.item())
        t = RandKSpaceSpikeNoise(prob=1.0, intensity_range=(v, v), channel_wise=False)
        with torch.no_grad():
            return t(x)


class Spikes_UNet(nn.Module):
    """ResUnet with a spike layer (:154-174)."""

    def __init__(self, intensity=15):
        super().__init__()
        self.spike = spike_layer(intensity)
        self.ResUnet = UNet(dimensions=3, in_channels=1, out_channels=1, channels=(16, 32, 64, 128, 256),
                            strides=(2, 2, 2, 2), num_res_units=2)

    def forward(self, img):
        return self.ResUnet(self.spike(img))
