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
from texbias import kprog as _K
from texbias import runtime as _rt
from texbias.unet import UNet

__all__ = ["Fourier", "GibbsNoiseLayer", "Gibbs_UNet", "spike_layer", "Spikes_UNet", "UNet"]


class Fourier(_Fourier):
    """Full-spectrum helpers (:16-52), shared with filters_and_operators."""


class _LayerFilter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img: torch.Tensor, alpha: torch.Tensor, spatial):
        ctx.spatial = spatial
        ctx.save_for_backward(alpha)
        return _layer_apply(img, alpha, spatial)

    @staticmethod
    def backward(ctx, gy):
        (alpha,) = ctx.saved_tensors
        gx = _layer_apply(gy.contiguous(), alpha, ctx.spatial) if ctx.needs_input_grad[0] else None
        ga = torch.zeros_like(alpha) if ctx.needs_input_grad[1] else None
        return gx, ga, None


def _layer_apply(img: torch.Tensor, alpha: torch.Tensor, spatial) -> torch.Tensor:
    B = img.shape[0]
    n_dims = img.dim() - 1
    a = alpha.detach().reshape(-1)[:1].to(device=img.device, dtype=torch.float32).contiguous()
    prog = [_K.layer_op(0.0, spatial, alpha_ptr=a.data_ptr())]
    x = img if img.dtype == torch.float32 else img.float()
    # `a` aliases the alpha buffer (or is a stream-ordered temporary): the caching allocator only
    # hands its memory to work queued after this launch, so the kernel's read is safe.
    y = _rt.kspace_filter(x.reshape((B, 1) + tuple(img.shape[1:])), n_dims, [prog] * B, 1)
    return y.reshape(img.shape)


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
        return _LayerFilter.apply(img, self.alpha, tuple(img.shape[1:]))


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
