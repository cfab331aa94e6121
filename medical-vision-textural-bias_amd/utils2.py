"""Drop-in replacement of the reference's ``50_reconstruction/reconGan/utils2.py``.

``RandZF`` (random k-space undersampling, :34-74) runs on the texbias HIP kernels as one k-space
op (``TB_OP_ZF``): every coefficient of the full spectrum (per channel) is zeroed with
probability p and the image is returned as the real part of the inverse transform, as in the
reference.  The reference draws its mask from torch's global CPU generator
(``torch.rand(k.size())``); here each call draws one 64-bit key from that generator and the
device hashes (key, channel, frequency) into the uniform -- the same Bernoulli(1 - p) mask law,
a different stream (parity hook: ``RandZF.last_seed``, replayed by ``oracle.filters_oracle``).

``FourierTransform`` and ``weights_init`` keep the reference's definitions (:6-31, :77-83);
the former is plain torch.fft (differentiable).

``freq_consistency_loss`` is the frequency-consistency term of reconGan_freq.py:131-142,
``MSE(Re F r, Re F f) + MSE(Im F r, Im F f)`` with F the unnormalised ``fftn`` over the last two
axes, in closed form: by Parseval, ``sum |F(r - f)|^2 = H W sum |r - f|^2``, so the term equals
``H * W * MSE(r, f)`` exactly -- one fused reduction over the images instead of two forward FFTs
(and two more in the backward pass).
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn

from filters_and_operators import _kspace
from texbias import kprog as _K
from texbias.transform_base import Transform

__all__ = ["FourierTransform", "RandZF", "freq_consistency_loss", "FreqConsistencyLoss", "weights_init"]


class FourierTransform:
    """Centred FFT helpers over the trailing ``n_dims`` axes (utils2.py:6-31)."""

    @staticmethod
    def shift_fourier(x: torch.Tensor, n_dims: int) -> torch.Tensor:
        dims = tuple(range(-n_dims, 0))
        return torch.fft.fftshift(torch.fft.fftn(x, dim=dims), dim=dims)

    @staticmethod
    def inv_shift_fourier(k: torch.Tensor, n_dims: int) -> torch.Tensor:
        dims = tuple(range(-n_dims, 0))
        return torch.fft.ifftn(torch.fft.ifftshift(k, dim=dims), dim=dims).real


class RandZF(Transform, FourierTransform):
    """Zero each k-space coefficient with probability p, keep the rest (utils2.py:34-74)."""

    def __init__(self, p: float = 0):
        self.p = min(max(0, p), 1.)
        if p < 0 or p > 1:
            warnings.warn(f'Setting p to {self.p}.')
        self.last_seed = None

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        n_dims = len(img.size()[1:])
        seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
        self.last_seed = seed
        geo = _K.geometry(tuple(img.shape[1:]))
        return _kspace(img, n_dims, [_K.zf_op(self.p, seed, geo.hwd)])


def freq_consistency_loss(real: torch.Tensor, fake: torch.Tensor) -> torch.Tensor:
    """``l2(Re fftn(real), Re fftn(fake)) + l2(Im .., Im ..)`` over dims (-2, -1) with
    ``l2 = nn.MSELoss()`` (reconGan_freq.py:60, :131-142), as ``H W MSE(real, fake)`` (Parseval)."""
    if real.shape != fake.shape:
        raise ValueError(f"shape mismatch {tuple(real.shape)} vs {tuple(fake.shape)}")
    if real.dim() < 2:
        raise ValueError("need at least two (transformed) axes")
    hw = real.shape[-2] * real.shape[-1]
    return hw * nn.functional.mse_loss(fake, real)


class FreqConsistencyLoss(nn.Module):
    """Module form of :func:`freq_consistency_loss` (``forward(real, fake)``)."""

    def forward(self, real: torch.Tensor, fake: torch.Tensor) -> torch.Tensor:
        return freq_consistency_loss(real, fake)


def weights_init(m):
    """utils2.py:77-83: conv weights N(0, 0.02); BatchNorm weight N(1, 0.02), bias 0."""
    name = m.__class__.__name__
    if name.find('Conv') != -1:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif name.find('BatchNorm') != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0)
