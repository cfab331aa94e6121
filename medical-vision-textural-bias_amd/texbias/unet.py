"""3-D residual U-Net equivalent to the MONAI 0.5 ``UNet`` the reference trains.

The reference builds ``monai.networks.nets.UNet(dimensions=3, in_channels, out_channels,
channels=(16, 32, 64, 128, 256), strides=(2, 2, 2, 2), num_res_units=2)``
(e.g. 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199).  MONAI is not a
dependency here; the module tree below reproduces the architecture printed in
source_code/test.ipynb:754-1010 (cell 21) module for module, so parameter shapes,
counts and default initialisation match (parity with MONAI's numerics is unpinned:
MONAI is not installed in this image).

Blocks (MONAI 0.5 semantics):
* ``Convolution`` = Conv3d / ConvTranspose3d -> InstanceNorm3d(affine=False) -> Dropout(0) -> PReLU
  ("NDA" order; on HIP tensors one fused texbias kernel pair, ``texbias.norm``), or the bare conv
  when ``conv_only``;
* ``ResidualUnit`` = ``subunits`` Convolutions (first one strided) + residual path (strided 3^3
  conv, 1^3 conv when only the channel count changes, else identity), summed;
* ``SkipConnection`` = cat([x, sub(x)], dim=1).

It runs on PyTorch-ROCm (MIOpen/CK forward and input-gradient convolutions); the weight
gradient of the long-reduction 3x3x3 layers runs on the texbias split-K MFMA kernel
(``texbias.conv``), the one U-Net op where MIOpen has no usable gfx950 path.
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn

from .conv import Conv3d, ConvTranspose3d
from . import norm as _norm
from .norm import instnorm_prelu


class ADN(nn.Sequential):
    def __init__(self, channels: int, dropout: float = 0.0):
        super().__init__()
        self.add_module("N", nn.InstanceNorm3d(channels, eps=1e-5, affine=False, track_running_stats=False))
        self.add_module("D", nn.Dropout(p=dropout))
        self.add_module("A", nn.PReLU(num_parameters=1))

    def forward(self, x):
        # On the GPU the N -> D(0) -> A chain is one fused texbias op (two HBM sweeps per direction).
        if _norm.ENABLED and x.is_cuda and x.dtype == torch.float32 and (self.D.p == 0.0 or not self.training):
            return instnorm_prelu(x, self.A.weight, self.N.eps)
        return super().forward(x)


class Convolution(nn.Sequential):
    def __init__(self, cin: int, cout: int, strides: int = 1, kernel_size: int = 3, conv_only: bool = False,
                 is_transposed: bool = False, dropout: float = 0.0):
        super().__init__()
        pad = (kernel_size - 1) // 2
        if is_transposed:
            conv = ConvTranspose3d(cin, cout, kernel_size, stride=strides, padding=pad, output_padding=strides - 1)
        else:
            conv = Conv3d(cin, cout, kernel_size, stride=strides, padding=pad)
        self.add_module("conv", conv)
        if not conv_only:
            self.add_module("adn", ADN(cout, dropout))


class ResidualUnit(nn.Module):
    def __init__(self, cin: int, cout: int, strides: int = 1, kernel_size: int = 3, subunits: int = 2,
                 last_conv_only: bool = False, dropout: float = 0.0):
        super().__init__()
        self.conv = nn.Sequential()
        sch, sst = cin, strides
        subunits = max(1, subunits)
        for su in range(subunits):
            conv_only = last_conv_only and su == subunits - 1
            self.conv.add_module(f"unit{su}", Convolution(sch, cout, sst, kernel_size, conv_only=conv_only,
                                                          dropout=dropout))
            sch, sst = cout, 1
        if strides != 1 or cin != cout:
            k, p = (kernel_size, (kernel_size - 1) // 2) if strides != 1 else (1, 0)
            self.residual = Conv3d(cin, cout, k, stride=strides, padding=p)
        else:
            self.residual = nn.Identity()

    def forward(self, x):
        res = self.residual(x)
        return self.conv(x) + res


class SkipConnection(nn.Module):
    def __init__(self, submodule: nn.Module):
        super().__init__()
        self.submodule = submodule

    def forward(self, x):
        return torch.cat([x, self.submodule(x)], dim=1)


class UNet(nn.Module):
    """``UNet(dimensions=3, in_channels, out_channels, channels, strides, num_res_units=2)``."""

    def __init__(self, dimensions: int = 3, in_channels: int = 1, out_channels: int = 1,
                 channels: Sequence[int] = (16, 32, 64, 128, 256), strides: Sequence[int] = (2, 2, 2, 2),
                 kernel_size: int = 3, up_kernel_size: int = 3, num_res_units: int = 2, dropout: float = 0.0):
        super().__init__()
        if dimensions != 3:
            raise ValueError("only the 3-D U-Net of the reference is provided")
        if len(channels) < 2 or len(strides) != len(channels) - 1:
            raise ValueError("len(strides) must be len(channels) - 1 >= 1")
        if num_res_units < 1:
            raise ValueError("the reference configuration uses residual units (num_res_units >= 1)")
        self.nru, self.k, self.uk, self.dropout = num_res_units, kernel_size, up_kernel_size, dropout

        def block(cin, cout, chs, sts, is_top):
            c, s = chs[0], sts[0]
            if len(chs) > 2:
                sub = block(c, c, chs[1:], sts[1:], False)
                upc = c * 2
            else:
                sub = self._down(c, chs[1], 1)
                upc = c + chs[1]
            return nn.Sequential(self._down(cin, c, s), SkipConnection(sub), self._up(upc, cout, s, is_top))

        self.model = block(in_channels, out_channels, tuple(channels), tuple(strides), True)

    def _down(self, cin, cout, s):
        return ResidualUnit(cin, cout, s, self.k, self.nru, dropout=self.dropout)

    def _up(self, cin, cout, s, is_top):
        conv = Convolution(cin, cout, s, self.uk, conv_only=False, is_transposed=True, dropout=self.dropout)
        ru = ResidualUnit(cout, cout, 1, self.k, subunits=1, last_conv_only=is_top, dropout=self.dropout)
        return nn.Sequential(conv, ru)

    def forward(self, x):
        return self.model(x)
