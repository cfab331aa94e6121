"""Conv3d / ConvTranspose3d whose weight gradient runs on the texbias MFMA split-K kernel.

Forward and input-gradient stay on MIOpen/CK (``aten.convolution_backward`` with the weight
output masked off); the weight gradient of 3x3x3 layers with a long reduction (the U-Net's
full- and half-resolution levels, where MIOpen falls back to naive or non-split-K kernels at
~350 ms per layer on gfx950) goes to ``tb_conv3d_wgrad_f32``.  Parameter names and shapes are
those of ``nn.Conv3d`` / ``nn.ConvTranspose3d``, so state dicts are interchangeable.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._lib import check, lib

# use the custom weight gradient when the reduction is long relative to the output tile;
# TEXBIAS_WGRAD=0 leaves every layer to MIOpen (e.g. to compare with MIOpen's Find choice)
MIN_K_PER_OUTPUT = 64
ENABLED = os.environ.get("TEXBIAS_WGRAD", "1") != "0"


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def wgrad(G: torch.Tensor, X: torch.Tensor, w_shape, stride: int, pad: int) -> torch.Tensor:
    """dW[m][c][k^3] = corr(G, X) -- see tb_conv3d_wgrad_f32 (include/texbias.h)."""
    G = G.contiguous()
    X = X.contiguous()
    N, M = G.shape[:2]
    Cc = X.shape[1]
    dW = torch.empty((M, Cc, 3, 3, 3), dtype=torch.float32, device=G.device)
    Do, Ho, Wo = G.shape[2:]
    Di, Hi, Wi = X.shape[2:]
    with torch.cuda.device(G.device):
        check(lib().tb_conv3d_wgrad_f32(G.data_ptr(), X.data_ptr(), dW.data_ptr(), N, M, Cc, Do, Ho, Wo, Di, Hi, Wi,
                                        stride, pad, _stream(G)), "tb_conv3d_wgrad_f32")
    return dW.view(w_shape)


def fast_wgrad_applies(x: torch.Tensor, w: torch.Tensor, out_spatial, stride, padding, transposed: bool) -> bool:
    if not ENABLED or not (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32):
        return False
    if tuple(w.shape[2:]) != (3, 3, 3) or len(set(stride)) != 1 or stride[0] not in (1, 2) or len(set(padding)) != 1:
        return False
    pos = x.shape[0] * math.prod(out_spatial if not transposed else x.shape[2:])
    return pos >= MIN_K_PER_OUTPUT * w.shape[0] * w.shape[1] * 27 // 16


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding, output_padding, transposed):
        if transposed:
            y = F.conv_transpose3d(x, w, b, stride, padding, output_padding)
        else:
            y = F.conv3d(x, w, b, stride, padding)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, padding, output_padding, transposed, b is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, output_padding, transposed, has_b = ctx.cfg
        gy = gy.contiguous()
        need_x, need_w, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gx = gb = gw = None
        if need_x or (need_b and has_b):
            cout = w.shape[1] if transposed else w.shape[0]
            gx, _, gb = torch.ops.aten.convolution_backward(
                gy, x, w, [cout] if has_b else None, list(stride), list(padding), [1, 1, 1], transposed,
                list(output_padding), 1, [need_x, False, need_b and has_b])
        if need_w:
            if transposed:   # dW[ci][co] = corr(x, gy)
                gw = wgrad(x, gy, w.shape, stride[0], padding[0])
            else:            # dW[co][ci] = corr(gy, x)
                gw = wgrad(gy, x, w.shape, stride[0], padding[0])
        return gx, gw, gb, None, None, None, None


class Conv3d(nn.Conv3d):
    def forward(self, x):
        out_sp = [(n + 2 * p - 3) // s + 1 for n, p, s in zip(x.shape[2:], self.padding, self.stride)]
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                fast_wgrad_applies(x, self.weight, out_sp, self.stride, self.padding, False):
            return _ConvFn.apply(x, self.weight, self.bias, self.stride, self.padding, (0, 0, 0), False)
        return super().forward(x)


class ConvTranspose3d(nn.ConvTranspose3d):
    def forward(self, x, output_size=None):
        if output_size is None and self.groups == 1 and self.dilation == (1, 1, 1) and \
                fast_wgrad_applies(x, self.weight, None, self.stride, self.padding, True):
            return _ConvFn.apply(x, self.weight, self.bias, self.stride, self.padding, self.output_padding, True)
        return super().forward(x, output_size)
