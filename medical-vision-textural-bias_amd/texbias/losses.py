"""DiceLoss as the reference configures it: ``DiceLoss(to_onehot_y=False, sigmoid=True,
squared_pred=True)`` (e.g. stylized_gibbs12p5.py:201), MONAI 0.5 semantics: per (batch, channel)
``1 - (2 sum(p t) + 1e-5) / (sum(t^2) + sum(p^2) + 1e-5)`` over the spatial axes, p = sigmoid(x),
mean-reduced.  Parity with MONAI is unpinned (MONAI is absent in this image); the formula is
MONAI's published one.  On HIP tensors the three per-instance sums come from one fused sweep
(``tb_dice_sums_ws_f32``, float64 block partials summed in block order: deterministic) with a fused backward (``tb_dice_sums_bwd_f32``), and the
finalize (the formula and its reduction, forward and backward) is one launch each way
(``tb_dice_loss_f32`` / ``tb_dice_loss_bwd_f32``).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from ._lib import check, lib

# TEXBIAS_DICE=0 (or ENABLED = False at run time) computes the sums with plain ATen reductions
ENABLED = os.environ.get("TEXBIAS_DICE", "1") != "0"


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _dice_sums(x, t, sums, nc: int, S: int, sigmoid: bool, squared: bool, stream: int) -> None:
    """sums[nc][3] = {sum t p, sum t^2 | t, sum p^2 | p} per instance (tb_dice_sums_ws_f32)."""
    nb = int(lib().tb_dice_sums_ws_bytes(nc, S))
    ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    check(lib().tb_dice_sums_ws_f32(x.data_ptr(), t.data_ptr(), sums.data_ptr(), nc, S, int(sigmoid), int(squared),
                                    ws.data_ptr(), nb, stream), "tb_dice_sums_ws_f32")


class _DiceSums(torch.autograd.Function):
    """(x, t) [N, C, *spatial] -> [N, C, 3] float32 sums {t p, t^2 | t, p^2 | p}, p = sigmoid(x)?"""

    @staticmethod
    def forward(ctx, x, t, sigmoid: bool, squared: bool):
        x, t = x.contiguous(), t.contiguous()
        nc, S = x.shape[0] * x.shape[1], math.prod(x.shape[2:])
        sums = torch.empty((x.shape[0], x.shape[1], 3), dtype=torch.float64, device=x.device)
        with torch.cuda.device(x.device):
            _dice_sums(x, t, sums, nc, S, sigmoid, squared, _stream(x))
        ctx.save_for_backward(x, t)
        ctx.cfg = (sigmoid, squared)
        return sums.float()

    @staticmethod
    def backward(ctx, g):
        x, t = ctx.saved_tensors
        sigmoid, squared = ctx.cfg
        g = g.contiguous().float()
        dx = torch.empty_like(x)
        nc, S = x.shape[0] * x.shape[1], math.prod(x.shape[2:])
        with torch.cuda.device(x.device):
            check(lib().tb_dice_sums_bwd_f32(x.data_ptr(), t.data_ptr(), g.data_ptr(), dx.data_ptr(), nc, S,
                                             int(sigmoid), int(squared), _stream(x)), "tb_dice_sums_bwd_f32")
        return dx, None, None, None


class _DiceLossFn(torch.autograd.Function):
    """The whole HIP DiceLoss: the fused sums sweep, then the finalize (f per instance / channel and its
    reduction) in one launch (``tb_dice_loss_f32``); backward: the sums' gradients in one launch
    (``tb_dice_loss_bwd_f32``), then the fused input-gradient sweep."""

    @staticmethod
    def forward(ctx, x, t, sigmoid: bool, squared: bool, batch: bool, red: int, nr: float, dr: float):
        x, t = x.contiguous(), t.contiguous()
        N, Cc = x.shape[0], x.shape[1]
        nc, S = N * Cc, math.prod(x.shape[2:])
        sums = torch.empty((N, Cc, 3), dtype=torch.float64, device=x.device)
        oshape = () if red else ((Cc,) if batch else (N, Cc))
        loss = torch.empty(oshape, dtype=torch.float32, device=x.device)
        with torch.cuda.device(x.device):
            st = _stream(x)
            _dice_sums(x, t, sums, nc, S, sigmoid, squared, st)
            check(lib().tb_dice_loss_f32(sums.data_ptr(), loss.data_ptr(), nc, Cc, int(batch), red, nr, dr, st),
                  "tb_dice_loss_f32")
        ctx.save_for_backward(x, t, sums)
        ctx.cfg = (sigmoid, squared, batch, red, nr, dr)
        return loss

    @staticmethod
    def backward(ctx, gl):
        x, t, sums = ctx.saved_tensors
        sigmoid, squared, batch, red, nr, dr = ctx.cfg
        gl = gl.contiguous().float()
        nc, S = x.shape[0] * x.shape[1], math.prod(x.shape[2:])
        gs = torch.empty((nc, 3), dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        with torch.cuda.device(x.device):
            st = _stream(x)
            check(lib().tb_dice_loss_bwd_f32(sums.data_ptr(), gl.data_ptr(), gs.data_ptr(), nc, x.shape[1], int(batch),
                                             red, nr, dr, st), "tb_dice_loss_bwd_f32")
            check(lib().tb_dice_sums_bwd_f32(x.data_ptr(), t.data_ptr(), gs.data_ptr(), dx.data_ptr(), nc, S,
                                             int(sigmoid), int(squared), st), "tb_dice_sums_bwd_f32")
        return dx, None, None, None, None, None, None, None


_REDUCTIONS = {"none": 0, "mean": 1, "sum": 2}


class DiceLoss(nn.Module):
    def __init__(self, include_background: bool = True, to_onehot_y: bool = False, sigmoid: bool = False,
                 softmax: bool = False, squared_pred: bool = False, jaccard: bool = False,
                 reduction: str = "mean", smooth_nr: float = 1e-5, smooth_dr: float = 1e-5, batch: bool = False):
        super().__init__()
        if to_onehot_y or softmax or jaccard or not include_background:
            raise NotImplementedError("only the reference's configuration is provided")
        self.sigmoid, self.squared = sigmoid, squared_pred
        self.reduction, self.nr, self.dr, self.batch = reduction, smooth_nr, smooth_dr, batch

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if input.shape != target.shape:
            raise AssertionError(f"ground truth has differing shape ({target.shape}) from input ({input.shape})")
        if ENABLED and input.is_cuda and input.dtype == torch.float32 and target.dtype == torch.float32 and \
                input.dim() > 2 and self.reduction in _REDUCTIONS:
            return _DiceLossFn.apply(input, target, self.sigmoid, self.squared, self.batch,
                                     _REDUCTIONS[self.reduction], self.nr, self.dr)
        if ENABLED and input.is_cuda and input.dtype == torch.float32 and target.dtype == torch.float32 and \
                input.dim() > 2:
            s = _DiceSums.apply(input, target, self.sigmoid, self.squared)
            if self.batch:
                s = s.sum(0)
            inter, go, po = s[..., 0], s[..., 1], s[..., 2]
        else:
            p = torch.sigmoid(input) if self.sigmoid else input
            axes = list(range(2, p.dim()))
            if self.batch:
                axes = [0] + axes
            inter = torch.sum(target * p, dim=axes)
            if self.squared:
                go, po = torch.sum(target * target, dim=axes), torch.sum(p * p, dim=axes)
            else:
                go, po = torch.sum(target, dim=axes), torch.sum(p, dim=axes)
        f = 1.0 - (2.0 * inter + self.nr) / (go + po + self.dr)
        if self.reduction == "mean":
            return f.mean()
        if self.reduction == "sum":
            return f.sum()
        return f
