"""DiceLoss as the reference configures it: ``DiceLoss(to_onehot_y=False, sigmoid=True,
squared_pred=True)`` (e.g. stylized_gibbs12p5.py:201), MONAI 0.5 semantics: per (batch, channel)
``1 - (2 sum(p t) + 1e-5) / (sum(t^2) + sum(p^2) + 1e-5)`` over the spatial axes, p = sigmoid(x),
mean-reduced.  Parity with MONAI is unpinned (MONAI is absent in this image); the formula is
MONAI's published one.
"""
from __future__ import annotations

import torch
import torch.nn as nn


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
