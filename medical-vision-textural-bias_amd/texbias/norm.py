"""Fused InstanceNorm3d(affine=False) + PReLU for the U-Net's ADN blocks (HIP, texbias library).

MONAI's ``Convolution`` ("NDA": InstanceNorm3d -> Dropout(0) -> PReLU, used by the reference's
U-Net, 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199) runs under ATen as
batch_norm over [1, N*C, ...] plus separate PReLU kernels; ``instnorm_prelu`` does each direction
in two HBM sweeps (``tb_instnorm_prelu_fwd_f32`` / ``_bwd_f32``, include/texbias.h).  CUDA (HIP)
tensors only -- the library raises if it is missing; CPU tensors keep the plain module path.
"""
from __future__ import annotations

import math
import os

import torch

from ._lib import check, lib

# TEXBIAS_NORM=0 (or ENABLED = False at run time) leaves ADN blocks on ATen's InstanceNorm3d + PReLU
ENABLED = os.environ.get("TEXBIAS_NORM", "1") != "0"


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _workspace(x: torch.Tensor, nc: int) -> torch.Tensor:
    return torch.empty(int(lib().tb_instnorm_prelu_workspace_bytes(nc)), dtype=torch.uint8, device=x.device)


class _InstNormPReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, eps: float):
        x = x.contiguous()
        nc = x.shape[0] * x.shape[1]
        S = math.prod(x.shape[2:])
        y = torch.empty_like(x)
        mean = torch.empty(nc, dtype=torch.float32, device=x.device)
        rstd = torch.empty(nc, dtype=torch.float32, device=x.device)
        ws = _workspace(x, nc)
        wc = w.detach().contiguous()
        with torch.cuda.device(x.device):
            check(lib().tb_instnorm_prelu_fwd_f32(x.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                                  wc.data_ptr(), nc, S, float(eps), ws.data_ptr(), ws.numel(),
                                                  _stream(x)), "tb_instnorm_prelu_fwd_f32")
        ctx.save_for_backward(x, wc, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x, w, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous()
        nc = x.shape[0] * x.shape[1]
        S = math.prod(x.shape[2:])
        dx = torch.empty_like(x)
        dw = torch.empty(1, dtype=torch.float32, device=x.device) if ctx.needs_input_grad[1] else None
        ws = _workspace(x, nc)
        with torch.cuda.device(x.device):
            check(lib().tb_instnorm_prelu_bwd_f32(x.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                                  w.data_ptr(), dx.data_ptr(), dw.data_ptr() if dw is not None else None,
                                                  nc, S, ws.data_ptr(), ws.numel(), _stream(x)),
                  "tb_instnorm_prelu_bwd_f32")
        if dw is not None:
            dw = dw.view(ctx.saved_tensors[1].shape)
        return dx, dw, None


def instnorm_prelu(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """prelu(instance_norm(x, eps), weight) for x [N, C, *spatial] float32 on a HIP device;
    ``weight`` is PReLU's single parameter."""
    if not x.is_cuda or x.dtype != torch.float32 or weight.numel() != 1:
        raise ValueError("instnorm_prelu: float32 HIP tensor and a 1-parameter PReLU expected")
    return _InstNormPReLU.apply(x, weight, eps)
