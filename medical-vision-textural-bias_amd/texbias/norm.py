"""Fused InstanceNorm3d(affine=False) + PReLU for the U-Net's ADN blocks (HIP, texbias library).

MONAI's ``Convolution`` ("NDA": InstanceNorm3d -> Dropout(0) -> PReLU, used by the reference's
U-Net, 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:192-199) runs under ATen as
batch_norm over [1, N*C, ...] plus separate PReLU kernels; here each direction is two HBM sweeps
(``tb_adn_fwd_f32`` / ``tb_adn_bwd_f32``, include/texbias.h): no accumulator memsets, deterministic
block-ordered reductions, optional channel-slice (batch-strided) operands, the ResidualUnit's sum fused
into the forward store and the preceding convolution's bias gradient out of the backward's store pass
(``adn_forward`` / ``adn_backward``, used by the fused units of ``texbias.unet``).  CUDA (HIP) tensors
only -- the library raises if it is missing; CPU tensors keep the plain module path.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch

from ._lib import check, lib

# TEXBIAS_NORM=0 (or ENABLED = False at run time) leaves ADN blocks on ATen's InstanceNorm3d + PReLU
ENABLED = os.environ.get("TEXBIAS_NORM", "1") != "0"

_COUNTERS = {}


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def counters(device: torch.device, n: int) -> torch.Tensor:
    """Persistent zeroed uint32 counters for the ADN kernels on (device, current stream); the kernels
    leave them zero.  Grown (re-zeroed) on demand."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    c = _COUNTERS.get(key)
    if c is None or c.numel() < n:
        c = torch.zeros(max(n, 4096), dtype=torch.int32, device=device)
        _COUNTERS[key] = c
    return c


def _sn(t: Optional[torch.Tensor], S: int) -> int:
    """Batch stride of a [N, C, *spatial] operand whose channels are contiguous S-voxel planes."""
    if t is None:
        return 0
    N, C = t.shape[:2]
    if t.stride(1) != S or math.prod(t.shape[2:]) != S or not t[0, 0].is_contiguous():
        raise ValueError("ADN operand: each channel must be one contiguous plane of S voxels")
    return t.stride(0)


def _plain(t: torch.Tensor) -> torch.Tensor:
    S = math.prod(t.shape[2:])
    try:
        _sn(t, S)
        return t
    except ValueError:
        return t.contiguous()


def adn_forward(x: torch.Tensor, w: torch.Tensor, eps: float, res: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """y = prelu(instance_norm(x, eps), w) (+ res); returns (y, mean, rstd).  x, res, out may be channel
    slices of wider tensors."""
    x = _plain(x)
    N, C = x.shape[:2]
    S = math.prod(x.shape[2:])
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device) if out is None else out
    if res is not None:
        res = _plain(res)
    mean = torch.empty(N * C, dtype=torch.float32, device=x.device)
    rstd = torch.empty(N * C, dtype=torch.float32, device=x.device)
    nb = int(lib().tb_adn_workspace_bytes(N, C, S))
    ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    cnt = counters(x.device, int(lib().tb_adn_counters(N, C)))
    wc = w.detach()
    with torch.cuda.device(x.device):
        check(lib().tb_adn_fwd_f32(x.data_ptr(), _sn(x, S), y.data_ptr(), _sn(y, S),
                                   res.data_ptr() if res is not None else None, _sn(res, S), mean.data_ptr(),
                                   rstd.data_ptr(), wc.data_ptr(), N, C, S, float(eps), ws.data_ptr(), nb,
                                   cnt.data_ptr(), _stream(x)), "tb_adn_fwd_f32")
    return y, mean, rstd


def adn_backward(x: torch.Tensor, dy: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor, w: torch.Tensor,
                 need_w: bool = True, need_bias: bool = False, dx_out: Optional[torch.Tensor] = None,
                 dysum_out: Optional[torch.Tensor] = None):
    """(dx, dw or None, dbias or None): the ADN's input gradient, its PReLU weight gradient and the
    bias gradient of the convolution that produced x (dx summed over n and the voxels).  ``dysum_out``
    (float32 [C], optional) receives dy summed over n and the voxels out of the same sweep (the bias
    gradient of a residual convolution added to this block's output)."""
    x = _plain(x)
    dy = _plain(dy)
    N, C = x.shape[:2]
    S = math.prod(x.shape[2:])
    dx = torch.empty(x.shape, dtype=torch.float32, device=x.device) if dx_out is None else dx_out
    dw = torch.empty(1, dtype=torch.float32, device=x.device) if need_w else None
    db = torch.empty(C, dtype=torch.float32, device=x.device) if need_bias else None
    nb = int(lib().tb_adn_workspace_bytes(N, C, S))
    ws = torch.empty(nb, dtype=torch.uint8, device=x.device)
    cnt = counters(x.device, int(lib().tb_adn_counters(N, C)))
    with torch.cuda.device(x.device):
        check(lib().tb_adn_bwd_f32(x.data_ptr(), _sn(x, S), dy.data_ptr(), _sn(dy, S), dx.data_ptr(), _sn(dx, S),
                                   mean.data_ptr(), rstd.data_ptr(), w.detach().data_ptr(),
                                   dw.data_ptr() if dw is not None else None,
                                   db.data_ptr() if db is not None else None,
                                   dysum_out.data_ptr() if dysum_out is not None else None, N, C, S, ws.data_ptr(), nb,
                                   cnt.data_ptr(), _stream(x)), "tb_adn_bwd_f32")
    if dw is not None:
        dw = dw.view(w.shape)
    return dx, dw, db


class _InstNormPReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, eps: float):
        x = x.contiguous()
        y, mean, rstd = adn_forward(x, w, eps)
        ctx.save_for_backward(x, w, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        x, w, mean, rstd = ctx.saved_tensors
        dx, dw, _ = adn_backward(x, dy, mean, rstd, w, need_w=ctx.needs_input_grad[1])
        return dx, dw, None


def instnorm_prelu(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    """prelu(instance_norm(x, eps), weight) for x [N, C, *spatial] float32 on a HIP device;
    ``weight`` is PReLU's single parameter."""
    if not x.is_cuda or x.dtype != torch.float32 or weight.numel() != 1:
        raise ValueError("instnorm_prelu: float32 HIP tensor and a 1-parameter PReLU expected")
    return _InstNormPReLU.apply(x, weight, eps)
