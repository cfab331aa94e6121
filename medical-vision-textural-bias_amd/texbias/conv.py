"""Conv3d / ConvTranspose3d whose weight gradient runs on the texbias MFMA split-K kernel.

Forward and input-gradient stay on MIOpen/CK (``aten.convolution_backward`` with the weight
and bias outputs masked off); the weight gradient of 3x3x3 layers with a long reduction (the
U-Net's full- and half-resolution levels, where MIOpen falls back to naive or non-split-K kernels
at ~350 ms per layer on gfx950) goes to ``tb_conv3d_wgrad_f32``, and every bias gradient (grad_out
summed over N, D, H, W -- ATen's generic reduction ran at 0.1-0.3 TB/s, ~7 ms of a 46 ms step) to
``tb_channel_sum_f32``.  Parameter names and shapes are those of ``nn.Conv3d`` /
``nn.ConvTranspose3d``, so state dicts are interchangeable.
"""
from __future__ import annotations

import functools
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
CONVT64 = os.environ.get("TEXBIAS_CONVT64", "1") != "0"
CONVMFMA = os.environ.get("TEXBIAS_CONVMFMA", "1") != "0"


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


def wgrad_config(g_shape, x_shape, stride: int, pad: int = 1) -> dict:
    """The tiling ``wgrad`` picks for G [N, M, Do, Ho, Wo] / X [N, Cc, Di, Hi, Wi] (host only,
    tb_conv3d_wgrad_config): SEG, TX, YB, chunks, lds_bytes."""
    import ctypes
    cfg = (ctypes.c_int64 * 5)()
    N, M, Do, Ho, Wo = g_shape
    Cc, Di, Hi, Wi = x_shape[1:]
    check(lib().tb_conv3d_wgrad_config(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad, cfg), "tb_conv3d_wgrad_config")
    return dict(zip(("SEG", "TX", "YB", "chunks", "lds_bytes"), list(cfg)))


def channel_sum(g: torch.Tensor) -> torch.Tensor:
    """g [N, C, *spatial] -> [C]: sum over N and the spatial axes (tb_channel_sum_f32)."""
    g = g.contiguous()
    N, Cc = g.shape[:2]
    out = torch.empty(Cc, dtype=torch.float32, device=g.device)
    with torch.cuda.device(g.device):
        check(lib().tb_channel_sum_f32(g.data_ptr(), out.data_ptr(), N, Cc, g[0, 0].numel(), _stream(g)),
              "tb_channel_sum_f32")
    return out


def custom_backward_applies(x: torch.Tensor, w: torch.Tensor) -> bool:
    """float32 HIP tensors: the layer's backward goes through _ConvFn (texbias bias/weight grads)."""
    return ENABLED and x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32


@functools.lru_cache(maxsize=256)
def _wgrad_tiles(g_shape, x_shape, stride: int) -> bool:
    """A tiling of tb_conv3d_wgrad_f32 exists for these shapes (tb_conv3d_wgrad_config, host only):
    rows too wide for the LDS budget at the channel tile go to ATen instead of failing."""
    import ctypes
    cfg = (ctypes.c_int64 * 5)()
    N, M, Do, Ho, Wo = g_shape
    Cc, Di, Hi, Wi = x_shape[1:]
    return lib().tb_conv3d_wgrad_config(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, 1, cfg) == 0


def fast_wgrad_applies(x: torch.Tensor, w: torch.Tensor, out_spatial, stride, padding, transposed: bool,
                       output_padding=(0, 0, 0)) -> bool:
    if not custom_backward_applies(x, w):
        return False
    if tuple(w.shape[2:]) != (3, 3, 3) or len(set(stride)) != 1 or stride[0] not in (1, 2) or padding[0] != 1 or \
            len(set(padding)) != 1:
        return False
    pos = x.shape[0] * math.prod(out_spatial if not transposed else x.shape[2:])
    if pos < MIN_K_PER_OUTPUT * w.shape[0] * w.shape[1] * 27 // 16:
        return False
    s = stride[0]
    if transposed:  # G = x [N, Cin, ...], X = grad of the output [N, Cout, (n - 1) s + 1 + output_padding]
        hi = tuple((n - 1) * s + 1 + op for n, op in zip(x.shape[2:], output_padding))
        return _wgrad_tiles(tuple(x.shape), (x.shape[0], w.shape[1]) + hi, s)
    return _wgrad_tiles((x.shape[0], w.shape[0]) + tuple(out_spatial), tuple(x.shape), s)


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, padding, output_padding, transposed, fast_w):
        if transposed and convT64_applies(x, w, stride, padding, output_padding):
            y = convT_mfma(x, w, b)
        elif transposed:
            y = F.conv_transpose3d(x, w, b, stride, padding, output_padding)
        else:
            y = F.conv3d(x, w, b, stride, padding)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, padding, output_padding, transposed, b is not None, fast_w)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, output_padding, transposed, has_b, fast_w = ctx.cfg
        gy = gy.contiguous()
        need_x, need_w, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gx = gb = gw = None
        lib_w = need_w and not fast_w
        if need_x and not transposed and s2_dgrad_applies(gy, x, w, stride, padding):
            gx = convT_mfma(gy, w, None)  # Conv3d(16 -> 32, s2)'s input gradient on k_convT_mfma64
            need_x = False
        if need_x or lib_w:
            gxl, gw, _ = torch.ops.aten.convolution_backward(
                gy, x, w, None, list(stride), list(padding), [1, 1, 1], transposed, list(output_padding), 1,
                [need_x, lib_w, False])
            gx = gxl if need_x else gx
        if need_w and fast_w:
            if transposed:   # dW[ci][co] = corr(x, gy)
                gw = wgrad(x, gy, w.shape, stride[0], padding[0])
            else:            # dW[co][ci] = corr(gy, x)
                gw = wgrad(gy, x, w.shape, stride[0], padding[0])
        if need_b and has_b:
            gb = channel_sum(gy)
        return gx, gw, gb, None, None, None, None, None


def small_conv(x: torch.Tensor, w: torch.Tensor, b) -> torch.Tensor:
    """Direct 3x3x3, stride 1, padding 1 convolution for <= 4 channels (tb_conv3d_small_f32)."""
    x = x.contiguous()
    w = w.contiguous()
    N, Cin, D, H, W = x.shape
    Cout = w.shape[0]
    y = torch.empty((N, Cout, D, H, W), dtype=torch.float32, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_small_f32(x.data_ptr(), w.data_ptr(), b.data_ptr() if b is not None else None,
                                        y.data_ptr(), N, Cin, Cout, D, H, W, _stream(x)), "tb_conv3d_small_f32")
    return y


def small_conv_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3) and \
        tuple(stride) == (1, 1, 1) and tuple(padding) == (1, 1, 1) and w.shape[0] <= 4 and w.shape[1] <= 4 and \
        x.shape[-1] <= 168


class _SmallConvFn(torch.autograd.Function):
    """Few-channel stride-1 3x3x3 Conv3d: forward and input gradient on the direct kernel, weight
    gradient on the split-K MFMA kernel, bias gradient on the channel-sum kernel."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = small_conv(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = small_conv(gy, w.flip(2, 3, 4).transpose(0, 1).contiguous(), None)
        if ctx.needs_input_grad[1]:
            gw = wgrad(gy, x, w.shape, 1, 1)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = channel_sum(gy)
        return gx, gw, gb


# ---------------------------------------------------------------- full-resolution stride-2 layers
def s2_pairs(wm: torch.Tensor) -> torch.Tensor:
    """[Mout, Cin, 3, 3, 3] -> the kernel's output-channel pairs [Mout / 2, Cin 27, 2]."""
    m = wm.shape[0]
    return wm.reshape(m // 2, 2, -1).permute(0, 2, 1).contiguous()


def conv_s2_fewin(inp: torch.Tensor, K: torch.Tensor, b, mout: int) -> torch.Tensor:
    """out[n][m][o] = b[m] + sum_{c, t} Wm[m][c][t] inp[n][c][2 o + t - 1] (3x3x3, stride 2, padding 1;
    tb_conv3d_s2_fewin_f32).  inp [N, Cin <= 4, 2 Do, 2 Ho, 2 Wo], K = s2_pairs(Wm)."""
    inp = inp.contiguous()
    N, Cin, Di, Hi, Wi = inp.shape
    out = torch.empty((N, mout, Di // 2, Hi // 2, Wi // 2), dtype=torch.float32, device=inp.device)
    with torch.cuda.device(inp.device):
        check(lib().tb_conv3d_s2_fewin_f32(inp.data_ptr(), K.data_ptr(), b.data_ptr() if b is not None else None,
                                           out.data_ptr(), N, Cin, mout, Di // 2, Hi // 2, Wi // 2, _stream(inp)),
              "tb_conv3d_s2_fewin_f32")
    return out


def convT_fewout(x: torch.Tensor, w: torch.Tensor, b) -> torch.Tensor:
    """ConvTranspose3d(Cin -> Cout <= 4, 3, stride 2, padding 1, output_padding 1) forward
    (tb_convT3d_fewout_f32; w as the module holds it, [Cin, Cout, 3, 3, 3])."""
    x = x.contiguous()
    N, Cin, D, H, W = x.shape
    Cout = w.shape[1]
    y = torch.empty((N, Cout, 2 * D, 2 * H, 2 * W), dtype=torch.float32, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_convT3d_fewout_f32(x.data_ptr(), w.contiguous().data_ptr(),
                                          b.data_ptr() if b is not None else None, y.data_ptr(), N, Cin, Cout, D, H,
                                          W, _stream(x)), "tb_convT3d_fewout_f32")
    return y


def _s2_shape_ok(spatial) -> bool:
    D, H, W = spatial
    return D % 2 == 0 and H % 2 == 0 and W % 4 == 0 and W <= 160  # (the weight gradient's z-march: W <= 160)


def s2_fewin_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    """Conv3d(Cin <= 4 -> 16 or 32, 3, stride 2, padding 1) on even spatial dims: k_conv_s2_fewin."""
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3) and \
        tuple(stride) == (2, 2, 2) and tuple(padding) == (1, 1, 1) and w.shape[1] <= 4 and \
        w.shape[0] in (16, 32) and _s2_shape_ok(x.shape[2:]) and x.data_ptr() % 16 == 0


def convT_fewout_applies(x: torch.Tensor, w: torch.Tensor, stride, padding, output_padding) -> bool:
    """ConvTranspose3d(Cin <= 32 -> Cout <= 4, 3, 2, 1, output_padding 1): forward on k_convT_fewout and
    input gradient on k_conv_s2_fewin (needs Cin 16 or 32)."""
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3) and \
        tuple(stride) == (2, 2, 2) and tuple(padding) == (1, 1, 1) and tuple(output_padding) == (1, 1, 1) and \
        w.shape[1] <= 4 and w.shape[0] in (16, 32) and x.shape[-1] % 4 == 0 and x.shape[-1] <= 80 and \
        _s2_shape_ok(tuple(2 * n for n in x.shape[2:]))


class _ConvS2FewInFn(torch.autograd.Function):
    """Conv3d(Cin <= 4, stride 2): forward on the direct stride-2 kernel; weight gradient on the
    z-marching MFMA kernel, bias gradient on the channel-sum kernel, input gradient (rarely needed:
    the first layer's input is data) on ATen."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = conv_s2_fewin(x, s2_pairs(w), b, w.shape[0])
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx, _, _ = torch.ops.aten.convolution_backward(gy, x, w, None, [2, 2, 2], [1, 1, 1], [1, 1, 1], False,
                                                           [0, 0, 0], 1, [True, False, False])
        if ctx.needs_input_grad[1]:
            gw = wgrad(gy, x, w.shape, 2, 1)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = channel_sum(gy)
        return gx, gw, gb


class _ConvTFewOutFn(torch.autograd.Function):
    """ConvTranspose3d(Cin -> Cout <= 4, stride 2): forward on the sub-pixel kernel, input gradient (a
    stride-2 convolution of dY with Cout input channels) on the direct stride-2 kernel, weight gradient
    on the z-marching MFMA kernel, bias gradient on the channel-sum kernel."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = convT_fewout(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:  # dX[m][i] = sum_{c, t} W[m][c][t] dY[c][2 i + t - 1]
            gx = conv_s2_fewin(gy, s2_pairs(w), None, w.shape[0])
        if ctx.needs_input_grad[1]:  # dW[ci][co] = corr(x, dY)
            gw = wgrad(x, gy, w.shape, 2, 1)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = channel_sum(gy)
        return gx, gw, gb


def convT_mfma(x: torch.Tensor, w: torch.Tensor, b) -> torch.Tensor:
    """ConvTranspose3d(Cin -> 16, 3, stride 2, padding 1, output_padding 1), Cin = 32 or 64, forward on the
    f32 matrix cores (tb_convT3d_mfma_f32; w [Cin, 16, 3, 3, 3] as the module holds it)."""
    x = x.contiguous()
    N, Cin, D, H, W = x.shape
    y = torch.empty((N, 16, 2 * D, 2 * H, 2 * W), dtype=torch.float32, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_convT3d_mfma_f32(x.data_ptr(), w.contiguous().data_ptr(),
                                        b.data_ptr() if b is not None else None, y.data_ptr(), N, Cin, D, H, W,
                                        _stream(x)), "tb_convT3d_mfma_f32")
    return y


convT_mfma64 = convT_mfma


def s2_dgrad_applies(gy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    """Conv3d(16 -> 32, 3, stride 2, padding 1) on even extents: its input gradient is
    conv_transpose3d(dY, W) with output_padding 1, i.e. k_convT_mfma64 with 32 input channels."""
    return CONVT64 and tuple(w.shape) == (32, 16, 3, 3, 3) and tuple(stride) == (2, 2, 2) and \
        tuple(padding) == (1, 1, 1) and gy.dim() == 5 and all(2 * a == b for a, b in zip(gy.shape[2:], x.shape[2:])) and \
        gy.shape[-1] % 4 == 0 and gy.shape[-1] <= 64 and gy.data_ptr() % 16 == 0


def convT64_applies(x: torch.Tensor, w: torch.Tensor, stride, padding, output_padding) -> bool:
    """ConvTranspose3d(64 -> 16, 3, 2, 1, output_padding 1), rows of 4k <= 64 floats: forward on
    k_convT_mfma64 (TEXBIAS_CONVT64=0: ATen).  Input and weight gradients stay where _ConvFn puts them."""
    return CONVT64 and custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape) == (64, 16, 3, 3, 3) and \
        tuple(stride) == (2, 2, 2) and tuple(padding) == (1, 1, 1) and tuple(output_padding) == (1, 1, 1) and \
        x.shape[-1] % 4 == 0 and x.shape[-1] <= 64 and x.data_ptr() % 16 == 0


def conv_fwd16(x: torch.Tensor, w: torch.Tensor, b) -> torch.Tensor:
    """Conv3d(16 -> 16, 3, stride 1, padding 1) forward on the f32 matrix cores (tb_conv3d_fwd16_f32)."""
    x = x.contiguous()
    N, _, D, H, W = x.shape
    y = torch.empty_like(x)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_fwd16_f32(x.data_ptr(), w.contiguous().data_ptr(), b.data_ptr() if b is not None else None,
                                        y.data_ptr(), N, D, H, W, _stream(x)), "tb_conv3d_fwd16_f32")
    return y


def conv16_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    """Conv3d(16 -> 16, 3, stride 1, padding 1), rows of 16k <= 128 floats: k_conv3d_fwd16 (forward and
    input gradient) + the z-marching weight gradient."""
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape) == (16, 16, 3, 3, 3) and \
        tuple(stride) == (1, 1, 1) and tuple(padding) == (1, 1, 1) and x.shape[-1] % 16 == 0 and \
        x.shape[-1] <= 80 and x.data_ptr() % 16 == 0 and os.environ.get("TEXBIAS_CONV16", "1") != "0"


class _Conv16Fn(torch.autograd.Function):
    """Conv3d(16 -> 16, stride 1): forward and input gradient (flipped, transposed weights) on the MFMA
    kernel, weight gradient on the z-marching MFMA kernel, bias gradient on the channel-sum kernel."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = conv_fwd16(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = conv_fwd16(gy, w.flip(2, 3, 4).transpose(0, 1).contiguous(), None)
        if ctx.needs_input_grad[1]:
            gw = wgrad(gy, x, w.shape, 1, 1)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = channel_sum(gy)
        return gx, gw, gb


def conv_mfma(x: torch.Tensor, w: torch.Tensor, b) -> torch.Tensor:
    """Conv3d(C -> C, 3, stride 1, padding 1), C = 32 or 64, forward on the f32 matrix cores
    (tb_conv3d_mfma_f32)."""
    x = x.contiguous()
    N, C, D, H, W = x.shape
    y = torch.empty_like(x)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_mfma_f32(x.data_ptr(), w.contiguous().data_ptr(), b.data_ptr() if b is not None else None,
                                       y.data_ptr(), N, C, D, H, W, _stream(x)), "tb_conv3d_mfma_f32")
    return y


def conv_mfma_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    """Conv3d(32 -> 32) with rows of 4k <= 64 floats, or Conv3d(64 -> 64) with rows <= 48, stride 1,
    padding 1: k_conv3d_mfma_s1 (forward and input gradient) + the z-marching weight gradient
    (TEXBIAS_CONVMFMA=0: _ConvFn)."""
    if not (custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3)):
        return False
    C = w.shape[0]
    return C in (32, 64) and w.shape[1] == C and tuple(stride) == (1, 1, 1) and tuple(padding) == (1, 1, 1) and \
        x.shape[-1] % 4 == 0 and x.shape[-1] <= (64 if C == 32 else 48) and x.data_ptr() % 16 == 0 and CONVMFMA


class _ConvMfmaFn(torch.autograd.Function):
    """Conv3d(C -> C, stride 1), C = 32 or 64: forward and input gradient (flipped, transposed weights)
    on the channel-split MFMA kernel, weight gradient on the z-marching MFMA kernel, bias gradient on
    the channel-sum kernel."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = conv_mfma(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = conv_mfma(gy, w.flip(2, 3, 4).transpose(0, 1).contiguous(), None)
        if ctx.needs_input_grad[1]:
            gw = wgrad(gy, x, w.shape, 1, 1)
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = channel_sum(gy)
        return gx, gw, gb


class Conv3d(nn.Conv3d):
    def forward(self, x):
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                conv16_applies(x, self.weight, self.stride, self.padding):
            return _Conv16Fn.apply(x, self.weight, self.bias)
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                conv_mfma_applies(x, self.weight, self.stride, self.padding):
            return _ConvMfmaFn.apply(x, self.weight, self.bias)
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                s2_fewin_applies(x, self.weight, self.stride, self.padding):
            return _ConvS2FewInFn.apply(x, self.weight, self.bias)
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                small_conv_applies(x, self.weight, self.stride, self.padding):
            return _SmallConvFn.apply(x, self.weight, self.bias)
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                custom_backward_applies(x, self.weight):
            k = self.weight.shape[2:]
            out_sp = [(n + 2 * p - kk) // s + 1 for n, p, s, kk in zip(x.shape[2:], self.padding, self.stride, k)]
            fast = fast_wgrad_applies(x, self.weight, out_sp, self.stride, self.padding, False)
            return _ConvFn.apply(x, self.weight, self.bias, self.stride, self.padding, (0, 0, 0), False, fast)
        return super().forward(x)


class ConvTranspose3d(nn.ConvTranspose3d):
    def forward(self, x, output_size=None):
        if output_size is None and self.groups == 1 and self.dilation == (1, 1, 1) and \
                convT_fewout_applies(x, self.weight, self.stride, self.padding, self.output_padding):
            return _ConvTFewOutFn.apply(x, self.weight, self.bias)
        if output_size is None and self.groups == 1 and self.dilation == (1, 1, 1) and \
                custom_backward_applies(x, self.weight):
            fast = fast_wgrad_applies(x, self.weight, None, self.stride, self.padding, True, self.output_padding)
            return _ConvFn.apply(x, self.weight, self.bias, self.stride, self.padding, self.output_padding, True,
                                 fast)
        return super().forward(x, output_size)
