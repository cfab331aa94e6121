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
CONVT64 = True   # module switches (tests and measurement scripts set them; no environment variables)
CONVMFMA = True
CONV16 = True


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


@functools.lru_cache(maxsize=256)
def _wgrad_ws_bytes(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad) -> int:
    return int(lib().tb_conv3d_wgrad_ws_bytes(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad))


def wgrad(G: torch.Tensor, X: torch.Tensor, w_shape, stride: int, pad: int) -> torch.Tensor:
    """dW[m][c][k^3] = corr(G, X) -- see tb_conv3d_wgrad_f32 / tb_conv3d_wgrad_ws_f32 (include/texbias.h): with a
    workspace from the caching allocator the z-marching kernels write per-workgroup partial tiles that one
    reduction sums in order, instead of contended float atomics."""
    G = G.contiguous()
    X = X.contiguous()
    N, M = G.shape[:2]
    Cc = X.shape[1]
    dW = torch.empty((M, Cc, 3, 3, 3), dtype=torch.float32, device=G.device)
    Do, Ho, Wo = G.shape[2:]
    Di, Hi, Wi = X.shape[2:]
    nb = _wgrad_ws_bytes(N, M, Cc, Do, Ho, Wo, Di, Hi, Wi, stride, pad)
    ws = torch.empty(max(nb, 4), dtype=torch.uint8, device=G.device) if nb > 0 else None
    with torch.cuda.device(G.device):
        check(lib().tb_conv3d_wgrad_ws_f32(G.data_ptr(), X.data_ptr(), dW.data_ptr(), N, M, Cc, Do, Ho, Wo, Di, Hi, Wi,
                                           stride, pad, ws.data_ptr() if ws is not None else None, nb,
                                           _stream(G)), "tb_conv3d_wgrad_ws_f32")
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
    """g [N, C, *spatial] -> [C]: sum over N and the spatial axes (tb_channel_sum_ws_f32: float64 block
    partials summed in block order -- deterministic, no float atomics)."""
    g = g.contiguous()
    N, Cc = g.shape[:2]
    S = g[0, 0].numel()
    out = torch.empty(Cc, dtype=torch.float32, device=g.device)
    nb = int(lib().tb_channel_sum_ws_bytes(N, Cc, S))
    ws = torch.empty(nb, dtype=torch.uint8, device=g.device)
    with torch.cuda.device(g.device):
        check(lib().tb_channel_sum_ws_f32(g.data_ptr(), out.data_ptr(), N, Cc, S, ws.data_ptr(), nb, _stream(g)),
              "tb_channel_sum_ws_f32")
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


def weight_grad(gy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, transposed: bool = False,
                output_padding=(0, 0, 0)) -> torch.Tensor:
    """The 3x3x3, padding-1 weight gradient of a layer whose forward ran on a texbias kernel: the
    texbias MFMA kernels when tb_conv3d_wgrad_config finds a tiling for the shapes, else ATen's
    (``aten.convolution_backward`` with only the weight output), never an error for a shape the
    forward accepted."""
    G, X = (x, gy) if transposed else (gy, x)
    if _wgrad_tiles(tuple(G.shape), tuple(X.shape), stride):
        return wgrad(G, X, w.shape, stride, 1)
    _, gw, _ = torch.ops.aten.convolution_backward(gy.contiguous(), x, w, None, [stride] * 3, [1, 1, 1], [1, 1, 1],
                                                   transposed, list(output_padding), 1, [False, True, False])
    return gw


# reduction length (positions) from which the z-marching weight gradients (partial tiles, no atomics) take a
# layer whatever its channel counts -- measured: 1 gives C3 156.7 vols/s but the 128 x 128 x 64 crop 516 (its
# deep layers are better on CK), 0 (off) 155.4 / 551, 20000 156.5 / 551
ZMARCH_MIN_POS = 20000


def pos_of(x: torch.Tensor, out_spatial, transposed: bool) -> int:
    return x.shape[0] * math.prod(out_spatial if not transposed else x.shape[2:])


def fast_wgrad_applies(x: torch.Tensor, w: torch.Tensor, out_spatial, stride, padding, transposed: bool,
                       output_padding=(0, 0, 0)) -> bool:
    if not custom_backward_applies(x, w):
        return False
    if tuple(w.shape[2:]) != (3, 3, 3) or len(set(stride)) != 1 or stride[0] not in (1, 2) or padding[0] != 1 or \
            len(set(padding)) != 1:
        return False
    s = stride[0]
    if transposed:  # G = x [N, Cin, ...], X = grad of the output [N, Cout, (n - 1) s + 1 + output_padding]
        g_shape = tuple(x.shape)
        x_shape = (x.shape[0], w.shape[1]) + tuple((n - 1) * s + 1 + op for n, op in zip(x.shape[2:], output_padding))
    else:
        g_shape, x_shape = (x.shape[0], w.shape[0]) + tuple(out_spatial), tuple(x.shape)
    # the z-marching kernels (partial tiles, no atomics) take any reduction length; the general split-K
    # kernel only long ones
    if ZMARCH_MIN_POS and pos_of(x, out_spatial, transposed) >= ZMARCH_MIN_POS and \
            _wgrad_ws_bytes(*g_shape[:2], x_shape[1], *g_shape[2:], *x_shape[2:], s, 1) > 0:
        return True
    pos = x.shape[0] * math.prod(out_spatial if not transposed else x.shape[2:])
    if pos < MIN_K_PER_OUTPUT * w.shape[0] * w.shape[1] * 27 // 16:
        return False
    return _wgrad_tiles(g_shape, x_shape, s)


GEMM = os.environ.get("TEXBIAS_CONVGEMM", "1") != "0"
# the sub-pixel (ConvTranspose3d forward / stride-2 input gradient) and 1x1x1 forms of the GEMM kernel
# measured slower than MIOpen at the C3 shapes (scripts/diag/gemm_conv_bench.py): off unless asked for
GEMM_T = False
GEMM_1 = False
# ConvTranspose3d input gradient (a stride-2 Conv3d of dY) on the GEMM kernel while its forward stays on MIOpen
# (off: up2 128 -> 32 at C3 measured 2 x 100 us + reduce in the step vs MIOpen/CK's 152 us)
GEMM_TDX = False
# the identity-residual unit's input gradient dconv(dY) + dY summed in the 16-channel kernel's store (its add
# values fetched at the start of each step), instead of a separate add pass
FWD16_DX_ADD = True
# the same for the 32 / 64-channel kernel: off (its add form holds 256 VGPRs, one wave per SIMD at 32 -> 32
# instead of two, for a 6-19 us add pass)
MFMA_DX_ADD = False


def _gemm_geom_ok(x: torch.Tensor, w: torch.Tensor, stride, padding, transposed: bool, output_padding) -> bool:
    """Shapes tb_conv3d_gemm_f32 takes: 3x3x3 (padding 1, stride 1 / 2) or 1x1x1 (padding 0, stride 1)
    Conv3d, or ConvTranspose3d(3, stride 2, padding 1, output_padding 1); float32 HIP tensors, input
    channels a multiple of 8, every tensor < 2^31 elements."""
    if not (GEMM and custom_backward_applies(x, w) and x.dim() == 5 and len(set(stride)) == 1 and
            len(set(padding)) == 1):
        return False
    k = tuple(w.shape[2:])
    s, p = stride[0], padding[0]
    if transposed:
        ok = k == (3, 3, 3) and s == 2 and p == 1 and tuple(output_padding) == (1, 1, 1) and x.shape[1] == w.shape[0]
    else:
        ok = x.shape[1] == w.shape[1] and ((k == (3, 3, 3) and p == 1 and s in (1, 2)) or
                                           (k == (1, 1, 1) and p == 0 and s == 1 and GEMM_1))
    return ok and x.shape[1] % 8 == 0 and x.numel() // x.shape[1] * 8 * max(w.shape[0], w.shape[1], x.shape[1]) < 2 ** 31


def gemm_applies(x, w, stride, padding, transposed: bool, output_padding=(0, 0, 0)) -> bool:
    """Forward on the implicit-GEMM kernel (csrc/conv_gemm.hip)."""
    return (GEMM_T or not transposed) and _gemm_geom_ok(x, w, stride, padding, transposed, output_padding)


def gemm_dgrad_applies(gy, x, w, stride, padding, transposed: bool, output_padding=(0, 0, 0)) -> bool:
    """The input gradient on the implicit-GEMM kernel: stride-1 Conv3d ("dgrad"), stride-2 Conv3d on even
    extents ("convT" with the layer's weight), ConvTranspose3d (a stride-2 Conv3d of dY with its weight)."""
    if not (_gemm_geom_ok(x, w, stride, padding, transposed, output_padding) and gy.is_cuda and
            gy.dtype == torch.float32):
        return False
    if transposed:
        return gy.shape[1] % 8 == 0
    if stride[0] == 2:
        return gy.shape[1] % 8 == 0 and all(2 * a == b for a, b in zip(gy.shape[2:], x.shape[2:]))
    return gy.shape[1] % 8 == 0


def gemm_dgrad(gy: torch.Tensor, w: torch.Tensor, stride: int, transposed: bool) -> torch.Tensor:
    if transposed:   # ConvTranspose3d(Cin -> M, s2): dX = Conv3d(dY, W as [Cin][M], stride 2)
        return conv_gemm(gy, w, None, "conv", 2, 3)
    if stride == 2:  # Conv3d(s2): dX = ConvTranspose3d(dY, W as [M][Cin])
        return conv_gemm(gy, w, None, "convT", 2, 3)
    return conv_gemm(gy, w, None, "dgrad", 1, w.shape[2])


def _add_ptr(add, shape):
    if add is None:
        return None
    assert tuple(add.shape) == tuple(shape) and add.is_contiguous(), "add: the output's shape, contiguous"
    return add.data_ptr()


def small_conv(x: torch.Tensor, w: torch.Tensor, b, add=None) -> torch.Tensor:
    """Direct 3x3x3, stride 1, padding 1 convolution for <= 4 channels (tb_conv3d_small_add_f32); ``add``
    (the output's shape) is summed into the store."""
    x = x.contiguous()
    w = w.contiguous()
    N, Cin, D, H, W = x.shape
    Cout = w.shape[0]
    y = torch.empty((N, Cout, D, H, W), dtype=torch.float32, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_small_add_f32(x.data_ptr(), w.data_ptr(), b.data_ptr() if b is not None else None,
                                            _add_ptr(add, y.shape), y.data_ptr(), N, Cin, Cout, D, H, W, _stream(x)),
              "tb_conv3d_small_add_f32")
    return y


def small_conv_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3) and \
        x.shape[1] == w.shape[1] and tuple(stride) == (1, 1, 1) and tuple(padding) == (1, 1, 1) and \
        w.shape[0] <= 4 and w.shape[1] <= 4 and \
        x.shape[-1] <= 168


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
        x.shape[1] == w.shape[1] and tuple(stride) == (2, 2, 2) and tuple(padding) == (1, 1, 1) and w.shape[1] <= 4 and \
        w.shape[0] in (16, 32) and _s2_shape_ok(x.shape[2:]) and x.data_ptr() % 16 == 0


def convT_fewout_applies(x: torch.Tensor, w: torch.Tensor, stride, padding, output_padding) -> bool:
    """ConvTranspose3d(Cin <= 32 -> Cout <= 4, 3, 2, 1, output_padding 1): forward on k_convT_fewout and
    input gradient on k_conv_s2_fewin (needs Cin 16 or 32)."""
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3) and \
        x.shape[1] == w.shape[0] and tuple(stride) == (2, 2, 2) and tuple(padding) == (1, 1, 1) and \
        tuple(output_padding) == (1, 1, 1) and w.shape[1] <= 4 and w.shape[0] in (16, 32) and x.shape[-1] % 4 == 0 and x.shape[-1] <= 80 and \
        _s2_shape_ok(tuple(2 * n for n in x.shape[2:]))


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
    return CONVT64 and gy.is_cuda and gy.dtype == torch.float32 and w.dtype == torch.float32 and \
        tuple(w.shape) == (32, 16, 3, 3, 3) and tuple(stride) == (2, 2, 2) and gy.shape[1] == 32 and \
        tuple(padding) == (1, 1, 1) and gy.dim() == 5 and all(2 * a == b for a, b in zip(gy.shape[2:], x.shape[2:])) and \
        gy.shape[-1] % 4 == 0 and gy.shape[-1] <= 64 and gy.data_ptr() % 16 == 0


def convT64_applies(x: torch.Tensor, w: torch.Tensor, stride, padding, output_padding) -> bool:
    """ConvTranspose3d(64 -> 16, 3, 2, 1, output_padding 1), rows of 4k <= 64 floats: forward on
    k_convT_mfma64 (CONVT64 = False: ATen).  Input and weight gradients stay where _ConvFn puts them."""
    return CONVT64 and custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape) == (64, 16, 3, 3, 3) and \
        x.shape[1] == 64 and \
        tuple(stride) == (2, 2, 2) and tuple(padding) == (1, 1, 1) and tuple(output_padding) == (1, 1, 1) and \
        x.shape[-1] % 4 == 0 and x.shape[-1] <= 64 and x.data_ptr() % 16 == 0


def conv_fwd16(x: torch.Tensor, w: torch.Tensor, b, add=None) -> torch.Tensor:
    """Conv3d(16 -> 16, 3, stride 1, padding 1) forward on the f32 matrix cores (tb_conv3d_fwd16_add_f32)."""
    x = x.contiguous()
    N, _, D, H, W = x.shape
    y = torch.empty_like(x)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_fwd16_add_f32(x.data_ptr(), w.contiguous().data_ptr(),
                                            b.data_ptr() if b is not None else None, _add_ptr(add, y.shape),
                                            y.data_ptr(), N, D, H, W, _stream(x)), "tb_conv3d_fwd16_add_f32")
    return y


def conv_fwd16_dgrad(gy: torch.Tensor, w: torch.Tensor, add=None) -> torch.Tensor:
    """The input gradient of Conv3d(16 -> 16, 3, 1, 1) with weight ``w``: the forward kernel reading
    W[c][m][26 - t] in place of a flipped, transposed copy (tb_conv3d_fwd16_dgrad_f32); ``add`` (the
    output's shape; a channel slice of a wider tensor is read in place) summed into the store."""
    gy = gy.contiguous()
    N, _, D, H, W = gy.shape
    dx = torch.empty_like(gy)
    sn = 0
    if add is not None:
        S = D * H * W
        if not (tuple(add.shape) == tuple(gy.shape) and add.stride(1) == S and add[0, 0].is_contiguous() and
                add.data_ptr() % 4 == 0):
            add = add.contiguous()
        sn = add.stride(0)
    with torch.cuda.device(gy.device):
        check(lib().tb_conv3d_fwd16_dgrad_f32(gy.data_ptr(), w.contiguous().data_ptr(),
                                              add.data_ptr() if add is not None else None, sn, dx.data_ptr(),
                                              N, D, H, W, _stream(gy)), "tb_conv3d_fwd16_dgrad_f32")
    return dx


def conv16_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    """Conv3d(16 -> 16, 3, stride 1, padding 1), rows of 16k <= 128 floats: k_conv3d_fwd16 (forward and
    input gradient) + the z-marching weight gradient."""
    return custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape) == (16, 16, 3, 3, 3) and \
        x.shape[1] == 16 and tuple(stride) == (1, 1, 1) and tuple(padding) == (1, 1, 1) and x.shape[-1] % 16 == 0 and \
        x.shape[-1] <= 80 and x.data_ptr() % 16 == 0 and CONV16


def conv_mfma(x: torch.Tensor, w: torch.Tensor, b, add=None) -> torch.Tensor:
    """Conv3d(C -> C, 3, stride 1, padding 1), C = 32 or 64, forward on the f32 matrix cores
    (tb_conv3d_mfma_add_f32)."""
    x = x.contiguous()
    N, C, D, H, W = x.shape
    y = torch.empty_like(x)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_mfma_add_f32(x.data_ptr(), w.contiguous().data_ptr(),
                                           b.data_ptr() if b is not None else None, _add_ptr(add, y.shape),
                                           y.data_ptr(), N, C, D, H, W, _stream(x)), "tb_conv3d_mfma_add_f32")
    return y


def conv_mfma_dgrad(gy: torch.Tensor, w: torch.Tensor, add=None) -> torch.Tensor:
    """The input gradient of Conv3d(C -> C, 3, 1, 1), C = 32 / 64, reading the flipped weight in the
    kernel (tb_conv3d_mfma_dgrad_f32); ``add`` summed into the store (a channel slice read in place)."""
    gy = gy.contiguous()
    N, C, D, H, W = gy.shape
    dx = torch.empty_like(gy)
    sn = 0
    if add is not None:
        S = D * H * W
        if not (tuple(add.shape) == tuple(gy.shape) and add.stride(1) == S and add[0, 0].is_contiguous()):
            add = add.contiguous()
        sn = add.stride(0)
    with torch.cuda.device(gy.device):
        check(lib().tb_conv3d_mfma_dgrad_f32(gy.data_ptr(), w.contiguous().data_ptr(),
                                             add.data_ptr() if add is not None else None, sn, dx.data_ptr(),
                                             N, C, D, H, W, _stream(gy)), "tb_conv3d_mfma_dgrad_f32")
    return dx


def conv_mfma_applies(x: torch.Tensor, w: torch.Tensor, stride, padding) -> bool:
    """Conv3d(32 -> 32) with rows of 4k <= 64 floats, or Conv3d(64 -> 64) with rows <= 48, stride 1,
    padding 1: k_conv3d_mfma_s1 (forward and input gradient) + the z-marching weight gradient
    (CONVMFMA = False: _ConvFn)."""
    if not (custom_backward_applies(x, w) and x.dim() == 5 and tuple(w.shape[2:]) == (3, 3, 3) and
            x.shape[1] == w.shape[1]):
        return False
    C = w.shape[0]
    return C in (32, 64) and w.shape[1] == C and tuple(stride) == (1, 1, 1) and tuple(padding) == (1, 1, 1) and \
        x.shape[-1] % 4 == 0 and x.shape[-1] <= (64 if C == 32 else 48) and x.data_ptr() % 16 == 0 and CONVMFMA


# ---------------------------------------------------------------- implicit-GEMM convolutions
CG_MODES = {"conv": 0, "dgrad": 1, "convT": 2}


def gemm_out_shape(x_shape, w_shape, mode: str, stride: int, ksize: int):
    N, _, D, H, Wd = x_shape
    if mode == "conv":
        p = 1 if ksize == 3 else 0
        return (N, w_shape[0]) + tuple((n + 2 * p - ksize) // stride + 1 for n in (D, H, Wd))
    if mode == "dgrad":
        return (N, w_shape[1], D, H, Wd)
    return (N, w_shape[1], 2 * D, 2 * H, 2 * Wd)


def conv_gemm(x: torch.Tensor, w: torch.Tensor, b=None, mode: str = "conv", stride: int = 1, ksize: int = 3,
              add=None, out=None) -> torch.Tensor:
    """tb_conv3d_gemm_f32 (csrc/conv_gemm.hip): mode "conv" = Conv3d(x, w, b, stride, padding (k-1)/2);
    "dgrad" = the input gradient of a stride-1 Conv3d whose weight is ``w`` (x = dY); "convT" =
    ConvTranspose3d(x, w, b, stride 2, padding 1, output_padding 1), which with a stride-2 Conv3d's
    weight is that layer's input gradient.  ``add`` (same shape as the output) is summed in; ``out`` may be
    given (batch stride free: a channel slice of a larger buffer) and may alias ``add``."""
    N, Cin, D, H, Wd = x.shape
    if x.stride(1) != D * H * Wd or x.stride(4) != 1 or x.stride(3) != Wd or x.stride(2) != H * Wd:
        x = x.contiguous()
    w = w.contiguous()
    md = CG_MODES[mode]
    M = w.shape[0] if mode == "conv" else w.shape[1]
    oshape = gemm_out_shape(x.shape, w.shape, mode, stride, ksize)
    y = torch.empty(oshape, dtype=torch.float32, device=x.device) if out is None else out
    sp = math.prod(oshape[2:])
    assert y.shape == oshape and y.stride(1) == sp and y.stride(4) == 1, "conv_gemm: out layout"
    if add is not None:
        assert add.shape == oshape and add.stride(1) == sp and add.stride(4) == 1, "conv_gemm: add layout"
    nb = int(lib().tb_conv3d_gemm_workspace_bytes(md, N, Cin, M, D, H, Wd, stride, ksize))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_conv3d_gemm_f32(md, x.data_ptr(), x.stride(0), w.data_ptr(),
                                       b.data_ptr() if b is not None else None,
                                       add.data_ptr() if add is not None else None,
                                       add.stride(0) if add is not None else 0, y.data_ptr(), y.stride(0), N, Cin, M,
                                       D, H, Wd, stride, ksize, ws.data_ptr(), nb, _stream(x)), "tb_conv3d_gemm_f32")
    return y


def conv_gemm_config(x_shape, M: int, mode: str = "conv", stride: int = 1, ksize: int = 3) -> dict:
    import ctypes
    cfg = (ctypes.c_int64 * 6)()
    N, Cin, D, H, Wd = x_shape
    check(lib().tb_conv3d_gemm_config(CG_MODES[mode], N, Cin, M, D, H, Wd, stride, ksize, cfg), "tb_conv3d_gemm_config")
    return dict(zip(("BM", "BP", "nsplit", "kper", "blocks", "positions"), list(cfg)))


# ---------------------------------------------------------------- routing: one kernel choice per call
class Route:
    """The kernels one Conv3d / ConvTranspose3d call runs on -- forward, input gradient, weight gradient,
    bias gradient -- chosen once from the shapes (the gates above), so that the layer's autograd function
    and the fused U-Net blocks (``texbias.unet``) share one dispatch.  Kinds: ``fwd16`` (k_conv3d_fwd16),
    ``mfma`` (k_conv3d_mfma_s1), ``fewin`` (k_conv_s2_fewin), ``small`` (k_conv3d_small_z), ``fewout``
    (k_convT_fewout), ``convT64`` (k_convT_mfma64), ``gemm`` (k_conv_gemm), ``aten`` (MIOpen / CK)."""

    __slots__ = ("kind", "dx", "stride", "padding", "output_padding", "transposed", "fast_w", "k")

    def __init__(self, x: torch.Tensor, w: torch.Tensor, stride, padding, output_padding, transposed: bool):
        self.stride, self.padding = tuple(stride), tuple(padding)
        self.output_padding, self.transposed = tuple(output_padding), transposed
        self.k = w.shape[2]
        st, pd, op = self.stride, self.padding, self.output_padding
        if not custom_backward_applies(x, w):
            self.kind = "aten"
        elif transposed:
            self.kind = ("fewout" if convT_fewout_applies(x, w, st, pd, op) else
                         "convT64" if convT64_applies(x, w, st, pd, op) else
                         "gemm" if gemm_applies(x, w, st, pd, True, op) else "aten")
        else:
            self.kind = ("fwd16" if conv16_applies(x, w, st, pd) else
                         "mfma" if conv_mfma_applies(x, w, st, pd) else
                         "fewin" if s2_fewin_applies(x, w, st, pd) else
                         "small" if small_conv_applies(x, w, st, pd) else
                         "gemm" if gemm_applies(x, w, st, pd, False) else "aten")
        # input gradient kernel
        if self.kind in ("fwd16", "mfma", "small", "fewout"):
            self.dx = self.kind
        else:
            self.dx = "aten"
            if self.kind != "aten" and not transposed and st[0] == 2 and tuple(w.shape) in ((32, 16, 3, 3, 3),
                                                                                         (64, 16, 3, 3, 3)) \
                    and CONVT64 and x.shape[-1] % 8 == 0 and x.shape[-1] // 2 <= 64 and \
                    all(n % 2 == 0 for n in x.shape[2:]):
                self.dx = "convT64"   # Conv3d(16 -> 32 / 64 stacked, s2)'s input gradient on k_convT_mfma64
            elif (self.kind != "aten" or (transposed and GEMM_TDX)) and _gemm_geom_ok(x, w, st, pd, transposed, op) and \
                    (w.shape[1] % 8 == 0 if transposed else w.shape[0] % 8 == 0) and \
                    (transposed or st[0] == 1 or (GEMM_T and all(n % 2 == 0 for n in x.shape[2:]))):
                # ConvTranspose3d: a stride-2 Conv3d of dY (the GEMM's conv form); stride-1 Conv3d: the
                # flipped-weight form; stride-2 Conv3d: the sub-pixel form (GEMM_T)
                self.dx = "gemm"
        # weight gradient: the texbias MFMA kernels where a tiling exists and the reduction is long
        if self.kind in ("fwd16", "mfma", "fewin", "small", "fewout"):
            self.fast_w = True
        elif self.kind == "aten" and not custom_backward_applies(x, w):
            self.fast_w = False
        else:
            osp = None if transposed else [(n + 2 * p - kk) // s + 1
                                          for n, p, s, kk in zip(x.shape[2:], pd, st, w.shape[2:])]
            self.fast_w = fast_wgrad_applies(x, w, osp, st, pd, transposed, op)

    # -- forward (``add``: summed into the output -- in the kernel's store where the kernel takes it)
    def forward(self, x, w, b, add=None):
        k = self.kind
        # (the 16- and 32/64-channel MFMA kernels' add epilogue measured slower than a separate add: 490 vs
        # 354 + 64 us for 16 -> 16 at 120 x 120 x 80 -- its scattered reads stall the store phase)
        if add is not None and k in ("small", "gemm"):
            add = add.contiguous()
            if k == "small":
                return small_conv(x, w, b, add)
            return conv_gemm(x, w, b, "convT" if self.transposed else "conv", self.stride[0], self.k, add=add)
        if add is not None:
            return self.forward(x, w, b).add_(add)
        if k == "fwd16":
            return conv_fwd16(x, w, b)
        if k == "mfma":
            return conv_mfma(x, w, b)
        if k == "fewin":
            return conv_s2_fewin(x, s2_pairs(w), b, w.shape[0])
        if k == "small":
            return small_conv(x, w, b)
        if k == "fewout":
            return convT_fewout(x, w, b)
        if k == "convT64":
            return convT_mfma(x, w, b)
        if k == "gemm":
            return conv_gemm(x, w, b, "convT" if self.transposed else "conv", self.stride[0], self.k)
        if self.transposed:
            return F.conv_transpose3d(x, w, b, self.stride, self.padding, self.output_padding)
        return F.conv3d(x, w, b, self.stride, self.padding)

    # -- input gradient (x only for its shape on the ATen path; ``add`` summed in, as in forward)
    def input_grad(self, gy, x, w, add=None):
        k = self.dx
        if add is not None:  # (a strided add -- a channel slice of the skip concatenation's gradient -- is
            if k == "fwd16" and FWD16_DX_ADD:  # copied only for the kernels that need it contiguous)
                return conv_fwd16_dgrad(gy, w, add)
            if k == "mfma" and MFMA_DX_ADD:
                return conv_mfma_dgrad(gy, w, add)
            if k == "small":
                return small_conv(gy, w.flip(2, 3, 4).transpose(0, 1).contiguous(), None, add.contiguous())
            if k == "gemm" and not self.transposed and self.stride[0] == 1:
                return conv_gemm(gy, w, None, "dgrad", 1, w.shape[2], add=add.contiguous())
            return self.input_grad(gy, x, w).add_(add)
        if k == "fwd16":
            return conv_fwd16_dgrad(gy, w)
        if k == "mfma":
            return conv_mfma_dgrad(gy, w)
        if k == "small":
            return small_conv(gy, w.flip(2, 3, 4).transpose(0, 1).contiguous(), None)
        if k == "fewout":   # dX[m][i] = sum_{c, t} W[m][c][t] dY[c][2 i + t - 1]
            return conv_s2_fewin(gy, s2_pairs(w), None, w.shape[0])
        if k == "convT64":
            return convT_mfma(gy if gy.data_ptr() % 16 == 0 else gy.clone(), w, None)
        if k == "gemm":
            return gemm_dgrad(gy, w, self.stride[0], self.transposed)
        gx, _, _ = torch.ops.aten.convolution_backward(
            gy, x, w, None, list(self.stride), list(self.padding), [1, 1, 1], self.transposed,
            list(self.output_padding), 1, [True, False, False])
        return gx

    # -- weight gradient
    def weight_grad(self, gy, x, w):
        if self.fast_w and tuple(w.shape[2:]) == (3, 3, 3) and self.padding[0] == 1:
            return weight_grad(gy, x, w, self.stride[0], self.transposed, self.output_padding)
        _, gw, _ = torch.ops.aten.convolution_backward(
            gy, x, w, None, list(self.stride), list(self.padding), [1, 1, 1], self.transposed,
            list(self.output_padding), 1, [False, True, False])
        return gw

    def backward(self, gy, x, w, need_x: bool, need_w: bool, need_b: bool, gb=None):
        gy = gy.contiguous()
        gx = self.input_grad(gy, x, w) if need_x else None
        gw = self.weight_grad(gy, x, w) if need_w else None
        if need_b and gb is None:
            gb = channel_sum(gy) if self.kind != "aten" else gy.sum(dim=(0, 2, 3, 4))
        return gx, gw, gb if need_b else None


class _RouteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, route):
        y = route.forward(x.contiguous() if route.kind != "aten" else x, w, b)
        ctx.save_for_backward(x, w)
        ctx.route, ctx.has_b = route, b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        n = ctx.needs_input_grad
        gx, gw, gb = ctx.route.backward(gy, x, w, n[0], n[1], n[2] and ctx.has_b)
        return gx, gw, gb, None


def route_of(mod, x: torch.Tensor) -> "Route":
    """The layer's route for this input (cached per shape / alignment / dtype / device)."""
    key = (tuple(x.shape), x.dtype, x.device, x.data_ptr() % 16 == 0, x.is_contiguous())
    cache = mod.__dict__.setdefault("_tb_routes", {})
    r = cache.get(key)
    if r is None:
        tr = isinstance(mod, nn.ConvTranspose3d)
        r = Route(x, mod.weight, mod.stride, mod.padding, mod.output_padding if tr else (0, 0, 0), tr)
        cache[key] = r
    return r


class Conv3d(nn.Conv3d):
    def forward(self, x):
        if self.groups == 1 and self.dilation == (1, 1, 1) and self.padding_mode == "zeros" and \
                custom_backward_applies(x, self.weight):
            return _RouteFn.apply(x, self.weight, self.bias, route_of(self, x))
        return super().forward(x)


class ConvTranspose3d(nn.ConvTranspose3d):
    def forward(self, x, output_size=None):
        if output_size is None and self.groups == 1 and self.dilation == (1, 1, 1) and \
                custom_backward_applies(x, self.weight):
            return _RouteFn.apply(x, self.weight, self.bias, route_of(self, x))
        return super().forward(x, output_size)
