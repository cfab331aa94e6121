"""PyTorch custom operators over the texbias C ABI (``torch.ops.texbias.*``).

The filters of ``filters_and_operators.py`` / ``stylization_layers.py`` run through these ops, so
they are visible to ``torch.compile`` (fake-tensor / meta propagation via ``register_fake``, no
graph break), to ``torch.cuda.graphs`` capture (stream-ordered launches on the current stream, no
host synchronisation) and to autograd where a backward exists.  The transform classes stay the
front end with the reference's signatures; the op boundary carries the sample
programs as a uint8 CPU tensor of ``tb_sample_ops`` records (``include/texbias.h``).

Reference interfaces each op replaces (file:line under the reference root):
  texbias::kspace_filter     Fourier.shift_fourier -> k-space op(s) -> inv_shift_fourier(...).real
                             source_code/filters_and_operators.py:236-252, 370-393, 503-515,
                             663-705, 906-983; stylization_layers.py:79-116
  texbias::salt_and_pepper_  SaltAndPepper.salt_and_pepper  filters_and_operators.py:465-482
  texbias::gibbs_layer       GibbsNoiseLayer.forward / _apply_mask  stylization_layers.py:79-116
                             (autograd: the filter is self-adjoint; d/d alpha = 0 as in the reference)
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import kprog as K
from ._abi import TbSampleOps, programs_array
from . import runtime as rt

_REC = C.sizeof(TbSampleOps)


def pack_programs(programs: Sequence[Sequence]) -> torch.Tensor:
    """list (per sample) of op lists -> uint8 CPU tensor [B, sizeof(tb_sample_ops)]; with a program
    longer than TB_MAX_OPS, [passes, B, sizeof(tb_sample_ops)] (cut by ``kprog.split_program``:
    needs the op's frequency geometry, so such programs go through ``pack_programs_split``)."""
    arr = programs_array(programs)
    buf = np.frombuffer(C.string_at(C.addressof(arr), C.sizeof(arr)), dtype=np.uint8).copy()
    return torch.from_numpy(buf).reshape(len(programs), _REC)


def pack_programs_split(programs: Sequence[Sequence], hwd: Sequence[int]) -> torch.Tensor:
    """``pack_programs`` for programs of any length: [passes, B, REC] when one exceeds TB_MAX_OPS."""
    from ._abi import TB_MAX_OPS
    if all(len(p) <= TB_MAX_OPS for p in programs):
        return pack_programs(programs)
    parts = [K.split_program(list(p), hwd) for p in programs]
    npass = max(len(c) for c in parts)
    return torch.stack([pack_programs([c[i] if i < len(c) else [] for c in parts]) for i in range(npass)])


def unpack_programs(t: torch.Tensor) -> List[TbSampleOps]:
    raw = bytes(t.contiguous().cpu().numpy().tobytes())
    n = t.shape[0]
    arr = (TbSampleOps * n).from_buffer_copy(raw)
    return list(arr)


def _as_prog_lists(recs: List[TbSampleOps]):
    return [[r.op[j] for j in range(r.n)] for r in recs]


@torch.library.custom_op("texbias::kspace_filter", mutates_args=())
def kspace_filter(x: torch.Tensor, n_dims: int, programs: torch.Tensor, channels: int,
                  pad: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """y = Re(IFFT(program_b(FFT(x)))) over the trailing ``n_dims`` axes of [B*channels..., *spatial]
    (last axis padded by ``pad`` zero columns); also the per-sample (min, max) order-preserving keys
    (int32 [B, 2]) that salt-and-pepper uses."""
    passes = [programs] if programs.dim() == 2 else list(programs)   # [passes, B, REC]: split programs
    progs = _as_prog_lists(unpack_programs(passes[0]))
    mm = torch.empty((len(progs), 2), dtype=torch.int32, device=x.device)
    y = rt._kspace_filter_pass(x, n_dims, progs, channels, pad=pad, minmax=mm)
    view = y[..., : x.shape[-1]] if pad else y
    for p in passes[1:]:
        rt._kspace_filter_pass(view, n_dims, _as_prog_lists(unpack_programs(p)), channels, out=view, minmax=mm)
    return y, mm


@kspace_filter.register_fake
def _kspace_filter_fake(x, n_dims, programs, channels, pad=0):
    shape = tuple(x.shape[:-1]) + (x.shape[-1] + pad,)
    return x.new_empty(shape), x.new_empty((programs.shape[-2], 2), dtype=torch.int32)


@torch.library.custom_op("texbias::salt_and_pepper_", mutates_args=("x",))
def salt_and_pepper_(x: torch.Tensor, minmax: torch.Tensor, thresholds: torch.Tensor, seed: int, offset: int,
                     per_sample_dims: int) -> None:
    """In place: voxels with u <= lo -> min/2, lo < u <= hi -> max/2 of their sample (keys from
    ``minmax``); u from the device Philox stream (seed, offset).  thresholds: float32 CPU [B, 2]."""
    thr = [(float(a), float(b)) for a, b in thresholds.tolist()]
    rt.salt_and_pepper(x, per_sample_dims, thr, minmax, out=x, seed=seed, offset=offset)


@salt_and_pepper_.register_fake
def _salt_and_pepper_fake(x, minmax, thresholds, seed, offset, per_sample_dims):
    return None


def kspace_filter_programs(x: torch.Tensor, n_dims: int, programs: Sequence[Sequence], channels: int,
                           pad: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Convenience: the op with Python op lists."""
    return torch.ops.texbias.kspace_filter(x, n_dims, pack_programs(programs), channels, pad)


def _layer_apply(img: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    B = img.shape[0]
    n_dims = img.dim() - 1
    spatial = tuple(img.shape[1:])
    a = alpha.detach().reshape(-1)[:1].to(device=img.device, dtype=torch.float32).contiguous()
    # the kernel reads alpha from device memory (no host round trip for Gibbs_GD updates); `a`
    # aliases the alpha buffer or is a stream-ordered temporary, so the read is safe
    prog = [K.layer_op(0.0, spatial, alpha_ptr=a.data_ptr())]
    x = img if img.dtype == torch.float32 else img.float()
    y = rt.kspace_filter(x.reshape((B, 1) + spatial), n_dims, [prog] * B, 1)
    return y.reshape(img.shape)


@torch.library.custom_op("texbias::gibbs_layer", mutates_args=())
def gibbs_layer(img: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    """GibbsNoiseLayer's low-pass over all non-batch axes with the device-resident alpha."""
    return _layer_apply(img.contiguous(), alpha)


@gibbs_layer.register_fake
def _gibbs_layer_fake(img, alpha):
    return torch.empty_like(img, dtype=torch.float32)


def _gibbs_layer_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[1])


def _gibbs_layer_backward(ctx, gy):
    (alpha,) = ctx.saved_tensors
    return torch.ops.texbias.gibbs_layer(gy, alpha), torch.zeros_like(alpha)


gibbs_layer.register_autograd(_gibbs_layer_backward, setup_context=_gibbs_layer_setup)
