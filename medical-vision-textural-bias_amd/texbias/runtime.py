"""Device runtime: plans, workspaces and the batched launch wrappers over the C ABI.

Tensors are torch CUDA (HIP) tensors; launches go on the caller's current
stream (``torch.cuda.current_stream``) so they order with surrounding torch
work and graph-capture with it.  Raises if a tensor is not on a HIP device:
this is the product path and it has no CPU implementation.
"""
from __future__ import annotations

import ctypes as C
import threading
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._abi import TB_MAX_BATCH, TB_MAX_OPS, programs_array
from ._lib import TexbiasError, check, lib
from .kprog import Geometry, geometry, split_program

_plans: Dict[Tuple[int, int, int, int], "Plan"] = {}
_ws: "OrderedDict[Tuple[int, int], torch.Tensor]" = OrderedDict()
_ws_lock = threading.Lock()
_mm: Dict[int, torch.Tensor] = {}
_lock = threading.Lock()


class Plan:
    def __init__(self, device: torch.device, H: int, W: int, D: int):
        self.device, self.H, self.W, self.D = device, H, W, D
        h = C.c_void_p()
        with torch.cuda.device(device):
            check(lib().tb_plan_create(H, W, D, C.byref(h)), f"plan {H}x{W}x{D}")
        self.handle = h

    def radices(self, axis: int) -> List[int]:
        buf = (C.c_int * 8)()
        n = lib().tb_plan_radices(self.handle, axis, buf)
        return list(buf[:n])

    def workspace_bytes(self, bc: int) -> int:
        return int(lib().tb_workspace_bytes(self.handle, bc))

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            if self.handle:
                lib().tb_plan_destroy(self.handle)
        except Exception:
            pass


def require_hip(t: torch.Tensor, what: str) -> None:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise TexbiasError(f"{what}: expected a HIP (cuda) tensor, got {getattr(t, 'device', type(t))}")
    if t.dtype != torch.float32:
        raise TexbiasError(f"{what}: expected float32, got {t.dtype}")


def plan_for(device: torch.device, H: int, W: int, D: int) -> Plan:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, H, W, D)
    p = _plans.get(key)
    if p is None:
        with _lock:
            p = _plans.get(key)
            if p is None:
                p = Plan(torch.device("cuda", idx), H, W, D)
                _plans[key] = p
    return p


def _ws_key(device: torch.device) -> Tuple[int, int]:
    """Workspaces are per (device, current stream): the launches of one stream are ordered, so they
    share one; launches from two streams (a side stream, a second thread) get separate scratch --
    the band passes keep their arrival counter and min/max partials in it."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return idx, torch.cuda.current_stream(torch.device("cuda", idx)).cuda_stream


# Bounded LRU caches: a caller that makes a fresh stream per iteration (or per thread) would otherwise
# keep one spectrum-sized workspace per stream it ever used.  An evicted workspace was allocated on its
# own stream, so the caching allocator hands its memory out again only in that stream's order.
_WS_CAP = 8


def _cached_ws(cache: "OrderedDict[Tuple[int, int], torch.Tensor]", device: torch.device, nbytes: int) -> torch.Tensor:
    key = _ws_key(device)
    with _ws_lock:
        ws = cache.get(key)
        if ws is None or ws.numel() < nbytes:
            ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=torch.device("cuda", key[0]))
        cache[key] = ws
        cache.move_to_end(key)
        while len(cache) > _WS_CAP:
            cache.popitem(last=False)
    return ws


def workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    return _cached_ws(_ws, device, nbytes)


_ws_prep: "OrderedDict[Tuple[int, int], torch.Tensor]" = OrderedDict()


def workspace_prep(device: torch.device, nbytes: int) -> torch.Tensor:
    """Small per-(device, stream) workspace of the preprocessing statistics (kept apart from the
    spectrum workspace so neither reallocates the other)."""
    return _cached_ws(_ws_prep, device, nbytes)


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _bc_view(x: torch.Tensor, n_dims: int):
    """View [*lead, *spatial] as (BC, spatial strides) with a single bc stride, else None."""
    lead = x.shape[: x.dim() - n_dims]
    sp = x.shape[x.dim() - n_dims:]
    bc = int(np.prod(lead)) if lead else 1
    st = x.stride()
    lead_st = st[: x.dim() - n_dims]
    sp_st = st[x.dim() - n_dims:]
    # lead dims must collapse to one stride
    bstride = None
    if lead:
        exp = None
        for size, s in zip(reversed(lead), reversed(lead_st)):
            if size == 1:
                continue
            if exp is None:
                exp, bstride = s * size, s
            elif s != exp:
                return None
            else:
                exp = s * size
    if bstride is None:
        bstride = int(np.prod(sp))
    return bc, bstride, sp, sp_st


def _hwd_strides(geo: Geometry, sp_st: Sequence[int]) -> Tuple[int, int, int]:
    k = [sp_st[i] for i in geo.kept]
    if len(k) == 3:
        return k[0], k[1], k[2]
    if len(k) == 2:
        return k[0], 0, k[1]
    if len(k) == 1:
        return 0, 0, k[0]
    return 0, 0, 1


def kspace_filter(x: torch.Tensor, n_dims: int, programs: Sequence[Sequence], channels: int,
                  out: Optional[torch.Tensor] = None, pad: int = 0,
                  minmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = Re(IFFT(program_b(FFT(x)))) over the trailing ``n_dims`` axes.

    ``x``: [*lead, *spatial] float32 on a HIP device, lead = (B, C) flattened to B*C with
    ``channels`` = C; ``programs``: B lists of TbOp.  ``pad`` appends zero columns to the
    last axis of the output (U-Net padding).  ``minmax``: optional int32 [B, 2] device
    tensor receiving the per-sample (min, max) keys of the output.  Programs longer than one
    launch holds (TB_MAX_OPS) run as several passes cut where that is exact
    (``kprog.split_program``); the later passes filter the output in place.
    """
    require_hip(x, "kspace_filter")
    if all(len(p) <= TB_MAX_OPS for p in programs):
        return _kspace_filter_pass(x, n_dims, programs, channels, out, pad, minmax)
    hwd = geometry(x.shape[x.dim() - n_dims:]).hwd
    parts = [split_program(list(p), hwd) for p in programs]
    npass = max(len(c) for c in parts)
    passes = [[c[i] if i < len(c) else [] for c in parts] for i in range(npass)]
    y = _kspace_filter_pass(x, n_dims, passes[0], channels, out, pad, minmax)
    view = y[..., : x.shape[-1]] if pad else y
    for prog in passes[1:]:
        _kspace_filter_pass(view, n_dims, prog, channels, view, 0, minmax)
    return y


def planes_closed_form(x: torch.Tensor, n_dims: int, programs: Sequence[Sequence], channels: int,
                       out: Optional[torch.Tensor] = None, pad: int = 0,
                       minmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The closed-form spike route alone (``tb_planes_closed_form_f32``): ``kspace_filter`` for
    programs made only of spikes that do not touch; raises for any other program."""
    require_hip(x, "planes_closed_form")
    return _kspace_filter_pass(x, n_dims, programs, channels, out, pad, minmax, entry="tb_planes_closed_form_f32")


def _kspace_filter_pass(x: torch.Tensor, n_dims: int, programs: Sequence[Sequence], channels: int,
                        out: Optional[torch.Tensor] = None, pad: int = 0,
                        minmax: Optional[torch.Tensor] = None, entry: str = "tb_kspace_filter_f32") -> torch.Tensor:
    """One launch group of ``kspace_filter`` (every program at most TB_MAX_OPS ops)."""
    geo = geometry(x.shape[x.dim() - n_dims:])
    H, W, D = geo.hwd
    v = _bc_view(x, n_dims)
    if v is None or _hwd_strides(geo, v[3])[2] != 1:
        x = x.contiguous()
        v = _bc_view(x, n_dims)
    bc, bstride, sp, sp_st = v
    B = len(programs)
    if bc != B * channels:
        raise ValueError(f"{B} programs x {channels} channels != {bc} volumes")
    sh, sw, sd = _hwd_strides(geo, sp_st)
    if sd != 1:
        raise TexbiasError("innermost transformed axis must be contiguous")
    if out is None:
        osh = tuple(x.shape[:-1]) + (x.shape[-1] + pad,)
        out = torch.empty(osh, dtype=torch.float32, device=x.device)
    require_hip(out, "kspace_filter(out)")
    if pad and len(geo.kept) and geo.kept[-1] != n_dims - 1:
        raise TexbiasError("padding requires a non-singleton last axis")
    vo = _bc_view(out, n_dims)
    if vo is None:
        raise TexbiasError("output must collapse its leading axes")
    geo_o = Geometry(tuple(out.shape[out.dim() - n_dims:]), geo.kept)
    osh_, osw, osd = _hwd_strides(geo_o, vo[3])
    if osd != 1:
        raise TexbiasError("output innermost axis must be contiguous")
    plan = plan_for(x.device, H, W, D)
    nbytes = plan.workspace_bytes(bc)
    with torch.cuda.device(x.device):
        ws = workspace(x.device, nbytes)
        xs = (C.c_int64 * 3)(bstride, sh, sw)
        ys = (C.c_int64 * 3)(vo[1], osh_, osw)
        progs = programs_array(programs)
        mm_ptr = None
        if minmax is not None:
            if minmax.dtype != torch.int32 or minmax.numel() < 2 * B or minmax.device != x.device:
                raise TexbiasError("minmax must be an int32 [B,2] tensor on the input's device")
            mm_ptr = minmax.data_ptr()
        check(getattr(lib(), entry)(plan.handle, x.data_ptr(), xs, out.data_ptr(), ys, pad, ws.data_ptr(),
                                    ws.numel(), B, channels, C.addressof(progs), mm_ptr, _stream(x.device)), entry)
    return out


def minmax_buffer(device: torch.device, B: int) -> torch.Tensor:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    m = _mm.get(idx)
    if m is None or m.shape[0] < B:
        m = torch.empty((max(B, 8), 2), dtype=torch.int32, device=torch.device("cuda", idx))
        _mm[idx] = m
    return m[:B]


def _rows_geometry(x: torch.Tensor, per_sample_dims: int):
    """(B, rows, len, ld, sb) of x viewed as B samples of rows x len (last axis contiguous)."""
    if x.stride(-1) != 1:
        raise TexbiasError("last axis must be contiguous")
    B = int(np.prod(x.shape[: x.dim() - per_sample_dims])) if x.dim() > per_sample_dims else 1
    inner = x.shape[x.dim() - per_sample_dims:]
    ln = int(inner[-1])
    rows = int(np.prod(inner[:-1])) if len(inner) > 1 else 1
    ld = x.stride(-2) if x.dim() >= 2 else ln
    # rows must be uniformly strided by ld within a sample
    exp = ld
    for size, s in zip(reversed(inner[:-1]), reversed(x.stride()[x.dim() - per_sample_dims:-1])):
        if size != 1 and s != exp:
            return None
        exp = s * size if size != 1 else exp
    sb = x.stride(x.dim() - per_sample_dims - 1) if x.dim() > per_sample_dims else rows * ld
    if B > 1:
        lead = x.shape[: x.dim() - per_sample_dims]
        lst = x.stride()[: x.dim() - per_sample_dims]
        e = None
        for size, s in zip(reversed(lead), reversed(lst)):
            if size == 1:
                continue
            if e is None:
                e, sb = s * size, s
            elif s != e:
                return None
            else:
                e = s * size
    return B, rows, ln, ld, sb


def minmax_keys(x: torch.Tensor, per_sample_dims: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    require_hip(x, "minmax")
    g = _rows_geometry(x, per_sample_dims)
    if g is None:
        x = x.contiguous()
        g = _rows_geometry(x, per_sample_dims)
    B, rows, ln, ld, sb = g
    mm = out if out is not None else torch.empty((B, 2), dtype=torch.int32, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_minmax_f32(x.data_ptr(), mm.data_ptr(), B, rows, ln, ld, sb, _stream(x.device)), "tb_minmax_f32")
    return mm


def keys_to_float(mm: torch.Tensor) -> np.ndarray:
    L = lib()
    return np.array([[L.tb_key_to_float(int(v) & 0xFFFFFFFF) for v in row] for row in mm.cpu().tolist()],
                    np.float32)


def salt_and_pepper(x: torch.Tensor, per_sample_dims: int, thresholds: Sequence[Tuple[float, float]],
                    minmax: torch.Tensor, out: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None,
                    cls: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0) -> torch.Tensor:
    """SaltAndPepper.salt_and_pepper over B samples.  out may be x (sparse in-place scatter)."""
    require_hip(x, "salt_and_pepper")
    if out is None:
        out = torch.empty_like(x)
    require_hip(out, "salt_and_pepper(out)")
    g = _rows_geometry(x, per_sample_dims)
    go = _rows_geometry(out, per_sample_dims)
    if g is None or go is None or g != go:
        raise TexbiasError("salt_and_pepper: input/output must share a row geometry")
    B, rows, ln, ld, sb = g
    if len(thresholds) != B:
        raise ValueError("one (lo, hi) threshold pair per sample")
    thr = np.asarray(thresholds, np.float32).reshape(B, 2)
    thr_c = (C.c_float * (2 * B))(*thr.ravel().tolist())
    for t, name in ((u, "u"),):
        if t is not None:
            require_hip(t, name)
            if _rows_geometry(t, per_sample_dims) != g:
                raise TexbiasError("u must share the input's geometry")
    if cls is not None and (cls.dtype != torch.int8 or cls.shape != x.shape or cls.stride() != x.stride()):
        raise TexbiasError("cls must be int8 with the input's shape and strides")
    with torch.cuda.device(x.device):
        check(lib().tb_salt_pepper_f32(x.data_ptr(), out.data_ptr(), cls.data_ptr() if cls is not None else None,
                                       u.data_ptr() if u is not None else None, seed & (2 ** 64 - 1),
                                       offset & (2 ** 64 - 1), thr_c, minmax.data_ptr(), B, rows, ln, ld, sb,
                                       _stream(x.device)), "tb_salt_pepper_f32")
    return out


def disk_mask_tensor(shape: Sequence[int], r, dim: int, inside_off: bool, device: torch.device) -> torch.Tensor:
    """disk_mask.binary_mask_{2d,3d} (filters_and_operators.py:136-197) built on the device."""
    shape = tuple(int(s) for s in shape)
    grid = shape[-dim:]
    outer = int(np.prod(shape[:-dim])) if len(shape) > dim else 1
    n0, n1, n2 = (1,) + grid if dim == 2 else grid
    m = torch.empty(shape, dtype=torch.float32, device=device)
    if isinstance(r, (int, np.integer)) and not isinstance(r, bool):
        int_r, r2i, r2f = 1, int(r) * int(r), 0.0
    else:
        int_r, r2i = 0, 0
        r2 = float(r) ** 2
        r2f = float(np.float32(r2)) if np.isfinite(r2) else float("inf")
    with torch.cuda.device(device):
        check(lib().tb_disk_mask_f32(m.data_ptr(), outer, n0, n1, n2, int_r, r2i, r2f, 1 if inside_off else 0,
                                     _stream(device)), "tb_disk_mask_f32")
    return m


def logabs_sums(x: torch.Tensor, n_dims: int, programs: Sequence[Sequence], channels: int) -> torch.Tensor:
    """Sum over the full spectrum of log(|k|+1e-10) per volume-channel (float64 [B*C])."""
    require_hip(x, "logabs_sums")
    geo = geometry(x.shape[x.dim() - n_dims:])
    H, W, D = geo.hwd
    x = x.contiguous()
    bc, bstride, sp, sp_st = _bc_view(x, n_dims)
    sh, sw, sd = _hwd_strides(geo, sp_st)
    plan = plan_for(x.device, H, W, D)
    out = torch.empty(bc, dtype=torch.float64, device=x.device)
    with torch.cuda.device(x.device):
        ws = workspace(x.device, plan.workspace_bytes(bc))
        xs = (C.c_int64 * 3)(bstride, sh, sw)
        progs = programs_array(programs)
        check(lib().tb_kspace_logabs_sum_f32(plan.handle, x.data_ptr(), xs, ws.data_ptr(), ws.numel(), len(programs),
                                             channels, C.addressof(progs), out.data_ptr(), _stream(x.device)),
              "tb_kspace_logabs_sum_f32")
    return out


def set_compiled_plans(enable: bool) -> None:
    """Passes A/C on the compile-time slab plans (240x155, 128x128) when True (default), else the
    generic run-time-planned kernels (tb_set_compiled_plans)."""
    check(lib().tb_set_compiled_plans(1 if enable else 0))


def set_band_plans(enable: bool) -> None:
    """Band-limited passes A'/B'/C' for low-pass programs when True (default), else the full
    spectrum passes for every program (tb_set_band_plans)."""
    check(lib().tb_set_band_plans(1 if enable else 0))


def set_point_plans(enable: bool) -> None:
    """Spike-only programs (plane waves, k-space spikes) in closed form when True (default), else
    on the full-spectrum passes (tb_set_point_plans)."""
    check(lib().tb_set_point_plans(1 if enable else 0))


def set_wrap_plans(enable: bool) -> None:
    """Wrap-only programs on the separable route (2-tap H/W combine + D circulant, one image read
    and write) when True (default), else on the full-spectrum passes (tb_set_wrap_plans)."""
    check(lib().tb_set_wrap_plans(1 if enable else 0))


def set_half_units(enable: bool) -> None:
    """Full-spectrum passes A / C as half units (row parity) over a split spectrum where the plan
    has them (240 x 240 x 155) when True (default), else whole slabs (tb_set_half_units)."""
    check(lib().tb_set_half_units(1 if enable else 0))


def set_band_inv16(enable: bool) -> None:
    """Pass C' synthesis in split f16 on the matrix cores when True (default, where the launch's
    V rows fit), else the f32 MFMA synthesis (tb_set_band_inv16)."""
    check(lib().tb_set_band_inv16(1 if enable else 0))


def set_chain_chunk(n: int) -> None:
    """Channel-volumes per pass A -> B -> C chain (tb_set_chain_chunk): n > 0 chunks, 0 = whole
    batch group per pass, n < 0 = default (Infinity-Cache-sized chunks)."""
    check(lib().tb_set_chain_chunk(int(n)))


def set_pass_timing(enable: bool) -> None:
    check(lib().tb_set_pass_timing(1 if enable else 0))


def pass_times_ms() -> Tuple[List[float], List[int]]:
    ms = (C.c_float * 4)()
    cnt = (C.c_int * 4)()
    check(lib().tb_get_pass_times_ms(ms, cnt))
    return list(ms), list(cnt)


def pass_stats() -> Tuple[List[float], List[int], List[float], List[str]]:
    """Per pass slot (0 forward, 1 k-space, 2 inverse, 3 salt-and-pepper / min-max) since timing
    was enabled: summed ms, launch count, summed algorithmic bytes, last kernel name; clears."""
    ms = (C.c_float * 4)()
    cnt = (C.c_int * 4)()
    nb = (C.c_double * 4)()
    names = [lib().tb_pass_kernel(i).decode() for i in range(4)]
    check(lib().tb_get_pass_stats(ms, cnt, nb))
    return list(ms), list(cnt), list(nb), names
