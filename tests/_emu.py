"""ctypes harness for the host emulator (tests/emu/emu.cpp) -- test infrastructure."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "medical-vision-textural-bias_amd")
SRC = os.path.join(HERE, "emu", "emu.cpp")
HDRS = [os.path.join(PKG, "csrc", h) for h in ("fft_core.h", "slab_ct.h", "kspace_ct.h", "plan_host.h", "sap_core.h")] + \
       [os.path.join(ROOT, "include", "texbias.h")]
OUT = os.path.join(HERE, "emu", "_build", "libtexbias_emu.so")

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    newest = max(os.path.getmtime(p) for p in [SRC] + HDRS)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < newest:
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        tmp = OUT + f".{os.getpid()}.tmp"
        # host clang++ (two-lane ext_vector complex type of slab_ct.h)
        cxx = os.environ.get("TB_EMU_CXX", "/opt/rocm/lib/llvm/bin/clang++")
        subprocess.check_call([cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-Wno-unknown-pragmas",
                               "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "csrc"),
                               SRC, "-o", tmp])
        os.replace(tmp, OUT)
    L = C.CDLL(OUT)
    L.tbemu_kspace_filter_f32.restype = C.c_int
    L.tbemu_kspace_filter_f32.argtypes = [C.c_int] * 3 + [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                          C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    L.tbemu_radices.argtypes = [C.c_int, C.c_void_p]
    L.tbemu_philox_u01.argtypes = [C.c_uint64, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p]
    L.tbemu_philox_u01.restype = None
    L.tbemu_sap_class.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_float, C.c_void_p]
    L.tbemu_f2key.argtypes = [C.c_float]
    L.tbemu_f2key.restype = C.c_uint32
    L.tbemu_key2f.argtypes = [C.c_uint32]
    L.tbemu_key2f.restype = C.c_float
    _lib = L
    return L


def kspace_filter(x: np.ndarray, n_dims: int, programs, pad: int = 0, T: int = 0, ct: bool = False):
    """x: [B, C, *spatial] float32 (numpy).  Returns (y [B, C, *spatial(+pad on last)], minmax [B,2]).
    ``ct``: passes A and C through the compile-time slab plan (slab_ct.h) when the shape has one."""
    from texbias._abi import programs_array
    from texbias.kprog import geometry
    x = np.ascontiguousarray(x, np.float32)
    B, Cc = x.shape[0], x.shape[1]
    spatial = x.shape[2:]
    assert len(spatial) == n_dims
    geo = geometry(spatial)
    H, W, D = geo.hwd
    xs = np.array([H * W * D, W * D, D], np.int64)
    ydpad = D + pad
    y = np.zeros((B * Cc, H, W, ydpad), np.float32)
    ys = np.array([H * W * ydpad, W * ydpad, ydpad], np.int64)
    mm = np.zeros((B, 2), np.float32)
    progs = programs_array(programs)
    rc = lib().tbemu_kspace_filter_f32(H, W, D, x.ctypes.data, xs.ctypes.data, y.ctypes.data, ys.ctypes.data, pad,
                                       B, Cc, C.addressof(progs), mm.ctypes.data, T, int(ct))
    if rc:
        raise RuntimeError(f"emulator error {rc}")
    if pad:
        return y.reshape(B, Cc, H, W, ydpad), mm
    return y.reshape(x.shape), mm
