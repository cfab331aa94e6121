"""ctypes mirror of include/texbias.h (structures and constants only; no library load).

Kept free of torch and of the HIP library so the op-program builders can be
used by the CPU test-suite against the host emulator as well.
"""
from __future__ import annotations

import ctypes as C

TB_OK = 0
TB_ERR_INVALID_ARG = 1
TB_ERR_UNSUPPORTED_SIZE = 2
TB_ERR_HIP = 3
TB_ERR_WORKSPACE = 4

TB_OP_NONE = 0
TB_OP_DISK = 1
TB_OP_GIBBS = 2
TB_OP_LAYER = 3
TB_OP_WRAP = 4
TB_OP_ZF = 6
TB_OP_SPIKE = 5

TB_MAX_OPS = 6
TB_MAX_BATCH = 8


class TbOp(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("chan", C.c_int32),
        ("i", C.c_int32 * 3),
        ("reserved", C.c_int32),
        ("l", C.c_int64),
        ("f", C.c_float * 4),
    ]


class TbSampleOps(C.Structure):
    _fields_ = [
        ("n", C.c_int32),
        ("reserved", C.c_int32 * 3),
        ("op", TbOp * TB_MAX_OPS),
    ]


assert C.sizeof(TbOp) == 48 and C.sizeof(TbSampleOps) == 304


def programs_array(programs):
    """list[list[TbOp]] -> ctypes array of TbSampleOps."""
    arr = (TbSampleOps * len(programs))()
    for b, prog in enumerate(programs):
        if len(prog) > TB_MAX_OPS:
            raise ValueError(f"at most {TB_MAX_OPS} k-space ops per sample, got {len(prog)}")
        arr[b].n = len(prog)
        for j, op in enumerate(prog):
            arr[b].op[j] = op
    return arr


class TbPrepParams(C.Structure):
    """tb_prep_params (include/texbias.h): one sample's preprocessing draws."""
    _fields_ = [("h0", C.c_int), ("w0", C.c_int), ("d0", C.c_int), ("flip", C.c_int),
                ("scale", C.c_float), ("shift", C.c_float), ("normalize", C.c_int), ("resample", C.c_int),
                ("m", C.c_float * 12)]
