"""Loader of the in-tree HIP library (libtexbias.so) with ctypes prototypes.

There is no CPU fallback: if the library is missing or no HIP device is
visible, every entry point raises.  Build it with ``python __graft_entry__.py``
(``build()``) or ``make -C medical-vision-textural-bias_amd/csrc``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from ._abi import TB_OK

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("TEXBIAS_LIB", os.path.join(PKG_DIR, "libtexbias.so"))

_lock = threading.Lock()
_lib = None


class TexbiasError(RuntimeError):
    pass


def _proto(L):
    P, I, I64, U64, F, SZ = C.c_void_p, C.c_int, C.c_int64, C.c_uint64, C.c_float, C.c_size_t
    sig = {
        "tb_version": (I, []),
        "tb_error_string": (C.c_char_p, [I]),
        "tb_last_hip_error": (I, []),
        "tb_plan_create": (I, [I, I, I, C.POINTER(P)]),
        "tb_plan_destroy": (I, [P]),
        "tb_workspace_bytes": (SZ, [P, I]),
        "tb_plan_radices": (I, [P, I, P]),
        "tb_kspace_filter_f32": (I, [P, P, P, P, P, I, P, SZ, I, I, P, P, P]),
        "tb_planes_closed_form_f32": (I, [P, P, P, P, P, I, P, SZ, I, I, P, P, P]),
        "tb_salt_pepper_f32": (I, [P, P, P, P, U64, U64, P, P, I, I64, I, I64, I64, P]),
        "tb_minmax_f32": (I, [P, P, I, I64, I, I64, I64, P]),
        "tb_key_to_float": (F, [C.c_uint32]),
        "tb_disk_mask_f32": (I, [P, I64, I, I, I, I, I64, F, I, P]),
        "tb_kspace_logabs_sum_f32": (I, [P, P, P, P, SZ, I, I, P, P, P]),
        "tb_conv3d_wgrad_f32": (I, [P, P, P] + [I] * 11 + [P]),
        "tb_conv3d_wgrad_config": (I, [I] * 11 + [P]),
        "tb_conv3d_wgrad_ws_bytes": (I64, [I] * 11),
        "tb_conv3d_wgrad_ws_f32": (I, [P, P, P] + [I] * 11 + [P, SZ, P]),
        "tb_instnorm_prelu_workspace_bytes": (SZ, [I64]),
        "tb_instnorm_prelu_fwd_f32": (I, [P, P, P, P, P, I64, I64, F, P, SZ, P]),
        "tb_instnorm_prelu_bwd_f32": (I, [P, P, P, P, P, P, P, I64, I64, P, SZ, P]),
        "tb_channel_sum_f32": (I, [P, P, I64, I64, I64, P]),
        "tb_channel_sum_ws_bytes": (SZ, [I64, I64, I64]),
        "tb_channel_sum_ws_f32": (I, [P, P, I64, I64, I64, P, SZ, P]),
        "tb_adn_workspace_bytes": (SZ, [I64, I64, I64]),
        "tb_adam_f32": (I, [I, P, P, P, P, P, P, P] + [C.c_double] * 5 + [I, P]),
        "tb_adn_counters": (I64, [I64, I64]),
        "tb_adn_fwd_f32": (I, [P, I64, P, I64, P, I64, P, P, P, I64, I64, I64, F, P, SZ, P, P]),
        "tb_adn_bwd_f32": (I, [P, I64, P, I64, P, I64, P, P, P, P, P, P, I64, I64, I64, P, SZ, P, P]),
        "tb_conv3d_small_f32": (I, [P, P, P, P] + [I] * 6 + [P]),
        "tb_conv3d_small_add_f32": (I, [P, P, P, P, P] + [I] * 6 + [P]),
        "tb_conv3d_fwd16_add_f32": (I, [P, P, P, P, P] + [I] * 4 + [P]),
        "tb_conv3d_mfma_add_f32": (I, [P, P, P, P, P] + [I] * 5 + [P]),
        "tb_conv3d_mfma_dgrad_f32": (I, [P, P, P, I64, P] + [I] * 5 + [P]),
        "tb_conv3d_fwd16_dgrad_f32": (I, [P, P, P, I64, P] + [I] * 4 + [P]),
        "tb_conv3d_s2_fewin_f32": (I, [P, P, P, P] + [I] * 6 + [P]),
        "tb_convT3d_fewout_f32": (I, [P, P, P, P] + [I] * 6 + [P]),
        "tb_conv3d_fwd16_f32": (I, [P, P, P, P] + [I] * 4 + [P]),
        "tb_convT3d_mfma64_f32": (I, [P, P, P, P] + [I] * 4 + [P]),
        "tb_convT3d_mfma_f32": (I, [P, P, P, P] + [I] * 5 + [P]),
        "tb_conv3d_mfma_f32": (I, [P, P, P, P] + [I] * 5 + [P]),
        "tb_conv3d_gemm_workspace_bytes": (SZ, [I] * 9),
        "tb_conv3d_gemm_f32": (I, [I, P, I64, P, P, P, I64, P, I64] + [I] * 8 + [P, SZ, P]),
        "tb_conv3d_gemm_config": (I, [I] * 9 + [P]),
        "tb_dice_sums_f32": (I, [P, P, P, I64, I64, I, I, P]),
        "tb_dice_sums_ws_bytes": (SZ, [I64, I64]),
        "tb_dice_sums_ws_f32": (I, [P, P, P, I64, I64, I, I, P, SZ, P]),
        "tb_dice_sums_bwd_f32": (I, [P, P, P, P, I64, I64, I, I, P]),
        "tb_dice_metric_sums_f32": (I, [P, P, P, I64, I64, P]),
        "tb_dice_loss_f32": (I, [P, P, I64, I64, I, I, F, F, P]),
        "tb_dice_loss_bwd_f32": (I, [P, P, P, I64, I64, I, I, F, F, P]),
        "tb_set_compiled_plans": (I, [I]),
        "tb_set_chain_chunk": (I, [I]),
        "tb_set_pass_timing": (I, [I]),
        "tb_get_pass_times_ms": (I, [P, P]),
        "tb_get_pass_stats": (I, [P, P, P]),
        "tb_pass_kernel": (C.c_char_p, [I]),
        "tb_set_band_plans": (I, [I]),
        "tb_set_band_inv16": (I, [I]),
        "tb_set_point_plans": (I, [I]),
        "tb_set_wrap_plans": (I, [I]),
        "tb_set_half_units": (I, [I]),
        "tb_brats_prep_workspace_bytes": (SZ, [I, I]),
        "tb_brats_prep_f32": (I, [P, P, I, I, I, I, I, P, I, I, I, P, P, P, SZ, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def lib():
    """The loaded library (raises TexbiasError if it cannot be loaded)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise TexbiasError(
                    f"texbias HIP library not found at {LIB_PATH}; build it (python __graft_entry__.py) -- "
                    "there is no CPU fallback")
            L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            _proto(L)
            _lib = L
    return _lib


def check(rc: int, what: str = "texbias") -> None:
    if rc != TB_OK:
        L = lib()
        msg = L.tb_error_string(rc).decode()
        if rc == 3:
            msg += f" (hipError {L.tb_last_hip_error()})"
        raise TexbiasError(f"{what}: {msg}")
