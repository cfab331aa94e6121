#!/usr/bin/env python3
"""Phase timing of the full-spectrum passes (measurement tool; needs the -DTB_SLAB_PROF build).

    bash scripts/build_variant.sh prof -DTB_SLAB_PROF "kern_slab_ct kern_kspace_ct"
    TEXBIAS_LIB=var/prof.so python scripts/diag/slab_prof.py

Runs the gibbs-aug chain (RandGibbsNoised(alpha=(0, 0.4)), C3 shape) and prints, per pass, the mean
shader-clock cycles each barrier-separated phase takes (thread 0 of workgroups < 256 stamps the
clock after every barrier of its first 16 units; the first unit is left out of the means).
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT):
    sys.path.insert(0, p)

import torch  # noqa: E402


def phases(st, names):
    """st: [blocks, units, stamps] clock values; mean cycles of stamp i -> i+1 over units >= 1."""
    v = st[:, 1:, :]
    ok = (v[:, :, 0] > 0) & (v[:, :, len(names)] > 0)
    out = {}
    for i, nm in enumerate(names):
        d = (v[:, :, i + 1].astype(np.int64) - v[:, :, i].astype(np.int64))[ok]
        out[nm] = round(float(d.mean()), 0)
    unit = (v[:, :, len(names)].astype(np.int64) - v[:, :, 0].astype(np.int64))[ok]
    out["unit_total"] = round(float(unit.mean()), 0)
    # whole-unit period: stamp 0 of unit u+1 minus stamp 0 of unit u
    per = (st[:, 2:, 0].astype(np.int64) - st[:, 1:-1, 0].astype(np.int64))
    per = per[(st[:, 2:, 0] > 0) & (st[:, 1:-1, 0] > 0)]
    out["unit_period"] = round(float(per.mean()), 0) if per.size else None
    out["units_sampled"] = int(ok.sum())
    return out


def main():
    import filters_and_operators as F
    from texbias.pipeline import FusedChain
    from texbias.synth import brats_like

    lib = ctypes.CDLL(os.environ.get("TEXBIAS_LIB", ""))  # the handle texbias dlopens too
    for nm in ("tb_debug_slab_prof", "tb_debug_kspace_prof", "tb_debug_slab_prof_clear"):
        if not hasattr(lib, nm):
            raise SystemExit(f"{nm} missing: build the -DTB_SLAB_PROF variant and set TEXBIAS_LIB")
    dev = torch.device("cuda", 0)
    x = brats_like(2, 4, (240, 240, 155), seed=0, device=dev)
    g = F.RandGibbsNoised("image", prob=1.0, alpha=(0.0, 0.4))
    g.set_random_state(100)
    chain = FusedChain([g])
    for _ in range(3):
        chain(x, pad=5)
    torch.cuda.synchronize()
    lib.tb_debug_slab_prof_clear()
    chain(x, pad=5)
    torch.cuda.synchronize()
    a = np.zeros((2, 256, 16, 12), np.uint64)
    b = np.zeros((256, 16, 8), np.uint64)
    lib.tb_debug_slab_prof(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes))
    lib.tb_debug_kspace_prof(ctypes.c_void_p(b.ctypes.data), ctypes.c_size_t(b.nbytes))
    res = {
        "A_k_slab_fwd_ct16": phases(a[0], ["wait_prev", "raw_store", "raw_read", "F0+prefetch", "D1",
                                           "U_read", "U_write", "W0", "W1_store"]),
        "C_k_slab_inv_ct": phases(a[1], ["wait_prev", "G0", "G1", "RE_load", "RE+prefetch", "E0_store",
                                         "pad+minmax"]),
        "B_k_kspace_ct2p": phases(b, ["wait_prev", "S0+prefetch", "mid", "S1_store"]),
    }
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
