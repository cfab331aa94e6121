"""Loader for the golden fixtures written by tests/golden/make_golden.py."""
from __future__ import annotations

import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases(prefix: str):
    """Return {case_name: (meta_dict, {array_name: ndarray})} for golden_<prefix>.npz."""
    out = {}
    with np.load(os.path.join(GOLDEN, f"golden_{prefix}.npz"), allow_pickle=False) as z:
        for key in z.files:
            name, field = key.rsplit(".", 1)
            meta, arrs = out.setdefault(name, ({}, {}))
            if field == "meta":
                meta.update(json.loads(str(z[key])))
            else:
                arrs[field] = z[key]
    return out


def all_prefixes():
    return sorted(os.path.basename(p)[len("golden_"):-4] for p in glob.glob(os.path.join(GOLDEN, "golden_*.npz")))


def relerr(a, b) -> float:
    """max|a-b| / max|b| -- the normwise criterion of SURVEY.md §8c."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))
