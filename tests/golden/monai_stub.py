"""Minimal stand-in for the MONAI 0.5 base classes the reference imports.

TEST INFRASTRUCTURE ONLY (used by ``make_golden.py`` in this container).

The reference's filter modules (``source_code/filters_and_operators.py:11-13``,
``source_code/stylization_layers.py:3-4``) import ``monai`` only for the
transform protocol and the per-transform ``RandomState`` plumbing; every piece
of filter arithmetic is the reference's own torch code.  MONAI is not installed
in this image, so ``make_golden.py`` registers this module under the names
``monai``, ``monai.transforms``, ``monai.config``, ``monai.utils`` and
``monai.networks.nets`` before importing the reference.  Semantics follow
MONAI 0.5.dev2113 (the version pinned by ``source_code/test.ipynb:53-55``):

* ``Randomizable.R`` is a CLASS-level ``np.random.RandomState`` shared by every
  instance until ``set_random_state`` gives the instance its own;
* ``RandomizableTransform.randomize`` draws ``R.rand() < prob``;
* ``MapTransform.key_iterator`` yields present keys and raises ``KeyError`` for
  a missing key unless ``allow_missing_keys``.
"""
from __future__ import annotations

import sys
import types
from typing import Any, Hashable

import numpy as np
import torch

MAX_SEED = np.iinfo(np.uint32).max + 1


def ensure_tuple(vals: Any) -> tuple:
    if isinstance(vals, (str, bytes)) or not hasattr(vals, "__iter__"):
        return (vals,)
    return tuple(vals)


class Transform:
    def __call__(self, data):  # pragma: no cover - abstract
        raise NotImplementedError


class Randomizable:
    R: np.random.RandomState = np.random.RandomState()

    def set_random_state(self, seed=None, state=None):
        if seed is not None:
            s = seed if isinstance(seed, (int, np.integer)) else id(seed)
            self.R = np.random.RandomState(int(s) % MAX_SEED)
            return self
        if state is not None:
            if not isinstance(state, np.random.RandomState):
                raise TypeError("state must be a np.random.RandomState")
            self.R = state
            return self
        self.R = np.random.RandomState()
        return self

    def randomize(self, data):  # pragma: no cover - abstract
        raise NotImplementedError


class RandomizableTransform(Randomizable, Transform):
    def __init__(self, prob: float = 1.0, do_transform: bool = True):
        self._do_transform = do_transform
        self.prob = min(max(prob, 0.0), 1.0)

    def randomize(self, data):
        self._do_transform = self.R.rand() < self.prob


class MapTransform(Transform):
    def __init__(self, keys, allow_missing_keys: bool = False):
        self.keys = ensure_tuple(keys)
        self.allow_missing_keys = allow_missing_keys
        if not self.keys:
            raise ValueError("keys must be non empty.")
        for key in self.keys:
            if not isinstance(key, Hashable):
                raise TypeError("keys must be hashable")

    def key_iterator(self, data, *extra_iterables):
        ex_iters = extra_iterables if extra_iterables else [[None] * len(self.keys)]
        for key, *ex in zip(self.keys, *ex_iters):
            if key in data:
                yield (key,) + tuple(ex) if extra_iterables else key
            elif not self.allow_missing_keys:
                raise KeyError(f"Key was missing ({key}) and allow_missing_keys==False")


class UNet(torch.nn.Module):
    """Placeholder: the golden generator never runs the reference U-Net."""

    def __init__(self, *a, **k):
        super().__init__()

    def forward(self, x):
        return x


def install() -> None:
    """Register this module as ``monai`` and its used sub-modules."""
    me = sys.modules[__name__]
    root = types.ModuleType("monai")
    for name in ("transforms", "config", "utils", "networks"):
        sub = types.ModuleType(f"monai.{name}")
        setattr(root, name, sub)
        sys.modules[f"monai.{name}"] = sub
    nets = types.ModuleType("monai.networks.nets")
    sys.modules["monai.networks.nets"] = nets
    root.networks.nets = nets
    t = sys.modules["monai.transforms"]
    t.Transform, t.MapTransform = me.Transform, me.MapTransform
    t.Randomizable, t.RandomizableTransform = me.Randomizable, me.RandomizableTransform
    sys.modules["monai.config"].KeysCollection = Any
    sys.modules["monai.utils"].ensure_tuple = me.ensure_tuple
    nets.UNet = me.UNet
    sys.modules["monai"] = root
