"""MONAI-0.5-compatible transform protocol (used when ``monai`` is not importable).

The reference's filters subclass MONAI's ``Transform``, ``MapTransform``,
``Randomizable`` and ``RandomizableTransform`` (filters_and_operators.py:11-13).
Their RNG plumbing is part of the observable behaviour (which draws a seed
reproduces), so the semantics are kept: a class-level shared ``RandomState``
until ``set_random_state``; ``randomize`` draws ``R.rand() < prob``;
``key_iterator`` raises ``KeyError`` for a missing key unless
``allow_missing_keys``.  When MONAI is installed its own classes are used, so
``Compose.set_random_state`` and MONAI's worker seeding reach these transforms.
"""
from __future__ import annotations

from typing import Any, Hashable

import numpy as np

try:  # pragma: no cover - MONAI is absent in this image
    from monai.transforms import MapTransform, Randomizable, RandomizableTransform, Transform  # type: ignore
    from monai.utils import ensure_tuple  # type: ignore
    HAVE_MONAI = True
except Exception:  # noqa: BLE001
    HAVE_MONAI = False

    _MAX_SEED = 2 ** 32

    def ensure_tuple(vals: Any) -> tuple:
        if isinstance(vals, (str, bytes)) or not hasattr(vals, "__iter__"):
            return (vals,)
        return tuple(vals)

    class Transform:
        def __call__(self, data):  # pragma: no cover - abstract
            raise NotImplementedError(f"{type(self).__name__} must implement __call__")

    class Randomizable:
        R: np.random.RandomState = np.random.RandomState()

        def set_random_state(self, seed=None, state=None):
            if seed is not None:
                s = seed if isinstance(seed, (int, np.integer)) else id(seed)
                self.R = np.random.RandomState(int(s) % _MAX_SEED)
            elif state is not None:
                if not isinstance(state, np.random.RandomState):
                    raise TypeError(f"state must be None or a np.random.RandomState but is {type(state).__name__}.")
                self.R = state
            else:
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
                    raise TypeError(f"keys must be one of (Hashable, Iterable[Hashable]) but is {type(keys).__name__}.")

        def key_iterator(self, data, *extra_iterables):
            extras = extra_iterables if extra_iterables else [[None] * len(self.keys)]
            for key, *ex in zip(self.keys, *extras):
                if key in data:
                    yield (key,) + tuple(ex) if extra_iterables else key
                elif not self.allow_missing_keys:
                    raise KeyError(f"Key was missing ({key}) and allow_missing_keys==False")

__all__ = ["Transform", "MapTransform", "Randomizable", "RandomizableTransform", "ensure_tuple", "HAVE_MONAI"]
