"""The per-(device, stream) workspace caches are bounded (texbias.runtime): a caller that uses a fresh
stream per iteration does not keep one spectrum-sized buffer per stream it ever used."""
from collections import OrderedDict

import torch


def test_workspace_cache_is_lru_bounded(monkeypatch):
    from texbias import runtime as rt
    keys = iter(range(100))
    monkeypatch.setattr(rt, "_ws_key", lambda device: (0, next(keys)))
    monkeypatch.setattr(torch, "empty", lambda n, dtype=None, device=None: torch.zeros(1, dtype=torch.uint8).expand(n))
    cache = OrderedDict()
    for _ in range(20):
        rt._cached_ws(cache, torch.device("cpu"), 16)
    assert len(cache) == rt._WS_CAP
    assert list(cache) == [(0, k) for k in range(20 - rt._WS_CAP, 20)]
