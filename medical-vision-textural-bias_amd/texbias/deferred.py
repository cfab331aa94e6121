"""Deferred execution of the texture filters from DataLoader worker processes.

The reference's drivers run their transforms per sample inside ``DataLoader(num_workers=4)``
worker processes (e.g. 127_.../..._3modalities.py:231), which are forked and cannot open a HIP
context.  Inside a worker (``torch.utils.data.get_worker_info()`` is set) the texbias dictionary
transforms therefore do NOT compute: they make exactly the draws the eager call makes -- same
``RandomState`` calls, same order, the salt-and-pepper Philox key from the worker's torch
generator -- and append the sample's stage (an op program, a salt-and-pepper threshold, a channel
selection) to a ``TexbiasPlan`` stored next to the image under ``"<key>_texbias_plan"``.  The
main process then runs the whole batch's plans on the GPU in one batched pass
(``run_deferred``), after the default collation of everything else (``deferred_collate``).

Guards (the deferred result must equal the eager one): the plan records the image's shape and an
position-dependent digest of its bits when the first stage was deferred; ``run_deferred`` raises if the
collated image differs -- i.e. if a transform that is not a texbias transform modified the image
after a deferred filter (texbias transforms must close the Compose; ``SelectChanneld`` and
``MultimodalSlicesd`` defer too).  A batch holding plans cannot go through ``default_collate``
(it raises on the plan object), so a loader without ``deferred_collate`` fails loudly instead of
returning unfiltered images.
"""
from __future__ import annotations

import hashlib
import os
from typing import Any, Dict, List, Optional

import torch

PLAN_SUFFIX = "_texbias_plan"
_force: Optional[bool] = None


def set_deferred(flag: Optional[bool]) -> None:
    """Force deferral on/off in this process (None: automatic, i.e. inside DataLoader workers)."""
    global _force
    _force = flag


def active() -> bool:
    if _force is not None:
        return _force
    if os.environ.get("TEXBIAS_DEFER", "1") == "0":
        return False
    return torch.utils.data.get_worker_info() is not None


try:  # xxh3-128 hashes ~15 GB/s on one core (a 143 MB BraTS sample in ~10 ms); BLAKE2b ~1 GB/s
    import xxhash as _xx

    def _digest(buf) -> int:
        return _xx.xxh3_128_intdigest(buf)
except ImportError:  # pragma: no cover - xxhash ships with this image
    def _digest(buf) -> int:
        return int.from_bytes(hashlib.blake2b(buf, digest_size=16).digest(), "little")


def _checksum(t: torch.Tensor) -> int:
    """Position-dependent 128-bit digest of a float32 tensor's bits: a transform that only moves
    voxels (a flip, a transpose, a rot90) changes it as surely as one that changes values.  The
    bytes are hashed in place (no ``tobytes`` copy); a tensor already contiguous float32 on the CPU
    (the collated batch's samples) is not copied at all."""
    x = torch.as_tensor(t).detach()
    if x.device.type != "cpu" or x.dtype != torch.float32 or not x.is_contiguous():
        x = x.to(device="cpu", dtype=torch.float32).contiguous()
    return _digest(memoryview(x.numpy()).cast("B"))


class TexbiasPlan:
    """One sample's deferred stages: ('k', ops) k-space program, ('sap', p or None, seed) salt and
    pepper, ('sel', channel) channel selection -- in Compose order."""

    __slots__ = ("stages", "shape", "checksum")

    def __init__(self, image):
        self.stages: List[tuple] = []
        t = torch.as_tensor(image)
        self.shape = tuple(t.shape)
        self.checksum = _checksum(t)

    def __repr__(self) -> str:
        return f"TexbiasPlan(shape={self.shape}, stages={[s[0] for s in self.stages]})"


def record(d: Dict[Any, Any], key, stage: tuple) -> None:
    """Append ``stage`` to the plan of ``d[key]`` (creating it from the current image)."""
    pk = f"{key}{PLAN_SUFFIX}"
    plan = d.get(pk)
    if plan is None:
        plan = TexbiasPlan(d[key])
    d[pk] = plan
    plan.stages.append(stage)


def has_plan(d: Dict[Any, Any], key) -> bool:
    return f"{key}{PLAN_SUFFIX}" in d


def deferred_collate(batch: List[Dict[Any, Any]]):
    """``collate_fn`` for a DataLoader whose dataset ends in texbias transforms: the plans are
    gathered into a list per key, everything else goes through torch's ``default_collate``."""
    from torch.utils.data import default_collate
    if not isinstance(batch[0], dict):
        return default_collate(batch)
    plan_keys = [k for k in batch[0] if isinstance(k, str) and k.endswith(PLAN_SUFFIX)]
    plans = {k: [b.pop(k) for b in batch] for k in plan_keys}
    out = default_collate(batch)
    out.update(plans)
    return out


def _normalise(stages: List[tuple]) -> List[tuple]:
    """Consecutive k-space programs merge into one pass (the reference's .real between filters is
    what the half-spectrum program reproduces); empty programs vanish."""
    out: List[tuple] = []
    for st in stages:
        if st[0] == "k":
            if out and out[-1][0] == "k":
                out[-1] = ("k", list(out[-1][1]) + list(st[1]))
            else:
                out.append(("k", list(st[1])))
        else:
            out.append(st)
    return out


def run_deferred(batch: Dict[Any, Any], device: Optional[torch.device] = None, key: str = "image",
                 pad: int = 0) -> Dict[Any, Any]:
    """Run the collated batch's deferred plans for ``key`` on ``device`` (default: the current HIP
    device); returns the batch with ``batch[key]`` filtered (on the device) and the plans removed."""
    from .pipeline import FusedChain
    pk = f"{key}{PLAN_SUFFIX}"
    out = dict(batch)
    plans = out.pop(pk, None)
    dev = device or torch.device("cuda", torch.cuda.current_device())
    x = torch.as_tensor(out[key]).to(device=dev, dtype=torch.float32)
    if plans is None:
        out[key] = x
        return out
    if len(plans) != x.shape[0]:
        raise ValueError(f"{len(plans)} plans for a batch of {x.shape[0]}")
    xc = out[key] if not torch.is_tensor(out[key]) or out[key].device.type == "cpu" else x
    for b, pl in enumerate(plans):
        if tuple(x.shape[1:]) != pl.shape or _checksum(torch.as_tensor(xc[b])) != pl.checksum:
            raise RuntimeError(
                f"sample {b}: the image changed after a deferred texbias filter (shape {tuple(x.shape[1:])} vs "
                f"{pl.shape}); only texbias transforms (and SelectChanneld / MultimodalSlicesd from "
                "filters_and_operators) may follow the first texbias filter in a deferred Compose")
    stages = [_normalise(pl.stages) for pl in plans]
    out[key] = FusedChain([], key=key).execute(x, stages, pad=pad)
    return out


class DeferredLoader:
    """Iterate a DataLoader built with ``collate_fn=deferred_collate`` and hand out batches whose
    texbias plans have run on the GPU: ``for batch in DeferredLoader(loader, device): ...``."""

    def __init__(self, loader, device: Optional[torch.device] = None, keys=("image",), pad: int = 0):
        self.loader, self.device, self.keys, self.pad = loader, device, tuple(keys), pad

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            for k in self.keys:
                batch = run_deferred(batch, self.device, key=k, pad=self.pad)
            yield batch
