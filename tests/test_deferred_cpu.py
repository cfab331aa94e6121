"""Deferred texbias transforms inside DataLoader workers (texbias.deferred), host side: the plans a
worker records equal the draws an in-process replay of that worker makes; the image is left
untouched for the GPU pass; a batch with plans cannot slip through default_collate; the guard
catches an image modified after a deferred filter."""
import pytest
import torch

from _deferred_case import DictSet, emulate, make_transforms, worker_seed


def _sig(plan):
    out = []
    for st in plan.stages:
        if st[0] == "k":
            out.append(("k", [(o.kind, o.chan, tuple(o.i), o.l, tuple(repr(round(float(f), 6)) for f in o.f), o.reserved)
                              for o in st[1]]))
        else:
            out.append(tuple(st))
    return out


def test_worker_plans_match_replay():
    from texbias.deferred import deferred_collate, set_deferred
    ts = make_transforms()
    loader = torch.utils.data.DataLoader(DictSet(ts), batch_size=2, num_workers=2, collate_fn=deferred_collate,
                                         worker_init_fn=worker_seed)
    got = {}
    for bi, batch in enumerate(loader):
        plans = batch["image_texbias_plan"]
        assert len(plans) == 2 and batch["label"].shape == (2, 1, 24, 20, 16)
        assert batch["image"].shape == (2, 4, 24, 20, 16)           # untouched: the filters run later
        for j, pl in enumerate(plans):
            assert [s[0] for s in pl.stages] == ["k", "k", "k", "sap", "sel"]
            got[2 * bi + j] = _sig(pl)
    set_deferred(True)
    try:
        ref = emulate(make_transforms(), 2, 2, lambda d: _sig(d["image_texbias_plan"]))
    finally:
        set_deferred(None)
    assert got == ref
    # the draws really vary: some samples skipped a filter, the channel choice differs
    assert len({str(v) for v in got.values()}) >= 4


def test_default_collate_refuses_plans():
    ts = make_transforms()
    loader = torch.utils.data.DataLoader(DictSet(ts), batch_size=2, num_workers=1)
    with pytest.raises(Exception):
        next(iter(loader))


def test_guard_catches_late_modification():
    from texbias.deferred import deferred_collate, run_deferred, set_deferred

    class Scale:  # a non-texbias transform after a deferred filter
        def __call__(self, d):
            d = dict(d)
            d["image"] = d["image"] * 2
            return d

    import filters_and_operators as F
    ts = [F.RandFourierDiskMaskd(keys="image", r=5.0, prob=1.0), Scale()]
    set_deferred(True)
    try:
        ds = DictSet(ts)
        batch = deferred_collate([ds[0], ds[1]])
    finally:
        set_deferred(None)
    with pytest.raises(RuntimeError, match="changed after a deferred"):
        run_deferred(batch, device=torch.device("cpu"))


def test_guard_catches_late_flip():
    """A transform that only rearranges voxels (a flip keeps every value, so an order-independent
    checksum would pass it) after a deferred filter is caught too."""
    from texbias.deferred import deferred_collate, run_deferred, set_deferred

    class Flip:
        def __call__(self, d):
            d = dict(d)
            d["image"] = torch.flip(torch.as_tensor(d["image"]), dims=[-1])
            return d

    import filters_and_operators as F
    ts = [F.WrapArtifactd("image", 0.5), Flip()]
    set_deferred(True)
    try:
        ds = DictSet(ts)
        batch = deferred_collate([ds[0], ds[1]])
    finally:
        set_deferred(None)
    with pytest.raises(RuntimeError, match="changed after a deferred"):
        run_deferred(batch, device=torch.device("cpu"))
