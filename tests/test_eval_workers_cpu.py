"""Batched validation iteration mirrors the reference's DataLoader(batch_size=2, shuffle=False,
num_workers=4) (source_code/utils.py:215): each epoch, every worker holds its own copy of the filter's
random state and batch k runs on worker k % 4; indexed samples draw from the object itself."""
import torch


def test_batches_draw_from_per_worker_copies(monkeypatch):
    from texbias.evaluation import BratsValIterDataset

    class Tr:  # stands in for a texbias filter object
        pass

    src = [(None, None)] * 16
    ds = BratsValIterDataset(src, {"f": Tr()}, return_loader=True, split=(4, 12), device=torch.device("cpu"))
    seen = []
    monkeypatch.setattr(ds, "run", lambda name, idx, transform=None: seen.append((tuple(idx), transform)) or {})
    list(ds["f"])
    assert [len(i) for i, _ in seen] == [2] * 6
    tfs = [t for _, t in seen]
    assert all(t is not None and t is not ds.transforms["f"] for t in tfs)
    assert [tfs.index(t) for t in tfs] == [0, 1, 2, 3, 0, 1]   # batch k -> worker k % 4
    first = tfs[0]
    seen.clear()
    list(ds["f"])                                               # a new epoch: fresh worker copies
    assert seen[0][1] is not first
    one = BratsValIterDataset(src, {"f": Tr()}, return_loader=False, split=(4, 12), device=torch.device("cpu"))
    seen.clear()
    monkeypatch.setattr(one, "run", lambda name, idx, transform=None: seen.append((tuple(idx), transform)) or {"x": [0]})
    list(one["f"])
    assert all(t is None for _, t in seen)                      # sequential draws from the object itself
