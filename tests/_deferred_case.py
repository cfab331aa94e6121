"""Shared fixture of the deferred-DataLoader tests: a small dict dataset through the reference's
127_* Compose order (disk -> plane wave -> wrap -> salt-and-pepper -> MultimodalSlicesd,
10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/..._3modalities.py:171-175)."""
import copy

import torch

SPATIAL = (24, 20, 16)
N = 8


class DictSet(torch.utils.data.Dataset):
    def __init__(self, transforms):
        g = torch.Generator().manual_seed(5)
        self.items = [{"image": torch.randn((4,) + SPATIAL, generator=g),
                       "label": (torch.rand((3,) + SPATIAL, generator=g) > 0.7).float()} for _ in range(N)]
        self.transforms = transforms

    def __len__(self):
        return N

    def __getitem__(self, i):
        d = dict(self.items[i])
        for t in self.transforms:
            d = t(d)
        return d


def make_transforms():
    import filters_and_operators as F
    disk = F.RandFourierDiskMaskd(keys="image", r=5.0, inside_off=False, prob=0.7)
    planes = F.RandPlaneWaves_ellipsoid("image", 6.0, 5.0, 4.0, intensity_value=8.0, prob=0.6)
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.1, prob=0.8)
    mm = F.MultimodalSlicesd(keys=["image", "label"], img_chan_indices=[0, 1, 2, 3], label_idx=1, seed=9)
    for j, t in enumerate((disk, planes, sap)):
        t.set_random_state(30 + j)
    planes.ellipsoid.set_random_state(37)
    return [disk, planes, wrap, sap, mm]


def worker_seed(wid):
    torch.manual_seed(100 + wid)


def worker_batches(n_workers, batch_size):
    """{worker: [batch indices]} for an unshuffled loader."""
    nb = (N + batch_size - 1) // batch_size
    return {w: [b for b in range(nb) if b % n_workers == w] for w in range(n_workers)}


def emulate(transforms, n_workers, batch_size, fn):
    """Replay each worker's samples in the main process with a fresh copy of the transforms (the
    fork's copy) and the worker's torch seed; fn(d) -> per-sample result, keyed by sample index."""
    out = {}
    for w, batches in worker_batches(n_workers, batch_size).items():
        ts = copy.deepcopy(transforms)
        worker_seed(w)
        ds = DictSet(ts)
        for b in batches:
            for i in range(b * batch_size, min(N, (b + 1) * batch_size)):
                out[i] = fn(ds[i])
    return out
