"""Evaluation harness: the reference's ``model_evaluation`` on the device.

Reference: source_code/utils.py:241-465 (``model_evaluation``): load a trained U-Net, run a test
loader, post-process the logits with ``Activations(sigmoid=True)`` + ``AsDiscrete(threshold 0.5)``
and accumulate MONAI 0.5 ``DiceMetric(include_background=True, reduction="mean")`` over the whole
label and per channel (TC, WT, ET), weighting every batch's mean by its count of non-NaN
(instance, channel) entries; ``add_eval`` stores the numbers under a name, ``save`` /
``load_dict`` persist them.

Here the thresholded Dice statistics come from one fused HIP sweep per batch
(``tb_dice_metric_sums_f32``: {sum t p, sum t, sum p} per instance and channel) and the running
sums stay on the device -- one host sync per evaluation instead of four per batch.  DiceMetric
semantics (MONAI 0.5 ``compute_meandice``): dice = 2 |P n T| / (|P| + |T|) per (instance,
channel), NaN where the ground truth is empty; ``reduction="mean"`` averages the non-NaN entries.
MONAI is not installed here, so the metric's parity is unpinned beyond this restatement
(``tests/test_gpu_eval.py`` checks it against a plain torch formula).

``BratsValIterDataset`` is the reference's per-filter evaluation set (utils.py:159-235): the fixed
validation split (``random_split(ds, [48, 48], Generator().manual_seed(0))``, second half) through
the validation Compose -- Spacingd(1.5, 1.5, 2.0) -> Orientationd(RAS) ->
CenterSpatialCropd(128, 128, 64) -> NormalizeIntensityd(nonzero, channel_wise) -- with one named
filter appended, one name at a time.  Here the Compose runs on the device over each collated
batch: ``texbias.prep.BratsPrep`` (one resample gather + normalisation), then the filter as a
``FusedChain``.  Filter draws: indexed samples (the reference's ``test_ds`` read in the main
process) draw sequentially from the filter object; batched iteration mirrors the reference's
``DataLoader(batch_size=2, shuffle=False, num_workers=4)``, whose 4 worker processes each hold a copy of
the transform's ``RandomState`` taken when the epoch starts and receive batches round-robin -- batch k
draws from copy k % 4 (``loader_workers``).  Per-sample draw parity with MONAI's loader is unpinned
(MONAI absent); the mapping restates torch's worker assignment.  ``ModelEvaluation`` loads ``Gibbs_UNet`` / ``Spikes_UNet``
checkpoints like the reference (``gibbs_unet=`` / ``spikes_unet=``, utils.py:286-297).
"""
from __future__ import annotations

import copy
import json
import math
from typing import Dict, Iterable, Optional, Tuple

import numpy as np
import torch

from ._lib import check, lib
from .train import reference_model

VAL_ROI = (128, 128, 64)     # CenterSpatialCropd(roi_size=[128, 128, 64]), utils.py:194
VAL_PIXDIM = (1.5, 1.5, 2.0)  # Spacingd(pixdim=(1.5, 1.5, 2.0)), utils.py:190-192


def dice_metric_sums(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """[N, C, *spatial] logits and 0/1 target -> float64 [N, C, 3] {sum t p, sum t, sum p}, p = sigmoid >= 0.5."""
    if logits.shape != target.shape:
        raise AssertionError(f"ground truth has differing shape ({target.shape}) from input ({logits.shape})")
    x = logits.float().contiguous()
    t = target.float().contiguous()
    n, c = x.shape[:2]
    sums = torch.empty((n, c, 3), dtype=torch.float64, device=x.device)
    with torch.cuda.device(x.device):
        check(lib().tb_dice_metric_sums_f32(x.data_ptr(), t.data_ptr(), sums.data_ptr(), n * c, math.prod(x.shape[2:]),
                                            torch.cuda.current_stream(x.device).cuda_stream), "tb_dice_metric_sums_f32")
    return sums


def dice_from_sums(s: torch.Tensor) -> torch.Tensor:
    """[..., 3] sums -> dice per entry, NaN where the ground truth is empty (DiceMetric)."""
    inter, t, p = s[..., 0], s[..., 1], s[..., 2]
    return torch.where(t > 0, 2.0 * inter / (t + p), torch.full_like(t, float("nan")))


class _Acc:
    """Running sum of batch means weighted by their non-NaN counts (utils.py:378-402), on device."""

    def __init__(self, device):
        self.sum = torch.zeros((), dtype=torch.float64, device=device)
        self.count = torch.zeros((), dtype=torch.float64, device=device)

    def add(self, dice: torch.Tensor) -> None:
        ok = ~torch.isnan(dice)
        n = ok.sum().to(torch.float64)
        mean = torch.where(n > 0, torch.nan_to_num(dice, nan=0.0).sum() / n.clamp(min=1), torch.zeros_like(n))
        self.sum += mean * n
        self.count += n

    def value(self) -> float:
        return float((self.sum / self.count).item())


class ModelEvaluation:
    """``model_evaluation`` (utils.py:241-465) with the same method names."""

    def __init__(self, model_path: Optional[str] = None, instance_name: Optional[str] = None, in_channels: int = 4,
                 out_channels: int = 3, gibbs_unet: bool = False, spikes_unet: bool = False,
                 device: Optional[torch.device] = None, model: Optional[torch.nn.Module] = None):
        """As the reference (utils.py:256-279): a given ``model_path`` is loaded at once, as a
        Gibbs_UNet, a Spikes_UNet or the plain U-Net."""
        self.model_path = model_path
        self.instance_name = instance_name
        self.in_channels, self.out_channels = in_channels, out_channels
        self.gibbs_unet, self.spikes_unet = gibbs_unet, spikes_unet
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.model = model.to(self.device) if model is not None else None
        self.eval_dict: Dict[str, Dict] = {}
        if model_path and model is None:
            if gibbs_unet:
                self.load_gibbs_unet()
            elif spikes_unet:
                self.load_spikes_unet()
            else:
                self.load_UNet()

    def _state(self):
        return torch.load(self.model_path, map_location=self.device, weights_only=True)

    def load_UNet(self) -> None:
        """The reference's U-Net from a state dict (tensors only: ``weights_only=True``)."""
        self.model = reference_model(self.in_channels, self.out_channels).to(self.device)
        self.model.load_state_dict(self._state())

    def load_gibbs_unet(self) -> None:
        """A ``Gibbs_UNet`` (utils.py:286-290).  The reference's layer keeps alpha out of its
        state dict; such a checkpoint loads with alpha at the class default (0.5)."""
        from stylization_layers import Gibbs_UNet
        self.model = Gibbs_UNet().to(self.device)
        missing, unexpected = self.model.load_state_dict(self._state(), strict=False)
        if unexpected or any(k != "gibbs.alpha" for k in missing):
            raise RuntimeError(f"Gibbs_UNet state dict mismatch: missing {missing}, unexpected {unexpected}")

    def load_spikes_unet(self) -> None:
        """A ``Spikes_UNet`` (utils.py:292-296)."""
        from stylization_layers import Spikes_UNet
        self.model = Spikes_UNet().to(self.device)
        self.model.load_state_dict(self._state())

    def _batches(self, loader: Iterable):
        for data in loader:
            yield data["image"].to(self.device, non_blocking=True), data["label"].to(self.device, non_blocking=True)

    def _require(self):
        if self.model is None:
            raise RuntimeError(f"current model is {self.model}. Use load_UNet to load model.")

    def dataset_eval_single(self, test_loader: Iterable) -> float:
        """Mean Dice over every (instance, channel) with a non-empty ground truth."""
        self._require()
        self.model.eval()
        acc = _Acc(self.device)
        with torch.no_grad():
            for x, y in self._batches(test_loader):
                acc.add(dice_from_sums(dice_metric_sums(self.model(x), y)))
        return acc.value()

    def dataset_eval_multi(self, test_loader: Iterable) -> Tuple[float, float, float, float]:
        """(mean, ET, TC, WT) -- the reference's return order (utils.py:411); channels are (TC, WT, ET)."""
        self._require()
        self.model.eval()
        accs = [_Acc(self.device) for _ in range(4)]
        with torch.no_grad():
            for x, y in self._batches(test_loader):
                d = dice_from_sums(dice_metric_sums(self.model(x), y))
                accs[0].add(d)
                for k in range(3):
                    accs[1 + k].add(d[:, k])
        mean, tc, wt, et = (a.value() for a in accs)
        return mean, et, tc, wt

    def add_eval(self, name: str, test_loader: Iterable, data_dict: Optional[dict] = None) -> None:
        m, et, tc, wt = self.dataset_eval_multi(test_loader)
        self.eval_dict[name] = {"mean": m, "et": et, "tc": tc, "wt": wt, **(data_dict or {})}

    def save(self, filename: Optional[str] = None) -> str:
        """JSON instead of the reference's pickle (nothing executable in the file)."""
        filename = filename or f"{self.instance_name or 'model_evaluation'}.json"
        with open(filename, "w") as f:
            json.dump({"model_path": self.model_path, "instance_name": self.instance_name,
                       "eval_dict": self.eval_dict}, f)
        return filename

    def load_dict(self, filename: str) -> None:
        with open(filename) as f:
            d = json.load(f)
        self.model_path, self.instance_name, self.eval_dict = d["model_path"], d["instance_name"], d["eval_dict"]


class _FilteredSplit:
    """One named filter's validation set: ``len`` samples, indexable (one sample dict, as the
    reference's ``Subset``) and iterable in batches (as its ``DataLoader(batch_size, shuffle=False)``)."""

    def __init__(self, owner: "BratsValIterDataset", name: str, batched: bool):
        self.owner, self.name, self.batched = owner, name, batched

    def __len__(self) -> int:
        return len(self.owner.test_indices)

    def _run(self, idx):
        return self.owner.run(self.name, idx)

    def __getitem__(self, i: int) -> Dict[str, torch.Tensor]:
        d = self._run([self.owner.test_indices[i]])
        return {k: v[0] for k, v in d.items()}

    def __iter__(self):
        ids, bs = self.owner.test_indices, self.owner.batch_size if self.batched else 1
        nw = self.owner.loader_workers if self.batched else 1
        # batched: one copy of the filter per loader worker, taken at the start of the epoch; batch k
        # goes to worker k % nw (torch's DataLoader order with shuffle=False)
        copies = [copy.deepcopy(self.owner.transforms[self.name]) for _ in range(nw)] if nw > 1 else None
        for k, b0 in enumerate(range(0, len(ids), bs)):
            d = self.owner.run(self.name, ids[b0:b0 + bs], copies[k % nw] if copies else None)
            if self.batched:
                yield d
            else:
                yield {k: v[0] for k, v in d.items()}


class BratsValIterDataset:
    """utils.py:159-235 on the device.

    ``source``: the validation section (the reference's ``DecathlonDataset(section="validation")``,
    96 BraTS cases) as a sequence of ``(image [4, H, W, D], label [H, W, D] class ids[, affine])``
    raw volumes, on the host or the device; ``transforms``: ``{name: transform}`` of the
    reference's filter objects (e.g. ``{"sap10": SaltAndPepper(0.10)}``), each appended to the
    validation Compose in turn.  ``return_loader``: yield batched loaders (batch 2, unshuffled)
    instead of per-sample datasets.  ``split``: the ``random_split`` lengths; the test half is kept.
    ``loader_workers``: worker copies of the filter's random state in batched iteration (the
    reference's ``num_workers=4``; 1 = one sequential stream).
    """

    def __init__(self, source, transforms: Dict, return_loader: bool = False, batch_size: int = 2,
                 split: Tuple[int, int] = (48, 48), seed: int = 0, device: Optional[torch.device] = None,
                 pixdim=VAL_PIXDIM, axcodes: str = "RAS", roi=VAL_ROI, loader_workers: int = 4):
        from .prep import BratsPrep
        if len(source) != sum(split):
            raise ValueError(f"random_split lengths {split} do not sum to the dataset size {len(source)}")
        self.source, self.transforms = source, dict(transforms)
        self.return_loader, self.batch_size = return_loader, int(batch_size)
        self.loader_workers = max(1, int(loader_workers))
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        # torch.utils.data.random_split: randperm(n, generator) then consecutive lengths
        perm = torch.randperm(sum(split), generator=torch.Generator().manual_seed(seed)).tolist()
        self.test_indices = perm[split[0]:]
        self.prep = BratsPrep(roi_size=roi, flip_prob=0.0, scale_prob=0.0, shift_prob=0.0, pixdim=pixdim,
                              axcodes=axcodes, center_crop=True)

    def run(self, name: str, idx, transform=None) -> Dict[str, torch.Tensor]:
        """The validation Compose + filter ``name`` (or ``transform``, a worker's copy of it) on the
        samples ``idx`` (one device batch)."""
        from .pipeline import FusedChain
        items = [self.source[i] for i in idx]
        img = torch.stack([torch.as_tensor(it[0], dtype=torch.float32) for it in items]).to(self.device)
        lab = torch.stack([torch.as_tensor(it[1], dtype=torch.float32) for it in items]).to(self.device)
        affs = [np.asarray(it[2], dtype=float) if len(it) > 2 else np.eye(4) for it in items]
        x, y = self.prep(img, lab, affines=affs)
        x = FusedChain([transform if transform is not None else self.transforms[name]])(x)
        return {"image": x, "label": y}

    def __iter__(self):
        for name in self.transforms:
            yield name, _FilteredSplit(self, name, self.return_loader)

    def __getitem__(self, key: str):
        if key not in self.transforms:
            raise KeyError(key)
        return _FilteredSplit(self, key, self.return_loader)
