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
"""
from __future__ import annotations

import json
import math
from typing import Dict, Iterable, Optional, Tuple

import torch

from ._lib import check, lib
from .train import reference_model


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
                 out_channels: int = 3, device: Optional[torch.device] = None, model: Optional[torch.nn.Module] = None):
        self.model_path = model_path
        self.instance_name = instance_name
        self.in_channels, self.out_channels = in_channels, out_channels
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.model = model.to(self.device) if model is not None else None
        self.eval_dict: Dict[str, Dict] = {}

    def load_UNet(self) -> None:
        """The reference's U-Net from a state dict (tensors only: ``weights_only=True``)."""
        self.model = reference_model(self.in_channels, self.out_channels).to(self.device)
        state = torch.load(self.model_path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(state)

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
