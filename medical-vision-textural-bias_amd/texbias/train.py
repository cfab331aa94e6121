"""The reference's training step on PyTorch-ROCm, and its data-parallel form over RCCL.

Reference loop (e.g. 10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:226-243 and
127_.../..._3modalities.py:277-288): ``optimizer.zero_grad(); outputs = model(inputs);
loss = DiceLoss(sigmoid, squared_pred)(outputs, labels); loss.backward(); optimizer.step()``
with ``Adam(lr=1e-4, weight_decay=1e-5, amsgrad=True)`` and batch 2, on one GPU.

MI355X form: one process per GPU (torchrun), ``DistributedDataParallel`` whose gradient
all-reduce runs on RCCL (backend "nccl") over xGMI, bucketed and overlapped with the backward.
The U-Net has ~4.81 M fp32 parameters (19.2 MB of gradients): one 25 MB bucket would serialise
the whole all-reduce behind the last layer, so buckets are sized to a few MB to start reducing
the deep layers while the shallow ones are still in backward.  The loss stays on the device (no
per-step ``.item()`` sync).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import optim as _optim
from .losses import DiceLoss
from .unet import UNet, pack_parameters


def dist_env() -> Tuple[int, int, int]:
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init_distributed(backend: Optional[str] = None) -> Tuple[int, int, int]:
    rank, world, local = dist_env()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def reference_model(in_channels: int = 4, out_channels: int = 3) -> UNet:
    return UNet(dimensions=3, in_channels=in_channels, out_channels=out_channels, channels=(16, 32, 64, 128, 256),
                strides=(2, 2, 2, 2), num_res_units=2)


def step_conv_flops(model_fn, input_shape) -> int:
    """Analytic FLOPs of one train step's convolutions (measurement, not used by training): the model built
    by ``model_fn()`` on the meta device, one forward over ``input_shape`` recording every Conv3d /
    ConvTranspose3d's multiply-adds (Conv3d: output elements x Cin x k^3; ConvTranspose3d: input elements x
    Cout x k^3); per layer 2 x MACs for the forward, the weight gradient and -- unless its input is the
    network input -- the input gradient.  Norms, activations, the loss and Adam are left out (< 1 %)."""
    import math

    import torch.nn as nn
    with torch.device("meta"):
        m = model_fn()
    total = 0

    def hook(mod, inp, out):
        nonlocal total
        k = math.prod(mod.kernel_size)
        macs = inp[0].numel() * mod.out_channels * k if isinstance(mod, nn.ConvTranspose3d) else \
            out.numel() * mod.in_channels * k
        total += 2 * macs * (3 if inp[0].requires_grad else 2)

    hs = [c.register_forward_hook(hook) for c in m.modules() if isinstance(c, (nn.Conv3d, nn.ConvTranspose3d))]
    try:
        m(torch.empty(tuple(input_shape), device="meta"))
    finally:
        for h in hs:
            h.remove()
    return total


class TrainStep:
    """model / loss / optimizer of the reference, optionally wrapped in DDP."""

    def __init__(self, model: torch.nn.Module, device: torch.device, distributed: bool = False,
                 bucket_cap_mb: float = 4.0, channels_last: bool = False, capturable: bool = False):
        """``capturable``: the optimizer keeps its step counters on the device so the whole step can be
        captured in a HIP graph (torch.cuda.graph)."""
        self.device = device
        self.channels_last = channels_last
        model = model.to(device)
        pack_parameters(model)  # strided units' [unit0; residual] weights in one storage (unet.py), before DDP/Adam
        if channels_last:
            model = model.to(memory_format=torch.channels_last_3d)
        self.module = model
        if distributed:
            kw = dict(bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True, static_graph=True)
            if device.type == "cuda":
                kw["device_ids"] = [device.index]
            self.model = torch.nn.parallel.DistributedDataParallel(model, **kw)
        else:
            self.model = model
        self.loss_fn = DiceLoss(to_onehot_y=False, sigmoid=True, squared_pred=True)
        opt_kw = dict(lr=1e-4, weight_decay=1e-5, amsgrad=True)
        if device.type == "cuda" and _optim.ENABLED:  # one texbias launch (csrc/optim.hip); capturable
            self.opt = _optim.Adam(self.model.parameters(), **opt_kw)
            return
        if device.type == "cuda":
            opt_kw["fused"] = True
            if capturable:
                opt_kw["capturable"] = True
        try:
            self.opt = torch.optim.Adam(self.model.parameters(), **opt_kw)
        except (RuntimeError, TypeError):
            opt_kw.pop("fused", None)
            self.opt = torch.optim.Adam(self.model.parameters(), **opt_kw)

    def __call__(self, inputs: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        if self.channels_last:
            inputs = inputs.contiguous(memory_format=torch.channels_last_3d)
        self.opt.zero_grad(set_to_none=True)
        out = self.model(inputs)
        loss = self.loss_fn(out, labels)
        loss.backward()
        self.opt.step()
        return loss.detach()


@torch.no_grad()
def gibbs_gd(inputs: torch.Tensor, labels: torch.Tensor, model: torch.nn.Module, loss_fn, layer=None,
             h: float = 0.01, learning_rate: float = 0.02) -> Tuple[torch.Tensor, torch.Tensor]:
    """Finite-difference update of a Gibbs layer's alpha (Gibbs_GD,
    10_scripts/300_instutional_distribution/350_stylized_layers/gibbs0p7_layer_domain_GD.py:252-269):
    loss at alpha and at alpha + h on the same batch, delta = (L_h - L_0) / h,
    alpha <- alpha - learning_rate * delta.

    ``layer`` defaults to ``model.gibbs`` (through a DDP wrapper).  Data-parallel form (the
    reference trains on one GPU): every rank sees a different batch, so the per-rank slopes differ;
    one 2-element all-reduce averages (delta, L_0) over the ranks before the update, and every
    replica's alpha moves identically.  Returns (L_0, alpha) as device tensors -- no host sync (the
    reference's ``.item()`` calls are left to the caller)."""
    if layer is None:
        layer = getattr(model, "module", model).gibbs
    # alpha is updated IN PLACE: the Gibbs kernel reads it through its device address (ops.py
    # _layer_apply), so a captured HIP graph keeps reading the live value after this update
    old = layer.alpha.clone()
    l0 = loss_fn(model(inputs), labels)
    layer.alpha.copy_(old + h)
    lh = loss_fn(model(inputs), labels)
    buf = torch.stack([(lh - l0) / h, l0]).to(torch.float32)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        buf /= dist.get_world_size()
    layer.alpha.copy_(old - learning_rate * buf[0].to(old.dtype))
    return buf[1], layer.alpha.clone()


@torch.no_grad()
def spike_gd(inputs: torch.Tensor, labels: torch.Tensor, model: torch.nn.Module, loss_fn, layer=None,
             h: float = 0.05, learning_rate: float = 0.1) -> Tuple[torch.Tensor, float]:
    """Finite-difference update of a spike layer's log-intensity (the spike drivers' Gibbs_GD,
    10_scripts/300_instutional_distribution/350_stylized_layers/spikes11_layer_domain_GD.py:260-275):
    loss at I and at I + h on the same batch (each forward draws its own spike location, as the
    reference's fresh RandKSpaceSpikeNoise does), I <- I - learning_rate * (L_h - L_0) / h.  The layer
    keeps I on the host (it builds the transform from ``intensity.item()``), so the update reads the
    slope back once per step, as the reference's ``.item()`` does.  Data-parallel: the slope and L_0
    are averaged over the ranks first (one 2-float all-reduce).  Returns (L_0 device tensor, new I)."""
    if layer is None:
        layer = getattr(model, "module", model).spike
    old = layer.intensity.clone()
    l0 = loss_fn(model(inputs), labels)
    layer.intensity = old + h
    lh = loss_fn(model(inputs), labels)
    buf = torch.stack([(lh - l0) / h, l0]).to(torch.float32)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM)
        buf /= dist.get_world_size()
    layer.intensity = old - learning_rate * float(buf[0].item())
    return buf[1], float(layer.intensity.item())
