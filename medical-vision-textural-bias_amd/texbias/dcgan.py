"""DCGAN on (filtered) BraTS slices -- BASELINE config 5, SURVEY §8f-2.

Reference: 50_reconstruction/networks.py:18-95 (Generator / Discriminator for 1 x 128 x 128
slices, nz = 100, ngf = ndf = 128, weights N(0, 0.02), BatchNorm weights N(1, 0.02)) and
50_reconstruction/dcgan.py:39-153 (batch 4, Adam(2e-4, betas=(0.5, 0.999)), BCEWithLogitsLoss;
per iteration: D on the real batch, D on G(z).detach(), one D step; then D on G(z) with real
labels, one G step).  Slices: 50_reconstruction/brats_data.py:60-80 (channel 0, 128x128x64 crop,
one axial slice from [25, 35)).

MI355X form: the slices are filtered on the device by the texbias k-space ops (``FusedChain`` on
[B, 1, 1, 128, 128]), the networks run under bf16 autocast (fp32 master weights, fp32 loss),
and data parallelism is one process per GPU with both networks in DDP over RCCL:
D's two backward passes accumulate locally (``no_sync`` on the first) and reduce once, and the
generator step's backward through D skips D's all-reduce (those gradients are discarded, as in
the reference, by the next ``zero_grad``).  No host sync per step (the reference's ``.item()``
logging is left to the caller).
"""
from __future__ import annotations

import contextlib
from typing import Optional, Tuple

import torch
import torch.nn as nn


def weights_init(m: nn.Module) -> None:
    """networks.py:8-14: conv weights N(0, 0.02); BatchNorm weight N(1, 0.02), bias 0."""
    name = type(m).__name__
    if "Conv" in name:
        nn.init.normal_(m.weight.data, 0.0, 0.02)
    elif "BatchNorm" in name:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0)


class Generator(nn.Module):
    """z [B, nz, 1, 1] -> image [B, nc, 128, 128] in (-1, 1): a 4x4 transposed conv to ngf*16
    channels, then five stride-2 transposed convs halving the channels (the last to nc) with
    BatchNorm + ReLU between and Tanh at the end (networks.py:18-58)."""

    def __init__(self, nz: int = 100, ngf: int = 128, nc: int = 1):
        super().__init__()
        widths = [ngf * 16, ngf * 8, ngf * 4, ngf * 2, ngf]
        layers = [nn.ConvTranspose2d(nz, widths[0], 4, 1, 0, bias=False), nn.BatchNorm2d(widths[0]), nn.ReLU(True)]
        for cin, cout in zip(widths[:-1], widths[1:]):
            layers += [nn.ConvTranspose2d(cin, cout, 4, 2, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(True)]
        layers += [nn.ConvTranspose2d(widths[-1], nc, 4, 2, 1, bias=False), nn.Tanh()]
        self.main = nn.Sequential(*layers)

    def forward(self, z):
        return self.main(z)


class Discriminator(nn.Module):
    """image [B, nc, 128, 128] -> logit [B, 1, 1, 1]: five stride-2 convs doubling the channels
    from ndf (BatchNorm after all but the first, LeakyReLU(0.2) after each), then a 4x4 conv to one
    logit -- no sigmoid, the loss is BCEWithLogits (networks.py:63-95)."""

    def __init__(self, nc: int = 1, ndf: int = 128):
        super().__init__()
        widths = [ndf, ndf * 2, ndf * 4, ndf * 8, ndf * 16]
        layers = [nn.Conv2d(nc, widths[0], 4, 2, 1, bias=False), nn.LeakyReLU(0.2, inplace=True)]
        for cin, cout in zip(widths[:-1], widths[1:]):
            layers += [nn.Conv2d(cin, cout, 4, 2, 1, bias=False), nn.BatchNorm2d(cout), nn.LeakyReLU(0.2, inplace=True)]
        layers += [nn.Conv2d(widths[-1], 1, 4, 1, 0, bias=False)]
        self.main = nn.Sequential(*layers)

    def forward(self, x):
        return self.main(x)


class DCGANStep:
    """One reference iteration (dcgan.py:86-130) per call: returns (errD, errG, D(x), D(G(z)) before
    and after the D step) as device tensors."""

    def __init__(self, device: torch.device, nz: int = 100, ngf: int = 128, ndf: int = 128, nc: int = 1,
                 lr: float = 2e-4, beta1: float = 0.5, distributed: bool = False, bf16: bool = True,
                 channels_last: bool = False):
        self.device, self.nz, self.bf16, self.channels_last = device, nz, bf16, channels_last
        G, D = Generator(nz, ngf, nc).to(device), Discriminator(nc, ndf).to(device)
        G.apply(weights_init)
        D.apply(weights_init)
        if channels_last:  # NHWC activations and weights (MIOpen's preferred layout for bf16)
            G, D = G.to(memory_format=torch.channels_last), D.to(memory_format=torch.channels_last)
        self.G_module, self.D_module = G, D
        if distributed:
            kw = dict(broadcast_buffers=False)  # BatchNorm running stats stay per rank (training uses batch stats)
            if device.type == "cuda":
                kw["device_ids"] = [device.index]
            G = nn.parallel.DistributedDataParallel(G, **kw)
            D = nn.parallel.DistributedDataParallel(D, **kw)
        self.G, self.D = G, D
        self.distributed = distributed
        self.crit = nn.BCEWithLogitsLoss()
        kw = dict(lr=lr, betas=(beta1, 0.999))
        if device.type == "cuda":
            kw["fused"] = True
        self.optD = torch.optim.Adam(D.parameters(), **kw)
        self.optG = torch.optim.Adam(G.parameters(), **kw)

    def _ac(self):
        if self.bf16 and self.device.type == "cuda":
            return torch.autocast("cuda", dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def _no_sync(self, m):
        return m.no_sync() if self.distributed else contextlib.nullcontext()

    def __call__(self, real: torch.Tensor, noise: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, ...]:
        b = real.size(0)
        if self.channels_last:
            real = real.contiguous(memory_format=torch.channels_last)
        ones = torch.ones((b,), dtype=torch.float32, device=real.device)
        zeros = torch.zeros((b,), dtype=torch.float32, device=real.device)
        if noise is None:
            noise = torch.randn(b, self.nz, 1, 1, device=real.device)
        # (1) D: maximise log D(x) + log(1 - D(G(z)))
        self.optD.zero_grad(set_to_none=True)
        with self._no_sync(self.D):
            with self._ac():
                out_real = self.D(real).view(-1)
            err_real = self.crit(out_real.float(), ones)
            err_real.backward()
        with self._ac():
            fake = self.G(noise)
            out_fake = self.D(fake.detach()).view(-1)
        err_fake = self.crit(out_fake.float(), zeros)
        err_fake.backward()  # D's gradients (real + fake) reduce here
        self.optD.step()
        # (2) G: maximise log D(G(z)) with the updated D
        self.optG.zero_grad(set_to_none=True)
        with self._no_sync(self.D):
            with self._ac():
                out_g = self.D(fake).view(-1)
            err_g = self.crit(out_g.float(), ones)
            err_g.backward()
        self.optG.step()
        return (err_real + err_fake).detach(), err_g.detach(), out_real.detach().float().mean(), \
            out_fake.detach().float().mean(), out_g.detach().float().mean()


def _conv_flops(net: nn.Module, x_shape) -> int:
    """Forward multiply-add flops (2 per MAC) of the conv / transposed-conv layers of ``net`` on
    one sample of ``x_shape`` (C, H, W)."""
    total, shape = 0, tuple(x_shape)
    for m in net.main:
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            k = m.kernel_size[0] * m.kernel_size[1]
            cin, cout = m.in_channels, m.out_channels
            h, w = shape[1:]
            s, p = m.stride[0], m.padding[0]
            if isinstance(m, nn.Conv2d):
                ho, wo = (h + 2 * p - m.kernel_size[0]) // s + 1, (w + 2 * p - m.kernel_size[1]) // s + 1
                total += 2 * cin * cout * k * ho * wo
            else:
                ho, wo = (h - 1) * s - 2 * p + m.kernel_size[0], (w - 1) * s - 2 * p + m.kernel_size[1]
                total += 2 * cin * cout * k * h * w
            shape = (cout, ho, wo)
    return total


def step_flops(nz: int = 100, ngf: int = 128, ndf: int = 128, nc: int = 1) -> int:
    """Analytic flops of one DCGANStep per sample: G forward + backward (x3), D forward + backward
    three times (real, fake.detach(), fake; x3 each) -- backward counted as twice the forward."""
    g = _conv_flops(Generator(nz, ngf, nc).to("meta"), (nz, 1, 1))
    d = _conv_flops(Discriminator(nc, ndf).to("meta"), (nc, 128, 128))
    return 3 * g + 9 * d
