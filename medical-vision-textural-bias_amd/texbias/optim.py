"""Adam on the texbias kernel (``tb_adam_f32``, csrc/optim.hip): the reference's optimizer,
``torch.optim.Adam(model.parameters(), 1e-4, weight_decay=1e-5, amsgrad=True)``
(10_scripts/20_Gibbs_filters/stylized_gibbs12p5.py:203-205), as one multi-tensor launch of ~1200
4096-element chunks instead of ATen's fused Adam (three launches of 40 / 84 / 3 blocks at the U-Net's
~4.8 M parameters: 112 us per step).

``Adam`` is a ``torch.optim.Adam`` (same constructor, param groups, state names and state_dict layout as
torch's capturable Adam: a float32 device ``step`` per parameter, ``exp_avg``, ``exp_avg_sq``,
``max_exp_avg_sq``); only ``step`` differs, and only for float32 HIP parameters with dense contiguous
gradients, float learning rates and no ``maximize`` / ``differentiable`` -- anything else runs torch's own
update.  The step counters are incremented on the device before the launch, so the update can be captured
in a HIP graph.  ``ENABLED = False`` (env ``TEXBIAS_ADAM=0``) makes ``TrainStep`` use ATen's fused Adam."""
from __future__ import annotations

import ctypes
import os

import torch

from ._lib import check, lib

ENABLED = os.environ.get("TEXBIAS_ADAM", "1") != "0"


def _eligible(p: torch.Tensor, group: dict) -> bool:
    g = p.grad
    return (p.is_cuda and p.dtype == torch.float32 and g.dtype == torch.float32 and not g.is_sparse and
            p.is_contiguous() and g.is_contiguous() and g.device == p.device)


class Adam(torch.optim.Adam):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         capturable=True)

    def _native_ok(self, group: dict) -> bool:
        return not (group.get("maximize") or group.get("differentiable") or torch.is_tensor(group["lr"]) or
                    group.get("decoupled_weight_decay", False))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if not (self._native_ok(group) and all(_eligible(p, group) for p in params)):
                self._torch_step(group)
                continue
            ams = bool(group["amsgrad"])
            cols = ([], [], [], [], [], [], [])
            steps = []
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    if ams:
                        st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                step = st["step"]
                if not (step.is_cuda and step.dtype == torch.float32):  # a state_dict from a host-step Adam
                    step = st["step"] = step.to(device=p.device, dtype=torch.float32)
                steps.append(step)
                cols[0].append(p.data_ptr())
                cols[1].append(p.grad.data_ptr())
                cols[2].append(st["exp_avg"].data_ptr())
                cols[3].append(st["exp_avg_sq"].data_ptr())
                cols[4].append(st["max_exp_avg_sq"].data_ptr() if ams else 0)
                cols[5].append(step.data_ptr())
                cols[6].append(p.numel())
            torch._foreach_add_(steps, 1.0)
            n = len(params)
            arr = [(ctypes.c_void_p * n)(*c) for c in cols[:6]]
            numel = (ctypes.c_int64 * n)(*cols[6])
            b1, b2 = group["betas"]
            dev = params[0].device
            with torch.cuda.device(dev):
                check(lib().tb_adam_f32(n, arr[0], arr[1], arr[2], arr[3], arr[4] if ams else None, arr[5], numel,
                                        float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                        float(group["weight_decay"]), 1 if ams else 0,
                                        torch.cuda.current_stream(dev).cuda_stream), "tb_adam_f32")
        return loss

    def _torch_step(self, group: dict) -> None:
        """torch.optim.Adam's own update of one parameter group (the other groups are left alone)."""
        saved = self.param_groups
        try:
            self.param_groups = [group]
            super().step()
        finally:
            self.param_groups = saved
