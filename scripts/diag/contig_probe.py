#!/usr/bin/env python3
"""Where the train step's large copies and adds come from (measurement tool): torch.profiler with Python
stacks over one U-Net step at 2 x 4 x 96 x 96 x 64; prints every aten copy_ / add / add_ / clone on a
16- or 32-channel activation with the innermost repo frames of its Python stack."""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from texbias.train import TrainStep, reference_model  # noqa: E402

dev = torch.device("cuda", 0)
step = TrainStep(reference_model(4, 3), dev)
x = torch.randn((2, 4, 96, 96, 64), device=dev)
lab = (torch.rand((2, 3, 96, 96, 64), device=dev) > 0.85).float()
for _ in range(2):
    step(x, lab)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    step(x, lab)
    torch.cuda.synchronize()
for e in prof.events():
    if e.name not in ("aten::copy_", "aten::add", "aten::add_", "aten::clone", "aten::fill_", "aten::zero_"):
        continue
    shp = str(e.input_shapes)
    if "48, 48, 32" not in shp and "24, 24, 16" not in shp:
        continue
    st = [f for f in (e.stack or []) if "profiler" not in f][:8]
    par, chain = e.cpu_parent, []
    while par is not None and len(chain) < 6:
        chain.append(par.name)
        par = par.cpu_parent
    print(f"{e.name:14s} {e.self_device_time_total:8.1f} {shp[:90]}  <  {' < '.join(chain)[:150]}")
    for f in st:
        print("      ", f[-120:])
