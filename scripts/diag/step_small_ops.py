#!/usr/bin/env python3
"""The train step's non-texbias device work by originating torch op (measurement tool): torch.profiler
over one bench-shaped step (2 x 4 x 240 x 240 x 160), every aten op with self device time, with its
input shapes and the autograd node it ran under."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from texbias.train import TrainStep, reference_model  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
step = TrainStep(reference_model(4, 3), dev)
x = torch.randn((2, 4, 240, 240, 160), device=dev)
lab = (torch.rand((2, 3, 240, 240, 160), device=dev) > 0.85).float()
for _ in range(3):
    step(x, lab)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step(x, lab)
    torch.cuda.synchronize()
rows = []
for e in prof.events():
    if not e.name.startswith("aten::") or e.self_device_time_total <= 0:
        continue
    par, chain = e.cpu_parent, []
    while par is not None and len(chain) < 4:
        chain.append(par.name)
        par = par.cpu_parent
    rows.append((e.self_device_time_total, e.name, str(e.input_shapes)[:110], " < ".join(chain)[:120]))
rows.sort(key=lambda r: -r[0])
tot = sum(r[0] for r in rows)
print(f"aten ops with device time: {len(rows)}, {tot:.1f} us total")
for r in rows[:70]:
    print(f"{r[0]:9.1f}  {r[1]:34s} {r[2]:110s} {r[3]}")
