#!/usr/bin/env python3
"""Which torch ops launch the train step's kernels: torch.profiler over one bench-shaped U-Net step
(2 x 4 x 240 x 240 x 160, DiceLoss, Adam), device time per op (self), top entries."""
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
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_device_time_total", row_limit=45,
                                                          max_name_column_width=60, max_shapes_column_width=80))
