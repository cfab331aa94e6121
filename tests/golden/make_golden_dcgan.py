#!/usr/bin/env python3
"""Golden vectors of the reference's DCGAN networks (50_reconstruction/networks.py:18-95).

TEST INFRASTRUCTURE.  Runs only in the build container: imports the reference's networks.py in
place (pure torch, no MONAI) and records, for a fixed torch seed, the outputs of Generator and
Discriminator (train mode, small widths ngf = ndf = 16 so the CPU test stays fast) on fixed
inputs, plus the parameter count of the full-size networks.  Only data is written.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dcgan.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, os.environ.get("TB_REFERENCE_RECON", "/root/reference/50_reconstruction"))
import networks  # noqa: E402

torch.set_num_threads(1)
out = {}
torch.manual_seed(7)
G = networks.Generator(nz=100, ngf=16, nc=1)
D = networks.Discriminator(nc=1, ndf=16)
G.apply(networks.weights_init)
D.apply(networks.weights_init)
z = torch.randn(2, 100, 1, 1)
x = torch.rand(2, 1, 128, 128) * 2 - 1
with torch.no_grad():
    out["g_out"] = G(z).numpy()
    out["d_out"] = D(x).numpy()
out["z"] = z.numpy()
out["x"] = x.numpy()
out["n_params_g_full"] = np.array(sum(p.numel() for p in networks.Generator().parameters()))
out["n_params_d_full"] = np.array(sum(p.numel() for p in networks.Discriminator().parameters()))
np.savez_compressed(os.path.join(HERE, "golden_dcgan.npz"), **out)
print({k: v.shape for k, v in out.items()})
