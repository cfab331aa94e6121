"""texbias -- MI355X-native k-space texture filters + 3-D U-Net training step.

Layering:
  _abi / kprog       C-ABI structs and host-side op programs (no device needed)
  _lib / runtime     libtexbias.so loader, plans, workspaces, batched launches (HIP only)
  shell              plane-wave ellipsoid shell candidates
  transform_base     MONAI-0.5 transform protocol (MONAI's own classes when installed)
  pipeline           batched device-side augmentation stage (fused chain) for training
  unet / losses      MONAI-equivalent 3-D residual U-Net and DiceLoss (PyTorch-ROCm)
  train              train step, DDP over RCCL
"""
import os as _os

__version__ = "0.1.0"

# MIOpen's naive direct-convolution solvers are reference kernels: on this U-Net's full-volume layers
# one trial of them takes up to 9 s, and MIOpen's Find (cudnn.benchmark) times every applicable
# solver on first use -- ~120 s of the first train step in every process (round-2 profile).  The
# implicit-GEMM / GEMM solvers cover every layer, so the naive ones are left out of the search.
# Set before MIOpen reads them (first convolution); an explicit setting wins.
for _d in ("FWD", "BWD", "WRW"):
    _os.environ.setdefault(f"MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_{_d}", "0")
