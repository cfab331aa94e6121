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
__version__ = "0.1.0"
