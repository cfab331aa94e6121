"""DCGAN (config 5) on the GPU: the networks' fp32 outputs match the reference's golden vectors
(same seed, MIOpen convolutions: max|d| <= 1e-4 of max|ref|), and the bf16 step fed by filtered
slices runs and stays finite."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_dcgan.npz")


def test_networks_on_gpu_match_reference_vectors(gpu):
    from texbias import dcgan
    g = np.load(GOLD, allow_pickle=False)
    torch.manual_seed(7)
    G = dcgan.Generator(nz=100, ngf=16, nc=1)
    D = dcgan.Discriminator(nc=1, ndf=16)
    G.apply(dcgan.weights_init)
    D.apply(dcgan.weights_init)
    G, D = G.cuda(), D.cuda()
    with torch.no_grad():
        go = G(torch.from_numpy(g["z"]).cuda()).cpu().numpy()
        do = D(torch.from_numpy(g["x"]).cuda()).cpu().numpy()
    assert np.abs(go - g["g_out"]).max() <= 1e-4 * np.abs(g["g_out"]).max()
    assert np.abs(do - g["d_out"]).max() <= 1e-4 * np.abs(g["d_out"]).max()


def test_bf16_step_on_filtered_slices(gpu):
    from texbias.dcgan import DCGANStep
    from texbias.pipeline import FusedChain, reference_c3_chain
    from texbias.synth import brats_like
    torch.manual_seed(0)
    _, tr = reference_c3_chain(0)
    chain = FusedChain([tr["disk"], tr["wrap"], tr["sap"]])
    x = brats_like(8, 1, (1, 128, 128), seed=1, device="cuda")
    step = DCGANStep(torch.device("cuda"), bf16=True)
    for _ in range(3):
        y = chain(x)
        out = step(y.view(8, 1, 128, 128))
    torch.cuda.synchronize()
    assert all(torch.isfinite(t).item() for t in out)
