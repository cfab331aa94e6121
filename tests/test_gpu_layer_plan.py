"""The in-model Gibbs layer at the drivers' crop shape, [B, 1, 128, 128, 64]
(10_scripts/300_instutional_distribution/350_stylized_layers/gibbs0p7_layer_domain_GD.py:252-269,
source_code/stylization_layers.py:79-116), on the compiled 128 x 64 slab plan (slab_ct.h) with the
device-resident alpha: equal to the run-time-planned generic passes (to rounding) and to the numpy
oracle per sample; the compiled kernels are the ones that ran.

Tolerances: vs the oracle max|y - y_ref| / max|y_ref| <= 1e-5 (north_star); compiled vs generic 2e-6.
"""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(gpu):
    import stylization_layers as SL
    from texbias import runtime as rt
    return SL, rt


@pytest.mark.parametrize("alpha", [0.7, 0.25])
def test_layer_compiled_128x64_plan(env, alpha):
    SL, rt = env
    torch.manual_seed(21)
    x = torch.randn((2, 1, 128, 128, 64), device="cuda")
    layer = SL.GibbsNoiseLayer(alpha).cuda()
    rt.set_pass_timing(True)
    y = layer(x)
    torch.cuda.synchronize()
    _, cnt, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    assert "ct" in names[0] and "ct" in names[2], names   # k_slab_fwd_ct16 / k_slab_inv_ct
    try:
        rt.set_compiled_plans(False)
        yg = layer(x)
    finally:
        rt.set_compiled_plans(True)
    torch.cuda.synchronize()
    assert (y - yg).abs().max().item() / yg.abs().max().item() < 2e-6
    for b in range(2):
        ref = O.gibbs_layer(x[b].cpu().numpy(), alpha)
        assert relerr(y[b].cpu().numpy(), ref) < 1e-5, b
