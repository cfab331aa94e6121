"""FusedChain over the driver chains round 2 could not batch, and spike programs past one launch:

* RandKSpaceSpikeNoised("image", 0.1, 1.0, intensity_ranges=...) -- the augmentation drivers'
  call (10_scripts/300_instutional_distribution/30_augmentation/baseline_domain_augment_spikes10-11.py:120),
  channel-wise, batched: each sample vs the oracle with the draws replayed on a twin transform;
* SelectChanneld before the filters (the one-channel drivers) and MultimodalSlicesd after them
  (127_.../..._3modalities.py:94-109,175) through ``FusedChain.apply`` with labels;
* KSpaceSpikeNoise with 9 locations (more than TB_MAX_OPS = 6 in one call) and a 4-channel
  channel-wise draws after a wrap (9 ops): programs cut into exact passes (kprog.split_program).
Tolerance: max|y - y_ref| / max|y_ref| <= 1e-5 (north_star); labels exact."""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F(gpu):
    import filters_and_operators
    return filters_and_operators


def test_fused_rand_kspace_spiked_channel_wise(F):
    from texbias.pipeline import FusedChain
    B, C, sp = 4, 4, (24, 20, 16)
    x = torch.randn((B, C) + sp, device="cuda")
    t = F.RandKSpaceSpikeNoised("image", 1.0, 0.6, intensity_ranges={"image": (10.0, 11.0)})
    twin = F.RandKSpaceSpikeNoised("image", 1.0, 0.6, intensity_ranges={"image": (10.0, 11.0)})
    t.set_rand_state(3)
    twin.set_rand_state(3)
    y = FusedChain([t])(x)
    inner = twin.transforms["image"]
    drew = 0
    for b in range(B):
        twin.randomize(None)
        inner.sampled_locs, inner.sampled_k_intensity = [], []
        inner._randomize(torch.empty((C,) + sp), inner._make_sequence(torch.empty((C,) + sp)))
        xb = x[b].cpu().numpy()
        ref = O.kspace_spike(xb, tuple(inner.sampled_locs), tuple(inner.sampled_k_intensity)) \
            if inner.sampled_locs else xb
        drew += len(inner.sampled_locs)
        assert relerr(y[b].cpu().numpy(), ref) < 1e-5, b
    assert 0 < drew < B * C   # prob 0.6 per channel: a mix of spiked and untouched channels


def test_select_and_multimodal_slices(F):
    from texbias.pipeline import FusedChain
    B, C, sp = 3, 4, (24, 20, 16)
    x = torch.randn((B, C) + sp, device="cuda")
    lab = (torch.rand((B, 3) + sp, device="cuda") > 0.5).float()
    sel = F.SelectChanneld(["image"], 2)
    disk = F.RandFourierDiskMaskd("image", r=5.0, prob=1.0)
    out = FusedChain([sel, disk]).apply({"image": x, "label": lab})
    assert out["image"].shape == (B, 1) + sp and torch.equal(out["label"], lab)
    for b in range(B):
        ref = O.fourier_disk(x[b, 2:3].cpu().numpy(), 5.0)
        assert relerr(out["image"][b].cpu().numpy(), ref) < 1e-5
    # out= of the input's shape cannot take a one-channel result: an error, not a broadcast copy
    with pytest.raises(ValueError):
        FusedChain([sel, disk])(x, out=torch.empty_like(x))
    # 127_*: filters on all four channels, then one random modality and the label's channel 1
    wrap = F.WrapArtifactd("image", 0.5)
    mm = F.MultimodalSlicesd(keys=["image", "label"], img_chan_indices=[0, 1, 2, 3], label_idx=1, seed=4)
    twin = np.random.RandomState(4)
    out = FusedChain([disk, wrap, mm]).apply({"image": x, "label": lab})
    assert out["image"].shape == (B, 1) + sp and out["label"].shape == (B, 1) + sp
    for b in range(B):
        c = int(twin.choice([0, 1, 2, 3]))
        ref = O.wrap_artifact(O.fourier_disk(x[b].cpu().numpy(), 5.0), 0.5)[c:c + 1]
        assert relerr(out["image"][b].cpu().numpy(), ref) < 1e-5
        assert torch.equal(out["label"][b], lab[b, 1:2])


def test_long_spike_programs_split_exactly(F):
    torch.manual_seed(2)
    C, sp = 4, (24, 20, 16)
    x = torch.randn((C,) + sp)
    rng = np.random.default_rng(1)
    locs = tuple((int(rng.integers(0, C)),) + tuple(int(rng.integers(0, n)) for n in sp) for _ in range(9))
    vals = tuple(float(v) for v in rng.uniform(8.0, 11.0, 9))
    y = F.KSpaceSpikeNoise(locs, vals)(x)
    assert relerr(y.numpy(), O.kspace_spike(x.numpy(), locs, vals)) < 1e-5
    # wrap + two 4-channel channel-wise spike draws in one FusedChain run: 1 + 4 + 4 = 9 ops per
    # sample, cut inside the second draw's group (no low-pass: a spike's phase after a low-pass is
    # rounding noise)
    from texbias.pipeline import FusedChain
    wrap = F.WrapArtifactd("image", 0.5)
    s1 = F.RandKSpaceSpikeNoised("image", 1.0, 1.0, intensity_ranges={"image": (9.0, 10.0)})
    s2 = F.RandKSpaceSpikeNoised("image", 1.0, 1.0, intensity_ranges={"image": (10.0, 11.0)})
    s1.set_rand_state(5)
    s2.set_rand_state(6)
    chain = FusedChain([wrap, s1, s2])
    xb = torch.randn((2, C) + sp, device="cuda")
    plans = chain.plan(2, sp, channels=C)
    assert all(len(p[0][1]) == 9 for p in plans)
    y = chain(xb, plans=plans)
    for b in range(2):
        ops = plans[b][0][1]
        ref = O.wrap_artifact(xb[b].cpu().numpy(), 0.5)
        for grp in (ops[1:5], ops[5:9]):
            geo_locs = []
            for op in grp:
                k = tuple(int(v) for v in op.i)
                shifted = tuple((kk + n // 2) % n for kk, n in zip(k, sp))
                geo_locs.append((int(op.chan),) + shifted)
            ref = O.kspace_spike(ref, tuple(geo_locs), tuple(float(np.log(op.f[0])) for op in grp))
        assert relerr(y[b].cpu().numpy(), ref) < 1e-5, b
