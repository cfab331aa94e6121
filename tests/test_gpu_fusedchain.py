"""GPU parity of ``FusedChain`` exactly as bench.py runs it: D padded 155 -> 160 (pad=5), the
k-space pass writing the padded U-Net input, salt-and-pepper on the strided padded view reusing
the pass-C min/max.  Checked against the reference's golden chain (…_3modalities.py:171-174:
disk -> plane wave -> wrap -> S&P) and against the numpy oracle per sample.

Tolerances: max|y - y_ref| / max|y_ref| <= 1e-5; S&P class map bit-exact given u; S&P values
bit-exact given the filtered volume; padding exactly zero; identity samples bit-identical.
"""
import numpy as np
import pytest
import torch

from _golden import load_cases, relerr
from oracle import filters_oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-5
PAD = 5


@pytest.fixture(scope="module")
def F(gpu):
    import filters_and_operators
    return filters_and_operators


@pytest.fixture(scope="module")
def FC(gpu):
    from texbias.pipeline import FusedChain
    return FusedChain


def golden_transforms(F, meta, with_sap=True):
    """The golden chain's transforms, seeded exactly as tests/golden/make_golden.py seeded the reference's."""
    seed = meta["seed"]
    disk = F.RandFourierDiskMaskd(keys="image", r=meta["r"], inside_off=False, prob=1.0)
    planes = F.RandPlaneWaves_ellipsoid("image", *meta["abc"], intensity_value=meta["intensity"], prob=1.0)
    wrap = F.WrapArtifactd("image", meta["alpha"])
    sap = F.SaltAndPepper(meta["p"])
    for j, tr in enumerate((disk, planes, sap)):
        tr.set_random_state(seed + j)
    planes.ellipsoid.set_random_state(seed + 100)
    ts = [disk, planes, wrap] + ([sap] if with_sap else [])
    return ts, planes


@pytest.mark.parametrize("name,case", sorted(load_cases("chain").items()))
def test_fused_chain_padded_vs_golden(F, FC, name, case):
    meta, a = case
    x = torch.from_numpy(a["x"]).cuda()[None]
    D = x.shape[-1]
    phases = [a["phase"].tolist()]
    # k-space segment alone: output padded, pass-C min/max == min/max of the unpadded view
    ts, planes = golden_transforms(F, meta, with_sap=False)
    y3 = FC(ts)(x, pad=PAD, phases=phases)
    assert tuple(planes.idx) == tuple(meta["idx"])          # same ellipsoid draw as the reference
    assert y3.shape == x.shape[:-1] + (D + PAD,)
    assert torch.all(y3[..., D:] == 0)
    assert relerr(y3[0, ..., :D].cpu().numpy(), a["y3"]) < TOL
    # the full chain, S&P with the reference's u on the strided padded view
    ts, planes = golden_transforms(F, meta)
    chain = FC(ts)
    cls = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    y = chain(x, pad=PAD, phases=phases, u=torch.from_numpy(a["u"]).cuda()[None], cls=cls)
    assert torch.all(y[..., D:] == 0)
    v3 = y3[..., :D].reshape(-1)
    np.testing.assert_array_equal(chain.last_minmax[0], [v3.min().item(), v3.max().item()])
    refz, refc = O.salt_and_pepper(y3[0, ..., :D].cpu().numpy(), meta["p"], a["u"])
    np.testing.assert_array_equal(cls[0].cpu().numpy(), refc)
    np.testing.assert_array_equal(y[0, ..., :D].cpu().numpy(), refz)
    assert relerr(y[0, ..., :D].cpu().numpy(), a["y"]) < TOL


def _draws(F, seeds, probs, abc, spatial, B):
    """Replay the per-sample Compose draws of (disk, planes, sap) on identically seeded twins."""
    disk = F.RandFourierDiskMaskd(keys="image", r=6.5, inside_off=False, prob=probs[0])
    planes = F.RandPlaneWaves_ellipsoid("image", *abc, intensity_value=9.0, prob=probs[1])
    sap = F.SaltAndPepper(0.1, prob=probs[2])
    for tr, s in zip((disk, planes, sap), seeds):
        tr.set_random_state(s)
    planes.ellipsoid.set_random_state(seeds[3])
    out = []
    for _ in range(B):
        disk.randomize()
        planes.randomize(None)
        idx = planes.ellipsoid.sample_ellipsoid(spatial) if planes._do_transform else None
        sap.randomize(None)
        out.append((disk._do_transform, idx, sap._do_transform))
    return out


def _transforms(F, seeds, probs, abc, order):
    disk = F.RandFourierDiskMaskd(keys="image", r=6.5, inside_off=False, prob=probs[0])
    planes = F.RandPlaneWaves_ellipsoid("image", *abc, intensity_value=9.0, prob=probs[1])
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.1, prob=probs[2])
    for tr, s in zip((disk, planes, sap), seeds):
        tr.set_random_state(s)
    planes.ellipsoid.set_random_state(seeds[3])
    by = {"disk": disk, "planes": planes, "wrap": wrap, "sap": sap}
    return [by[k] for k in order]


@pytest.mark.parametrize("order,probs,wrap", [
    (("disk", "planes", "sap"), (0.5, 0.5, 0.5), False),   # mixed batch, some samples untouched
    (("sap", "disk", "planes", "wrap"), (0.6, 1.0, 1.0), True),   # salt-and-pepper first
])
def test_fused_chain_mixed_batch_vs_oracle(F, FC, order, probs, wrap):
    B, C, spatial = 6, 4, (32, 30, 16)
    abc = (10.0, 9.0, 5.0)
    seeds = (101, 102, 103, 104)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((B, C) + spatial).astype(np.float32)
    u = rng.random((B, C) + spatial, dtype=np.float32)
    phases = rng.uniform(-np.pi, np.pi, (B, C)).astype(np.float32)
    draws = _draws(F, seeds, probs, abc, spatial, B)
    chain = FC(_transforms(F, seeds, probs, abc, order))
    xd = torch.from_numpy(x).cuda()
    cls = torch.empty(xd.shape, dtype=torch.int8, device="cuda")
    y = chain(xd, pad=PAD, phases=phases.tolist(), u=torch.from_numpy(u).cuda(), cls=cls)
    assert torch.all(y[..., spatial[-1]:] == 0)
    yh, ch = y[..., : spatial[-1]].cpu().numpy(), cls.cpu().numpy()
    for b, (do_disk, idx, do_sap) in enumerate(draws):
        ref = x[b]
        if order[0] == "sap" and do_sap:
            ref, _ = O.salt_and_pepper(ref, 0.1, u[b])
        if do_disk:
            ref = O.fourier_disk(ref, 6.5)
        if idx is not None:
            ref = O.plane_waves(ref, idx, 9.0, phase=phases[b])
        if wrap:
            ref = O.wrap_artifact(ref, 0.5)
        if order[-1] == "sap" and do_sap:
            # the class map depends on u only; the values on the filtered volume
            z, c = O.salt_and_pepper(ref, 0.1, u[b])
            np.testing.assert_array_equal(ch[b], c)
            ref = z
        if not (do_disk or idx is not None or wrap):
            if not do_sap:      # drew nothing at all: untouched, bit for bit
                np.testing.assert_array_equal(yh[b], x[b])
        assert relerr(yh[b], ref) < TOL, f"sample {b} draws {(do_disk, idx, do_sap)}"
    # the batch really was mixed
    assert len({(d, i is not None, s) for d, i, s in draws}) > 1


def test_fused_chain_c3_full_size(F, FC, heartbeat):
    """bench.py's configuration at full C3 size (2 x 4 x 240 x 240 x 155, pad 5): every (sample,
    channel) pair vs the oracle (one oracle pass per sample) with the golden phase hook, the S&P class
    map from the explicit u, the pass-C min/max of each sample."""
    torch.manual_seed(3)
    B, C, spatial = 2, 4, (240, 240, 155)
    x = torch.randn((B, C) + spatial, device="cuda")
    disk = F.RandFourierDiskMaskd(keys="image", r=12.5, inside_off=False, prob=1.0)
    planes = F.RandPlaneWaves_ellipsoid("image", 55.0, 55.0, 30.0, intensity_value=15.0, prob=1.0)
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.05)
    for j, t in enumerate((disk, planes, sap)):
        t.set_random_state(j)
    planes.ellipsoid.set_random_state(7)
    phases = [[0.1 * (b * C + c) for c in range(C)] for b in range(B)]
    u = torch.rand((B, C) + spatial, device="cuda")
    cls = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    chain = FC([disk, planes, wrap, sap])
    plans, idxs = [], []
    for b in range(B):   # the same draws as one plan(B) call, each sample's ellipsoid point recorded
        plans += chain.plan(1, spatial, [phases[b]])
        idxs.append(tuple(planes.idx))
    assert idxs[0] != idxs[1]
    y = chain(x, pad=PAD, plans=plans, u=u, cls=cls)
    assert y.shape == (B, C, 240, 240, 160) and torch.all(y[..., 155:] == 0)
    yh, ch, uh = y[..., :155].cpu().numpy(), cls.cpu().numpy(), u.cpu().numpy()
    for b in range(B):
        ref3 = O.wrap_artifact(O.plane_waves(O.fourier_disk(x[b].cpu().numpy(), 12.5), idxs[b], 15.0,
                                             phase=np.float32(phases[b])), 0.5)
        mn, mx = chain.last_minmax[b]
        np.testing.assert_allclose([mn, mx], [ref3.min(), ref3.max()], rtol=0, atol=1e-5 * np.abs(ref3).max())
        for c in range(C):
            z, cref = O.salt_and_pepper(ref3[c][None], 0.05, uh[b, c][None])
            np.testing.assert_array_equal(ch[b, c], cref[0], err_msg=f"class map ({b}, {c})")
            # S&P values come from the whole sample's min/max (all channels), not the channel's
            zc = ref3[c].copy()
            zc[cref[0] == 1] = np.float32(ref3.min()) / 2
            zc[cref[0] == 2] = np.float32(ref3.max()) / 2
            assert relerr(yh[b, c], zc) < TOL, (b, c)
