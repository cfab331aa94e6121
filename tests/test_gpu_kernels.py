"""GPU parity of the HIP kernels (through the C ABI via texbias.runtime) against the
reference's golden fixtures and the numpy oracle.

Tolerances: filtered outputs  max|y - y_ref| / max|y_ref| <= 1e-5 (north_star);
salt-and-pepper class maps and mask counts bit-exact.
"""
import numpy as np
import pytest
import torch

from _golden import load_cases, relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def rt(gpu):
    from texbias import runtime
    return runtime


def run(rt, x, n_dims, prog, pad=0):
    lead = x.shape[:-n_dims]
    chans = int(np.prod(lead))
    xb = torch.from_numpy(np.ascontiguousarray(x)).cuda().reshape((1, chans) + x.shape[-n_dims:])
    mm = torch.empty((1, 2), dtype=torch.int32, device="cuda")
    y = rt.kspace_filter(xb, n_dims, [prog], chans, pad=pad, minmax=mm)
    torch.cuda.synchronize()
    return y.cpu().numpy().reshape(x.shape[:-1] + (x.shape[-1] + pad,)), rt.keys_to_float(mm)[0]


@pytest.mark.parametrize("shape", [(2, 16, 16, 16), (1, 240, 240, 155), (4, 128, 128, 64), (1, 31, 17, 37 - 7),
                                   (3, 1, 1, 64), (2, 1, 256, 256), (1, 60, 1, 15)])
def test_identity_roundtrip(rt, shape):
    """Full-spectrum FFT round trip (wrap with alpha = 1 multiplies every coefficient by 1)."""
    x = np.random.default_rng(7).standard_normal(shape).astype(np.float32)
    try:
        rt.set_wrap_plans(False)  # this test is about the full-spectrum passes
        y, mm = run(rt, x, 3, [K.wrap_op(1.0)])
    finally:
        rt.set_wrap_plans(True)
    assert relerr(y, x) < 2e-6
    assert mm[0] == x.min() or abs(mm[0] - x.min()) < 1e-5
    assert abs(mm[1] - x.max()) < 1e-5


@pytest.mark.parametrize("name,case", sorted(load_cases("disk").items()))
def test_disk(rt, name, case):
    meta, a = case
    r = meta["r"]
    r = float("inf") if r == "inf" else (meta["r_used"] if isinstance(r, list) else r)
    y, _ = run(rt, a["x"], 3, [K.disk_op(r, meta["inside_off"])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("wrap").items()))
def test_wrap(rt, name, case):
    meta, a = case
    y, _ = run(rt, a["x"], 3, [K.wrap_op(meta["alpha"])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted((k, v) for k, v in load_cases("gibbs").items() if k != "gibbs_known"))
def test_gibbs(rt, name, case):
    meta, a = case
    x = a["x"]
    y, _ = run(rt, x, x.ndim - 1, [K.gibbs_op(meta["alpha"], x.shape[1:])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("planes").items()))
def test_planes(rt, name, case):
    meta, a = case
    geo = K.geometry(a["x"].shape[1:])
    y, _ = run(rt, a["x"], 3, [K.spike_op(meta["idx"], geo, meta["intensity"])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted((k, v) for k, v in load_cases("glayer").items() if k != "glayer_known"))
def test_gibbs_layer_device_alpha(rt, name, case):
    meta, a = case
    x = torch.from_numpy(a["x"]).cuda()
    alpha = torch.tensor([meta["alpha"]], dtype=torch.float32, device="cuda")
    progs = [[K.layer_op(0.0, x.shape[1:], alpha_ptr=alpha.data_ptr())] for _ in range(x.shape[0])]
    y = rt.kspace_filter(x[:, None], 4, progs, 1)
    assert relerr(y[:, 0].cpu().numpy(), a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("chain").items()))
def test_chain_fused_with_sap(rt, name, case):
    meta, a = case
    x = a["x"]
    geo = K.geometry(x.shape[1:])
    prog = [K.disk_op(meta["r"], False)]
    prog += [K.spike_op(meta["idx"], geo, meta["intensity"], phase=float(p), chan=c) for c, p in enumerate(a["phase"])]
    for op in prog[2:]:
        op.reserved = 1
    prog += [K.wrap_op(meta["alpha"])]
    xb = torch.from_numpy(x).cuda()[None]
    mm = torch.empty((1, 2), dtype=torch.int32, device="cuda")
    y3 = rt.kspace_filter(xb, 3, [prog], x.shape[0], minmax=mm)
    assert relerr(y3[0].cpu().numpy(), a["y3"]) < TOL
    # salt & pepper on the fused output with the reference's own u field
    u = torch.from_numpy(a["u"]).cuda()[None]
    cls = torch.empty(xb.shape, dtype=torch.int8, device="cuda")
    p = meta["p"]
    z = rt.salt_and_pepper(y3, 4, [(np.float32(p / 2), np.float32(p))], mm, u=u, cls=cls)
    zh = z[0].cpu().numpy()
    refz, refc = O.salt_and_pepper(y3[0].cpu().numpy(), p, a["u"])
    np.testing.assert_array_equal(cls[0].cpu().numpy(), refc)
    np.testing.assert_array_equal(zh, refz)
    assert relerr(zh, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("sap").items()))
def test_sap_golden(rt, name, case):
    meta, a = case
    x = torch.from_numpy(a["x"]).cuda()[None]
    mm = rt.minmax_keys(x, 4)
    p = meta["p_used"]
    cls = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    y = rt.salt_and_pepper(x, 4, [(np.float32(p / 2), np.float32(p))], mm, u=torch.from_numpy(a["u"]).cuda()[None],
                           cls=cls)
    np.testing.assert_array_equal(cls[0].cpu().numpy(), a["cls"])
    np.testing.assert_array_equal(y[0].cpu().numpy(), a["y"])


def test_sap_philox_sparse_inplace(rt):
    """Sparse in-place scatter == dense out-of-place with the same Philox stream; rate ~ p."""
    x = torch.randn((2, 4, 64, 60, 31), device="cuda")
    mm = rt.minmax_keys(x, 4)
    thr = [(np.float32(0.05), np.float32(0.1))] * 2
    cls = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    dense = rt.salt_and_pepper(x, 4, thr, mm, cls=cls, seed=1234, offset=7)
    inplace = x.clone()
    rt.salt_and_pepper(inplace, 4, thr, mm, out=inplace, seed=1234, offset=7)
    torch.testing.assert_close(inplace, dense, rtol=0, atol=0)
    frac1 = (cls == 1).float().mean().item()
    frac2 = (cls == 2).float().mean().item()
    assert abs(frac1 - 0.05) < 0.003 and abs(frac2 - 0.05) < 0.003
    mmf = rt.keys_to_float(mm)
    xs = x.reshape(2, -1)
    assert np.allclose(mmf[:, 0], xs.min(1).values.cpu().numpy()) and np.allclose(mmf[:, 1], xs.max(1).values.cpu().numpy())


def test_disk_mask_counts(rt):
    m = rt.disk_mask_tensor((1, 64, 64, 64), 12.5, 3, False, torch.device("cuda"))
    assert int(m.sum().item()) == 8217
    m2 = rt.disk_mask_tensor((1, 256, 256), 40, 2, False, torch.device("cuda"))
    assert int(m2.sum().item()) == 5013
    meta, a = load_cases("diskmask")["diskmask_counts"]
    m3 = rt.disk_mask_tensor((2, 20, 17), 6.5, 2, True, torch.device("cuda"))
    np.testing.assert_array_equal(m3.cpu().numpy(), a["mask2d_20x17"])


def test_full_size_c3_properties(rt):
    """BASELINE config 3 geometry 2 x 4 x 240 x 240 x 155: parity of one channel vs the oracle,
    linearity of the fused filter, zero D-padding to 160, identity at r = inf / alpha = 1."""
    torch.manual_seed(0)
    x = torch.randn((2, 4, 240, 240, 155), device="cuda")
    geo = K.geometry((240, 240, 155))
    prog = [K.disk_op(12.5, False), K.spike_op((70, 137, 71), geo, 15.0, phase=0.3), K.wrap_op(0.5)]
    y = rt.kspace_filter(x, 3, [prog, prog], 4, pad=5)
    assert y.shape == (2, 4, 240, 240, 160)
    assert torch.all(y[..., 155:] == 0)
    x0 = x[1, 2].cpu().numpy()
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x0[None], 12.5), (70, 137, 71), 15.0, phase=[0.3]), 0.5)[0]
    assert relerr(y[1, 2, ..., :155].cpu().numpy(), ref) < TOL
    # linearity of the mask part
    progm = [K.disk_op(20.0, False), K.wrap_op(0.25)]
    a, b = 0.75, -1.5
    x2 = torch.randn_like(x)
    lhs = rt.kspace_filter(a * x + b * x2, 3, [progm] * 2, 4)
    rhs = a * rt.kspace_filter(x, 3, [progm] * 2, 4) + b * rt.kspace_filter(x2, 3, [progm] * 2, 4)
    assert (lhs - rhs).abs().max().item() / rhs.abs().max().item() < 2e-6
    ident = rt.kspace_filter(x, 3, [[K.disk_op(float("inf"), False), K.wrap_op(1.0)]] * 2, 4)
    assert (ident - x).abs().max().item() / x.abs().max().item() < 2e-6


def test_default_intensity_stats(rt):
    meta, a = load_cases("kspike")["kspike_3"]
    x = torch.from_numpy(a["x"]).cuda()[None]
    s = rt.logabs_sums(x, 3, [[]], x.shape[1]).cpu().numpy()
    n = np.prod(a["x"].shape[1:])
    dflt = s / n * 2.5
    np.testing.assert_allclose(dflt, O.kspace_default_intensity(a["x"]), rtol=2e-3)


@pytest.mark.parametrize("shape", [(2, 4, 240, 240, 155), (1, 4, 128, 128, 128)])
def test_compiled_slab_plan_matches_generic(rt, shape):
    """Passes A/C on the compile-time slab plans == the generic passes (to rounding) and == the
    oracle on one channel; D padding zeroed; per-sample min/max keys identical in value."""
    torch.manual_seed(5)
    x = torch.randn(shape, device="cuda")
    geo = K.geometry(shape[2:])
    idx = (9, 17, 23)
    prog = [K.disk_op(12.5, False), K.spike_op(idx, geo, 12.0, phase=0.4), K.wrap_op(0.5)]
    B = shape[0]
    mm_c = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    mm_g = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    try:
        rt.set_band_plans(False)   # this test is about the full-spectrum passes
        rt.set_compiled_plans(True)
        yc = rt.kspace_filter(x, 3, [prog] * B, shape[1], pad=5, minmax=mm_c)
        rt.set_compiled_plans(False)
        yg = rt.kspace_filter(x, 3, [prog] * B, shape[1], pad=5, minmax=mm_g)
    finally:
        rt.set_compiled_plans(True)
        rt.set_band_plans(True)
    torch.cuda.synchronize()
    assert torch.all(yc[..., shape[-1]:] == 0)
    assert (yc - yg).abs().max().item() / yg.abs().max().item() < 2e-6
    x0 = x[B - 1, 1].cpu().numpy()
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x0[None], 12.5), idx, 12.0, phase=[0.4]), 0.5)[0]
    assert relerr(yc[B - 1, 1, ..., :shape[-1]].cpu().numpy(), ref) < TOL
    yv = yc[..., :shape[-1]].reshape(B, -1)
    mmf = rt.keys_to_float(mm_c)
    np.testing.assert_array_equal(mmf[:, 0], yv.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(mmf[:, 1], yv.max(1).values.cpu().numpy())


@pytest.mark.parametrize("shape", [(2, 4, 240, 240, 155), (2, 3, 32, 30, 16)])
def test_chain_chunking_is_bit_identical(rt, shape):
    """Running passes A -> B -> C per chunk of channel-volumes (Infinity-Cache-sized, chunk edges
    inside a sample) gives the same bits and the same per-sample min/max as one chain over the
    batch; the 16-B paired pass-B kernel (full C3 shape) is part of both runs."""
    torch.manual_seed(11)
    x = torch.randn(shape, device="cuda")
    geo = K.geometry(shape[2:])
    B, C = shape[0], shape[1]
    progs = [[K.disk_op(12.5, False), K.spike_op((3, 5, 7), geo, 12.0, phase=0.3 + b), K.wrap_op(0.5)]
             for b in range(B)]
    outs = []
    try:
        rt.set_band_plans(False)   # chunking applies to the full-spectrum passes
        for n in (0, 1, 3):
            rt.set_chain_chunk(n)
            mm = torch.empty((B, 2), dtype=torch.int32, device="cuda")
            y = rt.kspace_filter(x, 3, progs, C, pad=5, minmax=mm)
            outs.append((y, mm))
    finally:
        rt.set_chain_chunk(-1)
        rt.set_band_plans(True)
    torch.cuda.synchronize()
    for y, mm in outs[1:]:
        assert torch.equal(y, outs[0][0])
        assert torch.equal(mm, outs[0][1])


@pytest.mark.parametrize("p", [0.05, 0.35, 1.0])
def test_sap_geometric_stream_statistics(rt, p):
    """The device stream walks geometric gaps between changed voxels: the changed set must be a
    Bernoulli(p) field -- rate p, flat over the position inside the per-thread segments, classes
    MIN / MAX with probability 1/2 each given a change (thresholds p/2, p)."""
    n_rows, ln = 4096, 512
    x = torch.zeros((2, n_rows, ln), device="cuda")
    x[:, 0, 0] = -4.0
    x[:, 0, 1] = 6.0
    mm = rt.minmax_keys(x, 2)
    cls = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    thr = [(np.float32(p / 2), np.float32(p))] * 2
    rt.salt_and_pepper(x, 2, thr, mm, cls=cls, seed=99, offset=3)
    c = cls.reshape(2, -1).cpu().numpy()
    n = c.shape[1]
    hit = c > 0
    rate = hit.mean()
    sd = np.sqrt(p * (1 - p) / hit.size) + 1e-12
    assert abs(rate - p) < 6 * sd + 1e-9
    if p < 1.0:
        pmin = (c == 1).sum() / max(hit.sum(), 1)
        assert abs(pmin - 0.5) < 6 * np.sqrt(0.25 / hit.sum())
        pos = np.arange(n) % 1024
        bins = np.array([hit[:, (pos >= 128 * k) & (pos < 128 * (k + 1))].mean() for k in range(8)])
        sdb = np.sqrt(p * (1 - p) / (hit.size / 8))
        assert np.all(np.abs(bins - p) < 6 * sdb)
    # in place writes only the changed voxels and agrees with the out-of-place result
    y = x.clone()
    rt.salt_and_pepper(y, 2, thr, mm, out=y, seed=99, offset=3)
    z = rt.salt_and_pepper(x, 2, thr, mm, seed=99, offset=3)
    torch.testing.assert_close(y, z, rtol=0, atol=0)
    mmf = rt.keys_to_float(mm)
    zc = z.cpu().numpy().reshape(2, -1)
    for b in range(2):
        np.testing.assert_array_equal(zc[b][c[b] == 1], np.float32(mmf[b, 0]) / 2)
        np.testing.assert_array_equal(zc[b][c[b] == 2], np.float32(mmf[b, 1]) / 2)
