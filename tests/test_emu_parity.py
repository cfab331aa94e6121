"""CPU parity of the kernel bodies (host emulator of the gfx950 passes) against the oracle / golden.

The emulator compiles the SAME fft_core.h / sap_core.h the device kernels use, so these tests pin
the FFT schedule (mixed-radix in-place DIF/DIT, digit-reversed layout, pair-packed R2C/C2R), the
k-space op programs and the bit-exact mask geometry before any GPU time is spent.
"""
import numpy as np
import pytest

import _emu
from _golden import load_cases, relerr
from oracle import filters_oracle as O
from texbias import kprog as K

TOL = 1e-5


def run(x, n_dims, prog, **kw):
    """One sample: the trailing n_dims axes are transformed, the leading ones are channels."""
    lead = x.shape[:-n_dims]
    xb = x.reshape((1, int(np.prod(lead))) + x.shape[-n_dims:])
    y, mm = _emu.kspace_filter(xb, n_dims, [prog], **kw)
    return y.reshape(x.shape[:-1] + y.shape[-1:]), mm[0]


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 12, 15, 16, 17, 30, 31, 60, 64, 128, 155, 240, 256])
def test_identity_roundtrip(n):
    rng = np.random.default_rng(n)
    for shape in [(2, n, 3, 5), (1, 4, n, 6), (3, 2, 3, n)]:
        x = rng.standard_normal(shape).astype(np.float32)
        y, mm = run(x, 3, [])
        assert relerr(y, x) < 2e-6, shape
        np.testing.assert_allclose(mm, [x.min(), x.max()], rtol=1e-5, atol=1e-6)


def test_radices_supported():
    import ctypes
    L = _emu.lib()
    buf = (ctypes.c_int * 8)()
    assert L.tbemu_radices(155, buf) == 2 and list(buf[:2]) == [5, 31]
    assert L.tbemu_radices(240, buf) == 2 and list(buf[:2]) == [16, 15]
    assert L.tbemu_radices(37, buf) == -1   # prime > 31 rejected


@pytest.mark.parametrize("name,case", sorted(load_cases("disk").items()))
def test_disk(name, case):
    meta, a = case
    r = meta["r"]
    r = float("inf") if r == "inf" else (meta["r_used"] if isinstance(r, list) else r)
    x = a["x"]
    y, _ = run(x, 3, [K.disk_op(r, meta["inside_off"])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("wrap").items()))
def test_wrap(name, case):
    meta, a = case
    y, _ = run(a["x"], 3, [K.wrap_op(meta["alpha"])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted((k, v) for k, v in load_cases("gibbs").items() if k != "gibbs_known"))
def test_gibbs(name, case):
    meta, a = case
    x = a["x"]
    y, _ = run(x, x.ndim - 1, [K.gibbs_op(meta["alpha"], x.shape[1:])])
    assert relerr(y, a["y"]) < TOL


def test_gibbs_threshold_exact():
    for sp in [(128, 128, 64), (16, 16, 16), (40, 36), (31, 17), (240, 240, 155)]:
        for al in [0.0, 0.1, 0.3, 0.5, 0.77, 0.9, 1.0]:
            t = K.gibbs_threshold4(sp, al)
            m = O.gibbs_mask(sp, al)
            grids = np.meshgrid(*[(2 * np.arange(n) - (n - 1)) ** 2 for n in sp], indexing="ij")
            e = sum(grids)
            np.testing.assert_array_equal(e <= t, m)


@pytest.mark.parametrize("name,case", sorted(load_cases("planes").items()))
def test_planes(name, case):
    meta, a = case
    x = a["x"]
    geo = K.geometry(x.shape[1:])
    y, _ = run(x, 3, [K.spike_op(meta["idx"], geo, meta["intensity"])])
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("kspike").items()) + [("kspike_2d", load_cases("kspike")["kspike_2d"])])
def test_kspike(name, case):
    meta, a = case
    if "error" in meta:
        return
    x = a["x"]
    n = x.ndim - 1
    geo = K.geometry(x.shape[1:])
    loc, ki = meta["loc"], meta["k_intensity"]
    if ki is None:
        ki = meta["default_intensity"]
    if isinstance(loc[0], list):
        prog = [K.spike_op(l[1:], geo, v, chan=l[0]) for l, v in zip(loc, ki)]
        for op in prog[1:]:
            op.reserved = 1
    else:
        prog = [K.spike_op(loc, geo, ki)]
    y, _ = run(x, n, prog)
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("randkspike").items()))
def test_randkspike(name, case):
    meta, a = case
    x = a["x"]
    geo = K.geometry(x.shape[1:])
    prog = [K.spike_op(l[1:], geo, v, chan=l[0]) for l, v in zip(meta["locs"], meta["intens"])]
    for op in prog[1:]:
        op.reserved = 1
    y, _ = run(x, 3, prog)
    assert relerr(y, a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted((k, v) for k, v in load_cases("glayer").items() if k != "glayer_known"))
def test_gibbs_layer(name, case):
    meta, a = case
    x = a["x"]  # [B, 1, H, W, D] with n_dims = 4 (the singleton channel axis is transformed too)
    sp = x.shape[1:]
    progs = [[K.layer_op(meta["alpha"], sp)] for _ in range(x.shape[0])]
    y, _ = _emu.kspace_filter(x[:, None], 4, progs)
    assert relerr(y[:, 0], a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("slayer").items()))
def test_spike_layer(name, case):
    meta, a = case
    x = a["x"]
    sp = x.shape[1:]
    geo = K.geometry(sp)
    progs = [[K.spike_op(l[1:], geo, meta["intensity"])] for l in meta["locs"]]
    y, _ = _emu.kspace_filter(x[:, None], 4, progs)
    assert relerr(y[:, 0], a["y"]) < TOL


@pytest.mark.parametrize("name,case", sorted(load_cases("chain").items()))
def test_chain_fused(name, case):
    """disk -> planes -> wrap as ONE fused round trip equals the reference's three round trips."""
    meta, a = case
    x = a["x"]
    geo = K.geometry(x.shape[1:])
    prog = [K.disk_op(meta["r"], False)]
    prog += [K.spike_op(meta["idx"], geo, meta["intensity"], phase=float(ph), chan=c)
             for c, ph in enumerate(a["phase"])]
    prog += [K.wrap_op(meta["alpha"])]
    y3, mm = run(x, 3, prog)
    assert relerr(y3, a["y3"]) < TOL
    np.testing.assert_allclose(mm, [a["y3"].min(), a["y3"].max()], rtol=2e-5, atol=1e-5)


def test_pad_columns_zero():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 8, 6, 15)).astype(np.float32)
    y, _ = _emu.kspace_filter(x[None], 3, [[K.wrap_op(0.5)]], pad=5)
    ref = O.wrap_artifact(x, 0.5)
    assert relerr(y[0, ..., :15], ref) < TOL
    assert np.all(y[0, ..., 15:] == 0)


def test_tile_width_independent():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((3, 12, 10, 9)).astype(np.float32)
    prog = [K.gibbs_op(0.4, x.shape[1:]), K.wrap_op(0.3)]
    y1, _ = _emu.kspace_filter(x[None], 3, [prog], T=7)
    y2, _ = _emu.kspace_filter(x[None], 3, [prog], T=64)
    np.testing.assert_array_equal(y1, y2)


@pytest.mark.parametrize("shape", [(3, 5, 24, 35), (2, 4, 20, 28), (1, 3, 240, 155), (1, 2, 128, 128)])
def test_compiled_slab_plan(shape):
    """Passes A/C through the compile-time slab plan (slab_ct.h) == oracle, and == the generic path to
    rounding; pads zeroed, min/max epilogue exact."""
    rng = np.random.default_rng(sum(shape))
    x = rng.standard_normal(shape).astype(np.float32)
    geo = K.geometry(x.shape[1:])
    idx = (1, min(3, shape[2] - 1), min(7, shape[3] // 2))
    prog = [K.disk_op(0.3 * min(shape[1:]), False), K.spike_op(idx, geo, 6.0, phase=0.7), K.wrap_op(0.5)]
    yc, mmc = _emu.kspace_filter(x[None], 3, [prog], pad=3, ct=True)
    yg, _ = _emu.kspace_filter(x[None], 3, [prog], pad=3, ct=False)
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x, 0.3 * min(shape[1:])), idx, 6.0, phase=[0.7] * shape[0]), 0.5)
    assert relerr(yc[0, ..., :shape[-1]], ref) < TOL
    assert relerr(yc, yg) < 2e-6
    assert np.all(yc[0, ..., shape[-1]:] == 0)
    y0 = yc[0, ..., :shape[-1]]
    np.testing.assert_array_equal(mmc[0], [y0.min(), y0.max()])


def test_compiled_slab_identity():
    x = np.random.default_rng(3).standard_normal((2, 2, 6, 240, 155)).astype(np.float32)
    y, mm = _emu.kspace_filter(x, 3, [[], []], ct=True)
    assert relerr(y, x) < 2e-6


@pytest.mark.parametrize("shape", [(2, 20, 24, 35), (2, 36, 20, 28), (1, 128, 20, 28), (1, 240, 24, 35)])
def test_compiled_tile_plan(shape):
    """Pass B through the compile-time tile plan (kspace_ct.h, H in {20, 36, 128, 240}) together with
    the compiled slab passes: == oracle for disk/spike/wrap/Gibbs and a grouped pair of spikes."""
    rng = np.random.default_rng(sum(shape) + 1)
    x = rng.standard_normal(shape).astype(np.float32)
    sp = x.shape[1:]
    geo = K.geometry(sp)
    idx = (min(5, sp[0] - 1), min(3, sp[1] - 1), min(7, sp[2] // 2))
    prog = [K.disk_op(0.3 * min(sp), False), K.spike_op(idx, geo, 6.0, phase=0.7), K.wrap_op(0.5)]
    yc, _ = _emu.kspace_filter(x[None], 3, [prog], ct=True)
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x, 0.3 * min(sp)), idx, 6.0, phase=[0.7] * shape[0]), 0.5)
    assert relerr(yc[0], ref) < TOL
    yg, _ = _emu.kspace_filter(x[None], 3, [[K.gibbs_op(0.4, sp)]], ct=True)
    assert relerr(yg[0], O.gibbs_noise(x, 0.4)) < TOL
    # two spikes of one KSpaceSpikeNoise call (grouped), per channel
    prog2 = [K.spike_op(idx, geo, 5.0, phase=0.1, chan=0), K.spike_op((1, 1, 1), geo, 7.0, phase=-0.3, chan=0)]
    prog2[1].reserved = 1
    y2c, _ = _emu.kspace_filter(x[None], 3, [prog2], ct=True)
    y2g, _ = _emu.kspace_filter(x[None], 3, [prog2], ct=False)
    assert relerr(y2c, y2g) < 2e-6


@pytest.mark.parametrize("shape", [(2, 20, 48, 35), (1, 240, 240, 155)])
def test_half_units_split_spectrum(shape):
    """Passes A / C as half units (row parity) over the split spectrum, pass B finishing the W
    transform (slab_ct.h HalfPlan, kspace_ct.h b_mid_split): == oracle for the generic program path
    (disk, spike, wrap; a grouped spike pair) and each mask-only middle phase (Gibbs, disk), == the
    whole-slab compiled passes to rounding; pads zeroed, min/max epilogue exact."""
    rng = np.random.default_rng(sum(shape) + 5)
    x = rng.standard_normal(shape).astype(np.float32)
    sp = x.shape[1:]
    geo = K.geometry(sp)
    idx = (min(5, sp[0] - 1), min(3, sp[1] - 1), min(7, sp[2] // 2))
    prog = [K.disk_op(0.3 * min(sp), False), K.spike_op(idx, geo, 6.0, phase=0.7), K.wrap_op(0.5)]
    yh, mmh = _emu.kspace_filter(x[None], 3, [prog], pad=3, ct=2)
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x, 0.3 * min(sp)), idx, 6.0, phase=[0.7] * shape[0]), 0.5)
    assert relerr(yh[0, ..., :sp[-1]], ref) < TOL
    assert np.all(yh[0, ..., sp[-1]:] == 0)
    y0 = yh[0, ..., :sp[-1]]
    np.testing.assert_array_equal(mmh[0], [y0.min(), y0.max()])
    yw, _ = _emu.kspace_filter(x[None], 3, [prog], pad=3, ct=True)
    assert relerr(yh, yw) < 2e-6
    yg, _ = _emu.kspace_filter(x[None], 3, [[K.gibbs_op(0.4, sp)]], ct=2)
    assert relerr(yg[0], O.gibbs_noise(x, 0.4)) < TOL
    yd, _ = _emu.kspace_filter(x[None], 3, [[K.disk_op(0.25 * min(sp), True)]], ct=2)
    assert relerr(yd[0], O.fourier_disk(x, 0.25 * min(sp), inside_off=True)) < TOL
    prog2 = [K.spike_op(idx, geo, 5.0, phase=0.1, chan=0), K.spike_op((1, 1, 1), geo, 7.0, phase=-0.3, chan=0)]
    prog2[1].reserved = 1
    y2h, _ = _emu.kspace_filter(x[None], 3, [prog2], ct=2)
    y2g, _ = _emu.kspace_filter(x[None], 3, [prog2], ct=False)
    assert relerr(y2h, y2g) < 2e-6
