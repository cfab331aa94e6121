"""GPU parity of the band-limited passes A'/B'/C' (csrc/kern_band.hip) against the full-spectrum
passes A/B/C (same op program, tb_set_band_plans(0)) and against the numpy oracle; the identity
copy of empty programs; mixed routes inside one batch.

Tolerances: band vs full  max|d| / max|y| <= 2e-6;  vs oracle <= 1e-5 (north_star);  identity
samples, zero padding and min/max bit-exact.
"""
import numpy as np
import pytest
import torch

from _golden import relerr
from oracle import filters_oracle as O
from texbias import kprog as K

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt(gpu):
    from texbias import runtime
    return runtime


def both(rt, x, progs, C, pad=0, n_dims=3):
    """(band, full, band kernels seen, mm_band, mm_full)"""
    B = len(progs)
    mm_b = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    mm_f = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    rt.set_pass_timing(True)
    yb = rt.kspace_filter(x, n_dims, progs, C, pad=pad, minmax=mm_b)
    _, cnt, _, names = rt.pass_stats()
    rt.set_pass_timing(False)
    try:
        rt.set_band_plans(False)
        yf = rt.kspace_filter(x, n_dims, progs, C, pad=pad, minmax=mm_f)
    finally:
        rt.set_band_plans(True)
    torch.cuda.synchronize()
    return yb, yf, names, mm_b, mm_f


def spike(idx, spatial, li, phase=None, chan=-1, grouped=False):
    op = K.spike_op(idx, K.geometry(spatial), li, phase=phase, chan=chan)
    if grouped:
        op.reserved = 1
    return op


# D mod 4 = 0, 3, 2, 1, 0, 0, 3: every mirror-store alignment of pass C'; D = 64, 128: the Nyquist
# column summed on the VALU (D % 64 == 0)
SHAPES = [(2, 4, 32, 30, 16), (2, 3, 24, 20, 15), (1, 2, 31, 17, 30), (1, 3, 20, 22, 33), (1, 2, 40, 36, 64),
          (1, 4, 128, 128, 128), (2, 4, 240, 240, 155)]


@pytest.mark.parametrize("shape", SHAPES)
def test_band_disk_spike_wrap_matches_full(rt, shape):
    """The production chain program (disk -> plane-wave spike -> wrap), spike outside the box."""
    torch.manual_seed(1)
    x = torch.randn(shape, device="cuda")
    sp = shape[2:]
    r = 12.5 if min(sp) > 60 else 4.5
    idx = tuple(int(n * 0.8) for n in sp)
    progs = [[K.disk_op(r, False), spike(idx, sp, 10.0, phase=0.3 + b), K.wrap_op(0.5)] for b in range(shape[0])]
    yb, yf, names, mmb, mmf = both(rt, x, progs, shape[1], pad=5)
    assert names[0] == "k_band_fwd" and names[2] == "k_band_inv16"
    assert torch.all(yb[..., sp[-1]:] == 0)
    assert (yb - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    vb = yb[..., : sp[-1]].reshape(shape[0], -1)
    mmf_ = rt.keys_to_float(mmb)
    np.testing.assert_array_equal(mmf_[:, 0], vb.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(mmf_[:, 1], vb.max(1).values.cpu().numpy())
    # one channel against the oracle (reference semantics, phase hook)
    b, c = shape[0] - 1, shape[1] - 1
    ref = O.wrap_artifact(O.plane_waves(O.fourier_disk(x[b, c:c + 1].cpu().numpy(), r), idx, 10.0,
                                        phase=[0.3 + b]), 0.5)[0]
    assert relerr(yb[b, c, ..., : sp[-1]].cpu().numpy(), ref) < 1e-5


@pytest.mark.parametrize("prog_kind", ["int_radius", "spike_in_box", "spike_kd0", "spike_nyquist", "group_spikes",
                                       "highpass_after", "gibbs", "layer", "spike_before_lowpass", "empty_box"])
def test_band_program_variants(rt, prog_kind):
    torch.manual_seed(2)
    shape = (2, 3, 32, 30, 16)
    sp = shape[2:]
    x = torch.randn(shape, device="cuda")
    if prog_kind == "int_radius":
        prog = [K.disk_op(5, False), K.wrap_op(0.25)]
    elif prog_kind == "spike_in_box":      # spike inside the box: applied by pass B' to the kept coefficient
        prog = [K.disk_op(6.0, False), spike((17, 16, 9), sp, 9.0)]
    elif prog_kind == "spike_kd0":         # kd = 0 plane: both f and -f stored
        prog = [K.disk_op(4.0, False), spike((26, 5, 8), sp, 9.0, phase=1.1)]
    elif prog_kind == "spike_nyquist":     # self-conjugate coefficient (all axes at 0 or n/2)
        prog = [K.disk_op(4.0, False), spike((0, 0, 0), sp, 9.0, phase=0.7)]
    elif prog_kind == "group_spikes":      # one KSpaceSpikeNoise call, per-channel locations
        prog = [K.disk_op(5.0, False), spike((3, 4, 5), sp, 8.0, chan=0),
                spike((20, 9, 13), sp, 8.5, chan=1, grouped=True), spike((10, 25, 2), sp, 9.5, chan=2, grouped=True)]
    elif prog_kind == "highpass_after":
        prog = [K.disk_op(7.0, False), K.disk_op(3.0, True), K.wrap_op(0.75)]
    elif prog_kind == "gibbs":             # MONAI-style Gibbs, off-DC centre, float64 threshold
        prog = [K.gibbs_op(0.85, sp), K.wrap_op(0.5)]
    elif prog_kind == "layer":             # GibbsNoiseLayer mask with a host alpha
        prog = [K.layer_op(0.15, sp)]
    elif prog_kind == "spike_before_lowpass":
        prog = [spike((3, 4, 5), sp, 8.0), K.disk_op(5.0, False), spike((20, 9, 13), sp, 8.5)]
    else:                                   # radius below 1: only DC survives
        prog = [K.disk_op(0.5, False), spike((20, 9, 13), sp, 8.5)]
    yb, yf, names, mmb, mmf = both(rt, x, [prog, prog], shape[1], pad=3)
    assert names[0] == "k_band_fwd", names
    assert (yb - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    assert torch.all(yb[..., sp[-1]:] == 0)


@pytest.mark.parametrize("radius", [9.0, 15.5, 18.0, 20.0])
def test_band_tile_variants_unpadded(rt, radius):
    """All four pass-A' instantiations (NDk <= 16 or 32 kd columns, KW < 16 or 32 kw rows), whose
    slab-end O partials outgrow the 64-row chunk in LDS at the larger ones; odd D, no padding (the
    scalar-store path of pass C')."""
    torch.manual_seed(5)
    shape = (2, 2, 96, 112, 77)
    x = torch.randn(shape, device="cuda")
    geo = K.geometry(shape[2:])
    prog = [K.disk_op(radius, False), K.spike_op((60, 90, 30), geo, 9.0, phase=0.2), K.wrap_op(0.25)]
    yb, yf, names, mmb, mmf = both(rt, x, [prog, prog], shape[1])
    assert names[0] == "k_band_fwd", names
    assert torch.isfinite(yb).all()
    assert (yb - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    mmf_ = rt.keys_to_float(mmb)
    np.testing.assert_array_equal(mmf_[:, 1], yb.reshape(2, -1).max(1).values.cpu().numpy())


def test_band_2d_and_1d_geometry(rt):
    """Size-1 leading axes (the reference's 2-D slices: [C, 1, H, W] / [C, 256, 256])."""
    torch.manual_seed(3)
    x = torch.randn((1, 2, 1, 96, 80), device="cuda")
    prog = [K.disk_op(9.0, False), K.wrap_op(0.5)]
    yb, yf, names, _, _ = both(rt, x, [prog], 2)
    assert names[0] == "k_band_fwd"
    assert (yb - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    ref = O.wrap_artifact(O.fourier_disk(x[0].cpu().numpy(), 9.0), 0.5)
    assert relerr(yb[0].cpu().numpy(), ref) < 1e-5


def test_identity_copy_and_mixed_routes(rt):
    """Empty programs are copied through bit for bit (padding zeroed, exact min/max); a batch mixing
    band, empty and full-spectrum programs routes each run separately."""
    torch.manual_seed(4)
    shape = (4, 2, 24, 20, 15)
    sp = shape[2:]
    x = torch.randn(shape, device="cuda")
    progs = [[K.disk_op(4.0, False), K.wrap_op(0.5)], [], [K.wrap_op(0.5)], []]
    mm = torch.empty((4, 2), dtype=torch.int32, device="cuda")
    y = rt.kspace_filter(x, 3, progs, 2, pad=4, minmax=mm)
    assert torch.all(y[..., sp[-1]:] == 0)
    assert torch.equal(y[1, ..., : sp[-1]], x[1]) and torch.equal(y[3, ..., : sp[-1]], x[3])
    mmf = rt.keys_to_float(mm)
    for b in (1, 3):
        assert mmf[b, 0] == x[b].min().item() and mmf[b, 1] == x[b].max().item()
    xh = x.cpu().numpy()
    ref0 = O.wrap_artifact(O.fourier_disk(xh[0], 4.0), 0.5)
    ref2 = O.wrap_artifact(xh[2], 0.5)
    assert relerr(y[0, ..., : sp[-1]].cpu().numpy(), ref0) < 1e-5
    assert relerr(y[2, ..., : sp[-1]].cpu().numpy(), ref2) < 1e-5


def test_band_in_place_on_padded_view(rt):
    """Filtering the padded U-Net buffer in place (strided rows, y aliases x), as FusedChain does
    for a k-space segment that follows salt-and-pepper."""
    torch.manual_seed(5)
    shape = (2, 4, 32, 30, 16)
    x = torch.randn(shape, device="cuda")
    buf = torch.nn.functional.pad(x, (0, 5))
    view = buf[..., :16]
    prog = [K.disk_op(5.5, False), spike((25, 3, 9), shape[2:], 9.0, phase=0.2), K.wrap_op(0.5)]
    ref = rt.kspace_filter(x, 3, [prog, prog], 4)
    rt.kspace_filter(view, 3, [prog, prog], 4, out=view)
    torch.cuda.synchronize()
    assert torch.all(buf[..., 16:] == 0)
    assert (view - ref).abs().max().item() / ref.abs().max().item() < 1e-6


def test_band_c3_kernels_and_bytes(rt):
    """bench.py's launch: 2 x 4 x 240 x 240 x 155, pad 5 -> the band kernels, and the algorithmic
    bytes the library reports for them (image read once by A', written once by C')."""
    x = torch.randn((2, 4, 240, 240, 155), device="cuda")
    geo = K.geometry((240, 240, 155))
    prog = [K.disk_op(12.5, False), K.spike_op((70, 137, 71), geo, 15.0), K.wrap_op(0.5)]
    rt.set_pass_timing(True)
    rt.kspace_filter(x, 3, [prog, prog], 4, pad=5)
    ms, cnt, nbytes, names = rt.pass_stats()
    rt.set_pass_timing(False)
    assert names[:3] == ["k_band_fwd", "k_band_hcol", "k_band_inv16"]
    img = 8 * 240 * 240 * 155 * 4
    assert img < nbytes[0] < 1.05 * img
    assert 8 * 240 * 240 * 160 * 4 < nbytes[2] < 1.05 * 8 * 240 * 240 * 160 * 4


def _inv_both(rt, x, progs, C, pad=0):
    """(split-f16 C', f32 C', kernel names of each)"""
    out = []
    for on in (True, False):
        rt.set_band_inv16(on)
        try:
            rt.set_pass_timing(True)
            y = rt.kspace_filter(x, 3, progs, C, pad=pad)
            torch.cuda.synchronize()
            names = rt.pass_stats()[3]
            rt.set_pass_timing(False)
        finally:
            rt.set_band_inv16(True)
        out += [y, names[2]]
    return out


@pytest.mark.parametrize("shape,r,npts", [((2, 4, 240, 240, 155), 12.5, 1), ((2, 4, 240, 240, 155), 25.1, 1),
                                          ((4, 4, 128, 128, 128), 12.5, 0), ((3, 2, 40, 36, 33), 7.0, 3),
                                          ((2, 3, 40, 40, 30), 9.0, 2)])
def test_band_inv16_matches_f32(rt, shape, r, npts):
    """Pass C' in split f16 (k_band_inv16) against the f32 MFMA synthesis (k_band_inv) on the same
    band spectrum: max|d| / max|y| <= 1e-6; both routes' kernels identified."""
    torch.manual_seed(7)
    x = torch.randn(shape, device="cuda") * 3.0 + 1.5
    sp = shape[2:]
    progs = []
    for b in range(shape[0]):
        prog = [K.disk_op(r, False)]
        for j in range(npts):
            idx = tuple(int(n * (0.8 - 0.1 * j)) - b for n in sp)
            prog.append(spike(idx, sp, 9.0 + j, phase=0.3 * b + j))
        prog.append(K.wrap_op(0.5))
        progs.append(prog)
    y16, n16, y32, n32 = _inv_both(rt, x, progs, shape[1], pad=5)
    assert n16 == "k_band_inv16" and n32 == "k_band_inv", (n16, n32)
    assert torch.all(y16[..., sp[-1]:] == 0)
    assert (y16 - y32).abs().max().item() / y32.abs().max().item() < 1e-6


def test_band_inv16_falls_back_past_32_rows(rt):
    """More band columns + launch points than the split-f16 kernel's 64 V rows: the f32 kernel runs."""
    torch.manual_seed(8)
    shape = (8, 1, 96, 96, 80)
    sp = shape[2:]
    x = torch.randn(shape, device="cuda")
    progs = [[K.disk_op(20.0, False)] + [spike((40 + j, 30 - b, 50 - j), sp, 8.0) for j in range(3)]
             for b in range(shape[0])]
    rt.set_pass_timing(True)
    rt.kspace_filter(x, 3, progs, 1)
    torch.cuda.synchronize()
    names = rt.pass_stats()[3]
    rt.set_pass_timing(False)
    assert names[2] == "k_band_inv", names


@pytest.mark.parametrize("layout", ["ten_lowpass", "copy_then_band", "mixed_routes"])
def test_band_runs_at_nonzero_offset(rt, layout):
    """Band runs that do not start at sample 0 (bc0 != 0): a batch past TB_MAX_BATCH (second launch
    group), a band run after an identity sample, and band / closed-form / full / copy runs
    interleaved -- against the full-spectrum passes, with every sample's min/max keys exact."""
    torch.manual_seed(11)
    C, sp = 2, (24, 20, 15)
    lp = [K.disk_op(4.5, False), K.wrap_op(0.5)]
    if layout == "ten_lowpass":
        progs = [[K.disk_op(4.0 + 0.25 * b, False), K.wrap_op(0.5)] for b in range(10)]
    elif layout == "copy_then_band":
        progs = [[], lp, lp]
    else:
        progs = [lp, [spike((5, 7, 3), sp, 9.0)], [K.wrap_op(0.25)], lp, [], lp]
    B = len(progs)
    x = torch.randn((B, C) + sp, device="cuda")
    mm_b = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    mm_f = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    yb = rt.kspace_filter(x, 3, progs, C, pad=3, minmax=mm_b)
    try:
        rt.set_band_plans(False)
        rt.set_point_plans(False)
        yf = rt.kspace_filter(x, 3, progs, C, pad=3, minmax=mm_f)
    finally:
        rt.set_band_plans(True)
        rt.set_point_plans(True)
    torch.cuda.synchronize()
    assert torch.all(yb[..., sp[-1]:] == 0)
    assert (yb - yf).abs().max().item() / yf.abs().max().item() < 2e-6
    v = yb[..., : sp[-1]].reshape(B, -1)
    m = rt.keys_to_float(mm_b)
    np.testing.assert_array_equal(m[:, 0], v.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(m[:, 1], v.max(1).values.cpu().numpy())
    for b, p in enumerate(progs):
        if not p:
            assert torch.equal(yb[b, ..., : sp[-1]], x[b])


@pytest.mark.parametrize("extra,base", [(0, 0), (0, 1), (1, 0), (4, 0), (97, 2)])
def test_band_output_layouts(rt, extra, base):
    """Pass C' output orientations: 16-B aligned rows take the whole-line regrouped stores
    (tile_rows8), rows of odd stride or an unaligned base the 16-B / 4-B piecewise stores -- the same
    values, the pad columns zero, columns past the pad untouched, min/max keys of what was written."""
    torch.manual_seed(5)
    C, sp, pad = 2, (40, 37, 33), 3
    progs = [[K.disk_op(6.0, False), K.wrap_op(0.5)], [K.disk_op(9.5, False)]]
    B = len(progs)
    x = torch.randn((B, C) + sp, device="cuda")
    ref = rt.kspace_filter(x, 3, progs, C, pad=pad)
    row = sp[-1] + pad + extra
    buf = torch.full((B * C * sp[0] * sp[1] * row + base,), float("nan"), device="cuda")
    out = buf[base:].view(B, C, sp[0], sp[1], row)[..., : sp[-1] + pad]
    mm = torch.empty((B, 2), dtype=torch.int32, device="cuda")
    y = rt.kspace_filter(x, 3, progs, C, out=out, pad=pad, minmax=mm)
    torch.cuda.synchronize()
    assert y.data_ptr() == out.data_ptr()
    assert torch.all(out[..., sp[-1]:] == 0)
    assert (out - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    if extra:
        assert torch.isnan(buf[base:].view(B, C, sp[0], sp[1], row)[..., sp[-1] + pad:]).all()
    v = out[..., : sp[-1]].reshape(B, -1)
    m = rt.keys_to_float(mm)
    np.testing.assert_array_equal(m[:, 0], v.min(1).values.cpu().numpy())
    np.testing.assert_array_equal(m[:, 1], v.max(1).values.cpu().numpy())
