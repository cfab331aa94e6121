#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE code.

TEST INFRASTRUCTURE.  Runs only in the build container (where the read-only
reference checkout lives at /root/reference); the fixtures it writes are data
(inputs, parameters, RNG draws, outputs) and are what travels.  Nothing of the
reference's source is copied: the script imports
``source_code/filters_and_operators.py`` and ``source_code/stylization_layers.py``
in place (with ``monai_stub`` standing in for MONAI's base classes, see that
module's docstring) and records what they return.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("TB_REFERENCE", "/root/reference/source_code")

sys.dont_write_bytecode = True
sys.path.insert(0, HERE)
import monai_stub  # noqa: E402

monai_stub.install()
sys.path.insert(0, REF)
import filters_and_operators as fo  # noqa: E402
import stylization_layers as sl  # noqa: E402

torch.set_num_threads(1)


def brats_like(shape, seed):
    """BraTS-like z-scored volume: zero background, smooth field + noise in an
    ellipsoidal 'brain' (mirrors NormalizeIntensityd(nonzero, channel_wise))."""
    rng = np.random.default_rng(seed)
    c, sp = shape[0], shape[1:]
    grids = np.meshgrid(*[np.linspace(-1, 1, n) for n in sp], indexing="ij")
    r2 = sum((g / 0.8) ** 2 for g in grids)
    brain = r2 < 1.0
    out = np.zeros(shape, np.float32)
    for ch in range(c):
        k = np.fft.fftn(rng.standard_normal(sp))
        freq = np.meshgrid(*[np.fft.fftfreq(n) for n in sp], indexing="ij")
        k *= np.exp(-sum(f ** 2 for f in freq) / (2 * 0.08 ** 2))
        field = np.real(np.fft.ifftn(k))
        field = field / (field.std() + 1e-12) + 0.5 * rng.standard_normal(sp)
        v = field[brain]
        out[ch][brain] = ((v - v.mean()) / v.std()).astype(np.float32)
    return out


CASES = {}


def put(name, meta, **arrays):
    CASES[name] = (meta, arrays)


def t(x):
    return torch.from_numpy(np.ascontiguousarray(x))


def spectrum(x):
    return torch.fft.fftshift(torch.fft.fftn(x, dim=(-3, -2, -1)), dim=(-3, -2, -1))


# --------------------------------------------------------------------- disk
def gen_disk():
    specs = [
        ((4, 32, 30, 15), 5.0, False, None),
        ((4, 32, 30, 15), 5.0, True, None),
        ((4, 24, 20, 31), 7.5, False, None),
        ((4, 16, 16, 16), 3, False, None),          # int radius
        ((4, 16, 16, 16), float("inf"), False, None),
        ((4, 16, 16, 16), [2.0, 6.0], False, 11),   # sampled-then-frozen radius
        ((1, 256, 256), 40.0, False, None),          # config 1: 2-D slice
    ]
    for i, (shape, r, off, seed) in enumerate(specs):
        x = brats_like(shape, 100 + i)
        tr = fo.RandFourierDiskMaskd(keys="image", r=r, inside_off=off, prob=1.0)
        if seed is not None:
            tr.set_random_state(seed)
        y = tr({"image": t(x)})["image"]
        put(f"disk_{i}", dict(kind="disk", shape=shape, r=r if not isinstance(r, float) or np.isfinite(r) else "inf",
                               r_used=float(tr.r), inside_off=off, seed=seed),
            x=x, y=y.contiguous().numpy())
    # known answers: mask counts
    counts = {}
    k = torch.zeros((1, 64, 64, 64), dtype=torch.complex64)
    counts["disk3d_r12.5_64cube"] = int(fo.disk_mask(k, r=12.5, dim=3, inside_off=False).binary_mask.sum())
    k2 = torch.zeros((1, 256, 256), dtype=torch.complex64)
    counts["disk2d_r40_256"] = int(fo.disk_mask(k2, r=40, dim=2, inside_off=False).binary_mask.sum())
    m2 = fo.disk_mask(torch.zeros((2, 20, 17), dtype=torch.complex64), r=6.5, dim=2, inside_off=True).binary_mask
    put("diskmask_counts", dict(kind="counts", counts=counts), mask2d_20x17=m2.numpy())


# ------------------------------------------------------------------ planes
def gen_planes():
    specs = [((4, 24, 20, 16), (8.0, 7.0, 5.0), 6.0, 3),
             ((4, 20, 18, 15), (7.0, 6.0, 4.0), 9.0, 4),
             ((2, 16, 16, 16), (5.0, 5.0, 5.0), 7.5, 5)]
    for i, (shape, abc, inten, seed) in enumerate(specs):
        x = brats_like(shape, 200 + i)
        tr = fo.RandPlaneWaves_ellipsoid("image", *abc, intensity_value=inten, prob=1.0)
        tr.set_random_state(seed)
        tr.ellipsoid.set_random_state(seed + 1000)
        k = spectrum(t(x))
        y = tr({"image": t(x)})["image"]
        idx = tuple(int(v) for v in tr.idx)
        put(f"planes_{i}", dict(kind="planes", shape=shape, abc=abc, intensity=inten, seed=seed,
                                ell_seed=seed + 1000, idx=idx),
            x=x, y=y.contiguous().numpy(),
            phase=k[:, idx[0], idx[1], idx[2]].angle().numpy(),
            absk=k[:, idx[0], idx[1], idx[2]].abs().numpy())
    # known answers for the shell sampler
    e = fo.ellipsoid(55.0, 55.0, 30.0)
    cnt = int(e.binary_mask_3d(torch.zeros(128, 128, 64)).sum())
    draws = {}
    for shp in [(128, 128, 64), (240, 240, 155)]:
        e.set_random_state(0)
        draws[str(shp)] = [list(map(int, e.sample_ellipsoid(torch.zeros(shp)))) for _ in range(4)]
    put("ellipsoid_known", dict(kind="ellipsoid", abc=(55.0, 55.0, 30.0), count_128x128x64=cnt, draws_seed0=draws))


# -------------------------------------------------------------------- wrap
def gen_wrap():
    for i, (shape, a) in enumerate([((4, 32, 30, 15), 0.5), ((4, 16, 16, 16), 0.25),
                                     ((4, 16, 16, 16), 0.0), ((4, 24, 20, 31), 0.75),
                                     ((2, 15, 17, 9), 1.0)]):
        x = brats_like(shape, 300 + i)
        y = fo.WrapArtifactd("image", a)({"image": t(x)})["image"]
        put(f"wrap_{i}", dict(kind="wrap", shape=shape, alpha=a), x=x, y=y.contiguous().numpy())


# --------------------------------------------------------------------- S&P
def gen_sap():
    for i, (shape, p) in enumerate([((4, 16, 20, 12), 0.05), ((4, 16, 20, 12), 0.35),
                                     ((2, 8, 8, 8), 0.0), ((2, 8, 8, 8), 1.0), ((2, 9, 7, 5), 1.5)]):
        x = brats_like(shape, 400 + i)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            tr = fo.SaltAndPepper(p)
        tr.set_random_state(40 + i)
        torch.manual_seed(1234 + i)
        y = tr({"image": t(x)})["image"]
        torch.manual_seed(1234 + i)
        u = torch.rand(shape).numpy()
        cls = np.zeros(shape, np.int8)
        cls[u <= np.float32(tr.p / 2)] = 1
        cls[(u > np.float32(tr.p / 2)) & (u <= np.float32(tr.p))] = 2
        put(f"sap_{i}", dict(kind="sap", shape=shape, p=p, p_used=tr.p, torch_seed=1234 + i),
            x=x, y=y.numpy(), u=u, cls=cls)


# ------------------------------------------------------------------- Gibbs
def gen_gibbs():
    specs = [((4, 32, 30, 15), 0.5), ((4, 16, 16, 16), 0.3), ((4, 16, 16, 16), 0.0),
             ((4, 16, 16, 16), 1.0), ((4, 24, 20, 31), 0.9), ((2, 40, 36), 0.5), ((3, 31, 17), 0.7)]
    for i, (shape, a) in enumerate(specs):
        x = brats_like(shape, 500 + i)
        y = fo.GibbsNoise(a)(t(x))
        put(f"gibbs_{i}", dict(kind="gibbs", shape=shape, alpha=a), x=x, y=y.contiguous().numpy())
    x = brats_like((4, 16, 18, 14), 590)
    tr = fo.RandGibbsNoise(prob=0.7, alpha=(0.2, 0.8))
    tr.set_random_state(7)
    outs, alphas, dos = [], [], []
    for _ in range(3):
        outs.append(tr(t(x)).contiguous().numpy())
        alphas.append(float(tr.sampled_alpha))
        dos.append(bool(tr._do_transform))
    put("randgibbs", dict(kind="randgibbs", shape=x.shape, prob=0.7, alpha=(0.2, 0.8), seed=7,
                           sampled_alpha=alphas, do=dos), x=x, y=np.stack(outs))
    trd = fo.RandGibbsNoised("image", prob=1.0, alpha=(0.0, 0.6))
    trd.set_random_state(8)
    yd = trd({"image": t(x)})["image"]
    put("randgibbsd", dict(kind="randgibbsd", shape=x.shape, prob=1.0, alpha=(0.0, 0.6), seed=8,
                            sampled_alpha=float(trd.sampled_alpha)), x=x, y=yd.contiguous().numpy())
    # known answer: alpha=0.5 on 128x128x64 -> mask ones
    sh = (128, 128, 64)
    r = (1 - 0.5) * np.max(sh) * np.sqrt(2) / 2.0
    c = (np.array(sh) - 1) / 2
    co = np.ogrid[tuple(slice(0, i) for i in sh)]
    cnt = int((np.sqrt(sum((a - b) ** 2 for a, b in zip(co, c))) <= r).sum())
    put("gibbs_known", dict(kind="counts", counts={"gibbs_a0.5_128x128x64": cnt}))


# ------------------------------------------------------------------ spikes
def gen_spikes():
    x = brats_like((4, 16, 18, 14), 600)
    cases = [
        dict(loc=(5, 9, 3), k_intensity=11.0),
        dict(loc=((0, 5, 9, 3), (2, 12, 4, 7), (3, 0, 0, 0)), k_intensity=(10.0, 12.5, 9.0)),
        dict(loc=(8, 9, 7), k_intensity=None),
        dict(loc=((1, 3, 3, 3), (1, 13, 15, 11)), k_intensity=None),
    ]
    for i, cs in enumerate(cases):
        try:
            y = fo.KSpaceSpikeNoise(cs["loc"], cs["k_intensity"])(t(x))
        except Exception as e:  # the reference's own failure mode is part of the contract
            put(f"kspike_{i}", dict(kind="kspike", shape=x.shape, error=type(e).__name__, **cs), x=x)
            continue
        la = torch.log(torch.absolute(spectrum(t(x))) + 1e-10)
        dflt = [float(v) for v in torch.mean(la, dim=(-3, -2, -1)) * 2.5]   # the reference's own default (:933)
        put(f"kspike_{i}", dict(kind="kspike", shape=x.shape, default_intensity=dflt, **cs), x=x,
            y=y.contiguous().numpy())
    x2 = brats_like((3, 30, 28), 601)
    y2 = fo.KSpaceSpikeNoise(((0, 4, 20), (2, 15, 14)), (9.0, 8.0))(t(x2))
    put("kspike_2d", dict(kind="kspike", shape=x2.shape, loc=((0, 4, 20), (2, 15, 14)), k_intensity=(9.0, 8.0)),
        x=x2, y=y2.contiguous().numpy())
    rcases = [dict(prob=1.0, intensity_range=(10.0, 12.0), channel_wise=True, seed=21),
              dict(prob=0.6, intensity_range=((9.0, 10.0), (10.0, 11.0), (11.0, 12.0), (12.0, 13.0)),
                   channel_wise=True, seed=22),
              dict(prob=1.0, intensity_range=(11.0, 11.0), channel_wise=False, seed=23),
              dict(prob=1.0, intensity_range=None, channel_wise=True, seed=24)]
    for i, rc in enumerate(rcases):
        tr = fo.RandKSpaceSpikeNoise(rc["prob"], rc["intensity_range"], rc["channel_wise"])
        tr.set_random_state(rc["seed"])
        y = tr(t(x))
        put(f"randkspike_{i}", dict(kind="randkspike", shape=x.shape, **rc,
                                     locs=[list(map(int, l)) for l in tr.sampled_locs],
                                     intens=[float(v) for v in tr.sampled_k_intensity]),
            x=x, y=y.contiguous().numpy())
    trd = fo.RandKSpaceSpikeNoised("image", global_prob=1.0, prob=1.0, intensity_ranges={"image": (10.0, 11.0)})
    trd.set_rand_state(31)
    yd = trd({"image": t(x)})["image"]
    put("randkspiked", dict(kind="randkspiked", shape=x.shape, seed=31,
                             locs=[list(map(int, l)) for l in trd.transforms["image"].sampled_locs],
                             intens=[float(v) for v in trd.transforms["image"].sampled_k_intensity]),
        x=x, y=yd.contiguous().numpy())


# ------------------------------------------------------------------ layers
def gen_layers():
    for i, (shape, a) in enumerate([((2, 1, 16, 16, 8), 0.5), ((2, 1, 15, 16, 9), 0.7),
                                     ((1, 1, 12, 10, 8), 1.0), ((2, 1, 16, 16, 8), 0.05)]):
        x = brats_like(shape[1:], 700 + i)[None].repeat(shape[0], 0)
        x[1:] *= 0.5
        layer = sl.GibbsNoiseLayer(a)
        with torch.no_grad():
            y = layer(t(x))
        put(f"glayer_{i}", dict(kind="glayer", shape=shape, alpha=a), x=x, y=y.contiguous().numpy())
    layer = sl.GibbsNoiseLayer(0.7)
    ones = torch.ones((1, 1, 128, 128, 64), dtype=torch.complex64)
    cnt = int(layer._apply_mask(ones).real.sum())
    put("glayer_known", dict(kind="counts", counts={"layer_a0.7_128x128x64": cnt}))
    for i, (shape, inten, seed) in enumerate([((2, 1, 16, 16, 8), 9.0, 51), ((3, 1, 12, 14, 10), 12.0, 52)]):
        x = brats_like(shape[1:], 750 + i)[None].repeat(shape[0], 0)
        fo.Randomizable.R = np.random.RandomState(seed)
        sp = sl.spike_layer(inten)
        y = sp(t(x))
        fo.Randomizable.R = np.random.RandomState(seed)
        st = fo.RandKSpaceSpikeNoise(prob=1.0, intensity_range=(inten, inten), channel_wise=False)
        st._randomize(t(x), st._make_sequence(t(x)))
        put(f"slayer_{i}", dict(kind="slayer", shape=shape, intensity=inten, seed=seed,
                                 locs=[list(map(int, l)) for l in st.sampled_locs]),
            x=x, y=y.contiguous().numpy())
    fo.Randomizable.R = np.random.RandomState()


# ------------------------------------------------------------------- chain
def gen_chain():
    specs = [((4, 32, 30, 16), 5.0, (10.0, 9.0, 5.0), 8.0, 0.5, 0.05, 61),
             ((4, 24, 20, 15), 4.5, (8.0, 7.0, 5.0), 7.0, 0.25, 0.15, 62),
             ((2, 32, 32, 32), 20.0, (9.0, 9.0, 6.0), 10.0, 0.5, 0.05, 63)]
    for i, (shape, r, abc, inten, alpha, p, seed) in enumerate(specs):
        x = brats_like(shape, 800 + i)
        disk = fo.RandFourierDiskMaskd(keys="image", r=r, inside_off=False, prob=1.0)
        planes = fo.RandPlaneWaves_ellipsoid("image", *abc, intensity_value=inten, prob=1.0)
        wrap = fo.WrapArtifactd("image", alpha)
        sap = fo.SaltAndPepper(p)
        for j, tr in enumerate((disk, planes, sap)):
            tr.set_random_state(seed + j)
        planes.ellipsoid.set_random_state(seed + 100)
        d = {"image": t(x)}
        d1 = disk(d)
        k1 = spectrum(d1["image"])
        d2 = planes(d1)
        idx = tuple(int(v) for v in planes.idx)
        d3 = wrap(d2)
        torch.manual_seed(seed)
        d4 = sap(d3)
        torch.manual_seed(seed)
        u = torch.rand(shape).numpy()
        put(f"chain_{i}", dict(kind="chain", shape=shape, r=r, abc=abc, intensity=inten, alpha=alpha, p=p,
                                seed=seed, idx=idx),
            x=x, y1=d1["image"].contiguous().numpy(), y2=d2["image"].contiguous().numpy(),
            y3=d3["image"].contiguous().numpy(), y=d4["image"].contiguous().numpy(), u=u,
            phase=k1[:, idx[0], idx[1], idx[2]].angle().numpy(),
            absk=k1[:, idx[0], idx[1], idx[2]].abs().numpy())


def gen_labels():
    """ConvertToMultiChannelBasedOnBratsClassesd (filters_and_operators.py:61-87) on BraTS-style
    label maps (values 0..4; 4 is not a class of this dataset and maps to nothing)."""
    rng = np.random.default_rng(41)
    for i, shape in enumerate([(24, 20, 12), (1, 33, 17, 9)]):
        lab = rng.integers(0, 5, size=shape).astype(np.float32)
        t = fo.ConvertToMultiChannelBasedOnBratsClassesd(keys="label")
        out = t({"label": lab})["label"]
        put(f"labels_{i}", {"shape": list(shape)}, label=lab, out=out)


def gen_zf():
    """RandZF (50_reconstruction/reconGan/utils2.py:34-74) on 2-D slices and a 3-D volume, with
    the uniform field it drew (replayed from the same torch seed) so the oracle can be pinned."""
    sys.path.insert(0, os.path.join(os.path.dirname(REF), "50_reconstruction", "reconGan"))
    import utils2  # noqa: E402
    for i, (shape, p) in enumerate([((1, 32, 28), 0.3), ((2, 16, 12, 10), 0.6)]):
        x = brats_like(shape, 50 + i)
        torch.manual_seed(1234 + i)
        y = utils2.RandZF(p)(torch.from_numpy(x))
        torch.manual_seed(1234 + i)
        u = torch.rand(shape)  # the draw inside rand_mask (k has the image's shape)
        put(f"zf_{i}", {"p": p}, x=x, u=u.numpy(), y=y.numpy())


GENERATORS = {"disk": "gen_disk", "planes": "gen_planes", "wrap": "gen_wrap", "sap": "gen_sap",
              "gibbs": "gen_gibbs", "spikes": "gen_spikes", "layers": "gen_layers", "chain": "gen_chain",
              "labels": "gen_labels", "zf": "gen_zf"}


def main():
    """All generators, or only those named on the command line (e.g. ``make_golden.py labels``)."""
    names = sys.argv[1:] or list(GENERATORS)
    for n in names:
        globals()[GENERATORS[n]]()
    groups = {}
    for name, (meta, arrays) in CASES.items():
        groups.setdefault(name.split("_")[0], {})[name] = (meta, arrays)
    for g, cases in groups.items():
        out = {}
        for name, (meta, arrays) in cases.items():
            out[f"{name}.meta"] = np.array(json.dumps(meta))
            for k, v in arrays.items():
                out[f"{name}.{k}"] = np.asarray(v)
        np.savez_compressed(os.path.join(HERE, f"golden_{g}.npz"), **out)
        print(g, len(cases), "cases")


if __name__ == "__main__":
    main()
