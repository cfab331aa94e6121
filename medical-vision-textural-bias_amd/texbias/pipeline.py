"""Batched device-side augmentation: a list of the reference's transforms compiled into
fused k-space passes over a collated [B, C, *spatial] batch.

The reference applies its transforms per sample in DataLoader workers, one full FFT round
trip per filter (e.g. 127_.../..._3modalities.py:171-174: disk -> planes -> wrap -> S&P).
``FusedChain`` keeps the same transform objects -- so every host RNG draw (prob draws, sampled
radius / alpha, the ellipsoid point) happens in the same order as a sequential Compose over
each sample -- but runs each maximal run of k-space transforms as ONE forward-FFT -> op program
-> inverse-FFT pass (``.real`` between filters is a Hermitian symmetrisation, which
the half-spectrum program reproduces exactly), then salt-and-pepper as a sparse in-place
scatter.  The k-space pass also writes the U-Net's zero D-padding and the per-sample min/max
salt-and-pepper needs, so the batch is read from HBM once per pass.

Salt-and-pepper draws its uniform field from a device Philox stream keyed per call from
torch's global generator (the reference uses ``torch.rand`` on the CPU, :472).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from . import kprog as K
from . import ops as tbops
from . import runtime as rt


def _kind(t) -> str:
    return type(t).__name__


KSPACE = {"RandFourierDiskMaskd", "RandPlaneWaves_ellipsoid", "WrapArtifactd", "WrapArtifact", "GibbsNoise",
          "RandGibbsNoise", "RandGibbsNoised", "KSpaceSpikeNoise", "RandKSpaceSpikeNoise", "RandKSpaceSpikeNoised"}
POINTWISE = {"SaltAndPepper"}
CHANNEL = {"SelectChanneld", "MultimodalSlicesd"}


def select_channel_index(t, key: str, keys_present: Sequence[str]) -> Optional[int]:
    """The channel SelectChanneld (filters_and_operators.py:25-58) keeps for ``key`` given the keys
    present in the sample, or None when it does not touch ``key``."""
    order = [k for k in t.keys if k in keys_present]
    if key not in order:
        return None
    cn = t.chan_num
    if isinstance(cn, Sequence) and not isinstance(cn, (str, bytes)):
        if len(cn) > 1:
            i = order.index(key)
            return int(cn[i]) if i < len(cn) else None
        return int(cn[0])
    return int(cn)


def spike_program(t, c_cur: int, spatial) -> List:
    """RandKSpaceSpikeNoise's draws for one [c_cur, *spatial] image (filters_and_operators.py:
    1047-1103) and the KSpaceSpikeNoise program they call (:906-983)."""
    import filters_and_operators as F
    if t.intensity_range is None:
        raise ValueError("FusedChain needs RandKSpaceSpikeNoise's intensity_range (the default range is data "
                         "dependent: 2.5 * mean log |k| of the sample)")
    if isinstance(t.intensity_range[0], Sequence) and len(t.intensity_range) != c_cur:
        raise AssertionError("If intensity_range is a sequence of sequences, then there must be one (low, high) "
                             "tuple for each channel.")
    meta = torch.empty((c_cur,) + tuple(spatial), device="meta")
    t.sampled_k_intensity = []
    t.sampled_locs = []
    t._randomize(meta, t._make_sequence(meta))
    if not t.sampled_locs:
        return []
    return F.KSpaceSpikeNoise(t.sampled_locs, t.sampled_k_intensity).program(meta)


class FusedChain:
    """Compile ``transforms`` (instances from filters_and_operators) for batched device execution.

    ``__call__(x, pad=0)``: x [B, C, *spatial] float32 on a HIP device (spatial = 3 axes);
    returns [B, C', *spatial[:-1], spatial[-1] + pad] (C' = 1 after a channel selection).  The
    same transform objects draw for every sample in turn, exactly like a per-sample Compose
    (per-rank streams: seed the transforms per rank with ``set_random_state``).  ``apply(data)``
    takes a collated dict ({"image", "label"}) and also applies the channel selections to the
    label (``SelectChanneld`` / ``MultimodalSlicesd``).

    Parity hooks (the reference's draws that a device run cannot reproduce):
    ``phases`` -- per sample, the per-channel phase of the plane-wave spike coefficient as the
    reference measured it (``angle(K[idx])`` after the low-pass is rounding noise); ``u`` -- the
    salt-and-pepper uniform field [B, C, *spatial] (the reference's ``torch.rand``, :472);
    ``cls`` -- int8 [B, C, *spatial] receiving the salt-and-pepper class map (0 keep, 1 MIN, 2 MAX).
    After a call, ``last_minmax`` holds the per-sample (min, max) the salt-and-pepper stage used.
    """

    def __init__(self, transforms: Sequence, key: str = "image"):
        for t in transforms:
            if _kind(t) not in KSPACE | POINTWISE | CHANNEL:
                raise TypeError(f"{_kind(t)} is not a fusable texbias transform")
        self.transforms = list(transforms)
        self.key = key
        self._mm: Optional[torch.Tensor] = None
        self._mm_b = 0
        self._last_mm: Optional[torch.Tensor] = None
        self._label_sel: List[Optional[int]] = []

    @property
    def last_minmax(self) -> Optional[np.ndarray]:
        """float32 [B, 2] (min, max) per sample that the last call's salt-and-pepper stage used
        (decoded on demand: reading it synchronises), or None when no such stage ran."""
        return rt.keys_to_float(self._last_mm) if self._mm_b else None

    # --- host side: one sample's draws, in Compose order --------------------------------
    def _sample_plan(self, spatial, channels: int = 4, phase: Optional[Sequence[float]] = None,
                     keys_present: Sequence[str] = ("image",)) -> List:
        """Returns a list of stages for one sample: ('k', program), ('sap', p or None) or
        ('sel', channel); records the label channel a selection keeps in ``self._label_sel``."""
        stages: List = []
        prog: List = []
        seg = False   # the current segment holds a k-space transform (structure, not draws)
        c_cur = channels
        lsel: Optional[int] = None

        def close():
            nonlocal prog, seg
            if seg:
                stages.append(("k", prog))
            prog, seg = [], False

        for t in self.transforms:
            k = _kind(t)
            seg = seg or k in KSPACE
            if k == "RandFourierDiskMaskd":
                t.randomize()
                if t._do_transform:
                    prog += t.program()
            elif k == "RandPlaneWaves_ellipsoid":
                t.randomize(None)
                if t._do_transform:
                    ops = t.program_for(spatial, phase)
                    for op in ops[1:]:
                        op.reserved = 1   # one plane-wave call: all channels read the pre-call spectrum
                    prog += ops
            elif k == "WrapArtifactd":
                prog += t.transform.program()
            elif k == "WrapArtifact":
                prog += t.program()
            elif k == "GibbsNoise":
                prog += t.program(spatial)
            elif k in ("RandGibbsNoise", "RandGibbsNoised"):
                t._randomize(None)
                if t._do_transform:
                    prog += [K.gibbs_op(t.sampled_alpha, spatial)]
            elif k == "KSpaceSpikeNoise":
                if t.k_intensity is None:
                    raise ValueError("FusedChain needs explicit k_intensity (the default is data dependent)")
                prog += t.program(torch.empty((c_cur,) + tuple(spatial), device="meta"))
            elif k == "RandKSpaceSpikeNoise":
                prog += spike_program(t, c_cur, spatial)
            elif k == "RandKSpaceSpikeNoised":
                t.randomize(None)                   # the global probability (:1218)
                if t.common_sampling:
                    for kk in t.keys:
                        t.transforms[kk].set_random_state(t.common_seed)
                if self.key in t.keys and t._do_transform:
                    prog += spike_program(t.transforms[self.key], c_cur, spatial)
            elif k == "SaltAndPepper":
                t.randomize(None)
                close()
                stages.append(("sap", t.p if t._do_transform else None))
            elif k == "SelectChanneld":
                close()
                c = select_channel_index(t, self.key, keys_present)
                if c is not None:
                    if not 0 <= c < c_cur:
                        raise AssertionError(f"Provided channel index {c} larger than max channel index for key = "
                                             f"{self.key}")
                    stages.append(("sel", c))
                    c_cur = 1
                if "label" in keys_present:
                    lsel = select_channel_index(t, "label", keys_present)
            elif k == "MultimodalSlicesd":
                close()
                c = int(t.R.choice(t.img_chan_indices))   # one draw per call (…3modalities.py:99)
                if self.key in t.keys:
                    stages.append(("sel", c))
                    c_cur = 1
                if "label" in t.keys and "label" in keys_present:
                    lsel = int(t.label_idx)
        close()
        self._label_sel.append(lsel)
        return stages

    def plan(self, B: int, spatial, phases: Optional[Sequence[Sequence[float]]] = None, channels: int = 4,
             keys_present: Sequence[str] = ("image",)) -> List[List]:
        if phases is not None and len(phases) != B:
            raise ValueError("one phase list per sample")
        self._label_sel = []
        return [self._sample_plan(spatial, channels, None if phases is None else phases[b], keys_present)
                for b in range(B)]

    # --- device side --------------------------------------------------------------------
    def __call__(self, x: torch.Tensor, pad: int = 0, plans: Optional[List[List]] = None,
                 phases: Optional[Sequence[Sequence[float]]] = None, u: Optional[torch.Tensor] = None,
                 cls: Optional[torch.Tensor] = None, seed: Optional[int] = None,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``seed``: Philox key of the salt-and-pepper field (default: drawn from torch's global
        generator, which synchronises with the host; pass it explicitly to capture the chain in a
        HIP graph).  ``out``: optional [B, C, *spatial[:-1], D + pad] float32 buffer receiving the
        result (the first k-space pass writes it directly, e.g. a captured train step's static input)."""
        rt.require_hip(x, "FusedChain")
        if x.dim() != 5:
            raise ValueError("FusedChain expects [B, C, H, W, D]")
        B, C = x.shape[:2]
        plans = plans if plans is not None else self.plan(B, tuple(x.shape[2:]), phases, C)
        return self.execute(x, plans, pad=pad, u=u, cls=cls, seed=seed, out=out)

    def apply(self, data: dict, pad: int = 0, **kw) -> dict:
        """Dictionary form: ``data[self.key]`` through the chain; a "label" entry gets the channel
        selections (SelectChanneld / MultimodalSlicesd) the draws made for it."""
        d = dict(data)
        x = d[self.key]
        keys = [k for k in d]
        plans = self.plan(x.shape[0], tuple(x.shape[2:]), kw.pop("phases", None), x.shape[1], keys)
        d[self.key] = self.__call__(x, pad=pad, plans=plans, **kw)
        if "label" in d and any(s is not None for s in self._label_sel):
            lab = d["label"]
            idx = torch.tensor([s if s is not None else 0 for s in self._label_sel], device=lab.device)
            d["label"] = lab[torch.arange(lab.shape[0], device=lab.device), idx][:, None]
        return d

    def execute(self, x: torch.Tensor, plans: List[List], pad: int = 0, u: Optional[torch.Tensor] = None,
                cls: Optional[torch.Tensor] = None, seed: Optional[int] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Run per-sample stage lists (``plan`` or deferred plans) over the batch x [B, C, *spatial]
        (``out``: see ``__call__``)."""
        rt.require_hip(x, "FusedChain")
        if x.dim() != 5:
            raise ValueError("FusedChain expects [B, C, H, W, D]")
        B = x.shape[0]
        spatial = tuple(x.shape[2:])
        for t, nm in ((u, "u"), (cls, "cls")):
            if t is not None and tuple(t.shape) != tuple(x.shape):
                raise ValueError(f"{nm} must have the input's shape {tuple(x.shape)}")
        if len(plans) != B:
            raise ValueError(f"{len(plans)} plans for a batch of {B}")
        if out is not None:
            want = tuple(x.shape[:-1]) + (x.shape[-1] + pad,)
            if tuple(out.shape) != want or out.dtype != torch.float32 or out.device != x.device:
                raise ValueError(f"out must be a float32 {want} tensor on the input's device")
        nst = len(plans[0])
        if any(len(p) != nst or [s[0] for s in p] != [s[0] for s in plans[0]] for p in plans):
            raise ValueError("all samples of a batch must share the stage structure")
        if out is not None and any(s[0] == "sel" for s in plans[0]):
            raise ValueError("out= cannot take a chain with a channel selection (its result has fewer channels)")
        if self._mm is None or self._mm.shape[0] < B or self._mm.device != x.device:
            self._mm = torch.empty((max(B, 8), 2), dtype=torch.int32, device=x.device)
        mm = self._mm[:B]
        self._mm_b = 0
        self._last_mm = None
        cur = x
        padded = False
        mm_valid = False
        for si in range(nst):
            kind = plans[0][si][0]
            C = cur.shape[1]
            if kind == "k":
                progs = [p[si][1] for p in plans]
                if not any(progs):
                    continue   # every sample drew "no transform": identity
                out_pad = pad if not padded else 0
                if out is not None and cur is x and C == x.shape[1]:   # first pass: straight into the caller's buffer
                    rt.kspace_filter(cur, 3, progs, C, out=out, pad=out_pad, minmax=mm)
                    cur = out
                    padded = out_pad > 0
                elif padded:   # filter the padded buffer in place (pass A reads all before C writes)
                    view = cur[..., : spatial[-1]]
                    rt.kspace_filter(view, 3, progs, C, out=view, minmax=mm)
                else:   # the functional custom op (torch.compile / graph-capture friendly)
                    cur, mm = torch.ops.texbias.kspace_filter(cur, 3, tbops.pack_programs_split(progs, K.geometry(spatial).hwd), C,
                                                              out_pad)
                    padded = out_pad > 0
                mm_valid = True
            elif kind == "sel":
                chans = [int(p[si][1]) for p in plans]
                cur = cur[torch.arange(B, device=cur.device), torch.tensor(chans, device=cur.device)][:, None]
                if u is not None:
                    u = u[torch.arange(B, device=u.device), torch.tensor(chans, device=u.device)][:, None]
                if cls is not None:
                    raise ValueError("the cls hook is not supported across a channel selection")
                mm_valid = False   # the per-sample min/max was over the unselected channels
            else:
                ps = [p[si][1] for p in plans]
                seeds = [p[si][2] if len(p[si]) > 2 else None for p in plans]
                if all(v is None for v in ps):
                    continue
                if cur is x:
                    cur = x.clone() if not pad else torch.nn.functional.pad(x, (0, pad))
                    padded = padded or pad > 0
                view = cur[..., : spatial[-1]] if padded else cur
                if not mm_valid:
                    rt.minmax_keys(view, 4, out=mm)
                thr = [((np.float32(p / 2), np.float32(p)) if p is not None else (-1.0, -1.0)) for p in ps]
                if any(sd is not None for sd in seeds):
                    # deferred samples: each its own Philox key, drawn in its worker (the eager stream)
                    for b in range(B):
                        if ps[b] is not None:
                            torch.ops.texbias.salt_and_pepper_(view[b:b + 1], mm[b:b + 1],
                                                               torch.tensor([thr[b]], dtype=torch.float32),
                                                               int(seeds[b]), 0, 4)
                elif u is None and cls is None:
                    sd = seed if seed is not None else int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
                    torch.ops.texbias.salt_and_pepper_(view, mm, torch.tensor(thr, dtype=torch.float32), sd, 0, 4)
                else:
                    # parity mode: the explicit field / class map share the (padded) view's strides
                    def like_view(t, dtype):
                        if t is None:
                            return None
                        if not padded:
                            return t.to(device=x.device, dtype=dtype).contiguous()
                        full = torch.zeros(cur.shape, dtype=dtype, device=x.device)
                        full[..., : spatial[-1]] = t.to(device=x.device, dtype=dtype)
                        return full[..., : spatial[-1]]
                    uv = like_view(u, torch.float32)
                    cv = like_view(cls, torch.int8) if cls is not None else None
                    sd = 0 if u is not None else (
                        seed if seed is not None else int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item()))
                    rt.salt_and_pepper(view, 4, thr, mm, out=view, u=uv, cls=cv, seed=sd)
                    if cls is not None:
                        cls.copy_(cv)
                self._mm_b = B
                self._last_mm = mm
                mm_valid = False
        if cur is x:
            cur = x.clone() if not pad else torch.nn.functional.pad(x, (0, pad))
        elif pad and not padded:
            cur = torch.nn.functional.pad(cur, (0, pad))
        if out is not None and cur is not out:
            if tuple(cur.shape) != tuple(out.shape):  # e.g. a channel-selection stage: no silent broadcast
                raise ValueError(f"the chain's result {tuple(cur.shape)} does not fit out {tuple(out.shape)}")
            out.copy_(cur)
            cur = out
        return cur


def reference_c3_chain(rank: int = 0, seed_base: int = 10):
    """The C3 chain (10_scripts/127_gibbs_spikes_wraparound_sap_OneChannel/
    stylized_gibbs12p5_spikes15_wrap0p5_sap0p05_3modalities.py:171-174): disk r=12.5 -> plane wave on
    the (55, 55, 30) ellipsoid shell, I=15 -> wrap 0.5 -> salt-and-pepper 0.05, with every random
    transform seeded per data-parallel rank (``seed_base * rank + j``; the ellipsoid's own stream
    ``seed_base * rank + 7``), so ranks draw distinct, reproducible streams -- the DataLoader
    workers' independent streams in the reference.  Returns (FusedChain, {name: transform})."""
    import filters_and_operators as F
    disk = F.RandFourierDiskMaskd(keys="image", r=12.5, inside_off=False, prob=1.0)
    planes = F.RandPlaneWaves_ellipsoid("image", 55.0, 55.0, 30.0, intensity_value=15.0, prob=1.0)
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.05)
    for j, t in enumerate((disk, planes, sap)):
        t.set_random_state(seed_base * rank + j)
    planes.ellipsoid.set_random_state(seed_base * rank + 7)
    return FusedChain([disk, planes, wrap, sap]), dict(disk=disk, planes=planes, wrap=wrap, sap=sap)
