"""Evaluation harness (texbias.evaluation.ModelEvaluation, utils.py:241-465) on the GPU: the fused
thresholded Dice statistics equal a plain torch restatement of Activations(sigmoid) +
AsDiscrete(0.5) + DiceMetric (counts are integers: exact), and the per-batch weighted averages
of dataset_eval_multi match the reference loop restated in torch (1e-12)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_meandice(logits, y):
    p = (torch.sigmoid(logits) >= 0.5).float()
    ax = tuple(range(2, p.dim()))
    inter = (p * y).sum(ax).double()
    yo, po = y.sum(ax).double(), p.sum(ax).double()
    f = torch.where(yo > 0, 2 * inter / (yo + po), torch.full_like(yo, float("nan")))
    ok = ~torch.isnan(f)
    n = int(ok.sum())
    return (float(torch.nan_to_num(f, nan=0.0).sum()) / n if n else 0.0), n


def test_metric_sums_exact(gpu):
    from texbias.evaluation import dice_from_sums, dice_metric_sums
    torch.manual_seed(0)
    x = torch.randn((3, 3, 20, 18, 16), device="cuda")
    y = (torch.rand_like(x) > 0.7).float()
    y[1, 2] = 0.0  # an empty ground truth: NaN entry
    s = dice_metric_sums(x, y)
    p = (torch.sigmoid(x) >= 0.5).float()
    ref = torch.stack([(p * y).sum((2, 3, 4)), y.sum((2, 3, 4)), p.sum((2, 3, 4))], -1).double()
    assert torch.equal(s, ref)
    d = dice_from_sums(s)
    assert torch.isnan(d[1, 2]) and torch.isfinite(d[0]).all()


def test_dataset_eval_multi_matches_reference_loop(gpu, tmp_path):
    from texbias.evaluation import ModelEvaluation
    from texbias.train import reference_model
    torch.manual_seed(1)
    model = reference_model(4, 3).cuda()
    batches = []
    for i in range(3):
        x = torch.randn((2, 4, 32, 32, 32))
        y = (torch.rand((2, 3, 32, 32, 32)) > 0.8).float()
        if i == 1:
            y[0, 2] = 0.0
        batches.append({"image": x, "label": y})
    ev = ModelEvaluation(model=model, instance_name="t")
    got = ev.dataset_eval_multi(batches)
    # the reference loop (utils.py:373-411), restated in torch
    sums, cnts = [0.0] * 4, [0] * 4
    model.eval()
    with torch.no_grad():
        for b in batches:
            out = model(b["image"].cuda())
            lab = b["label"].cuda()
            for k, (o, l) in enumerate([(out, lab)] + [(out[:, c:c + 1], lab[:, c:c + 1]) for c in range(3)]):
                v, n = _torch_meandice(o, l)
                sums[k] += v * n
                cnts[k] += n
    mean, tc, wt, et = (s / c for s, c in zip(sums, cnts))
    np.testing.assert_allclose(got, (mean, et, tc, wt), rtol=1e-12, atol=1e-12)
    assert abs(ev.dataset_eval_single(batches) - mean) < 1e-12
    ev.add_eval("gibbs", batches, {"r": 12.5})
    f = ev.save(str(tmp_path / "ev.json"))
    ev2 = ModelEvaluation()
    ev2.load_dict(f)
    assert ev2.eval_dict == ev.eval_dict


def _raw_cases(n, sp, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        img = (rng.standard_normal((4,) + sp) * 2.0 + 1.0).astype(np.float32)
        img[:, :2] = 0.0                                   # background slab
        lab = rng.integers(0, 4, size=sp).astype(np.float32)
        out.append((img, lab, np.diag([-1.0, -1.0, 1.0, 1.0])))
    return out


def test_brats_val_iter_dataset_disk_matches_oracle(gpu):
    """utils.py:159-235: the fixed split's test half through Spacing -> Orientation(RAS) ->
    CenterSpatialCrop -> NormalizeIntensity -> the named filter, on the device; the disk filter's
    output against the oracle chain (1e-5), labels exact; loaders batch 2, unshuffled."""
    import filters_and_operators as F
    from oracle import filters_oracle as O
    from oracle import prep_oracle as PO
    from texbias.evaluation import BratsValIterDataset, ModelEvaluation
    from texbias.train import reference_model
    sp, roi = (40, 36, 30), (16, 16, 16)
    src = _raw_cases(8, sp, 4)
    tr = {"disk": F.RandFourierDiskMaskd(keys="image", r=5.5, inside_off=False, prob=1.0),
          "sap": F.SaltAndPepper(0.1)}
    ds = BratsValIterDataset(src, tr, return_loader=True, split=(4, 4), roi=roi)
    names = []
    for name, loader in ds:
        names.append(name)
        batches = list(loader)
        assert [b["image"].shape[0] for b in batches] == [2, 2]
        for bi, b in enumerate(batches):
            for j in range(2):
                img, lab, aff = src[ds.test_indices[2 * bi + j]]
                shp = PO.spacing_orientation(img, aff, (1.5, 1.5, 2.0)).shape[1:]
                corner = tuple(n // 2 - r // 2 for n, r in zip(shp, roi))   # CenterSpatialCrop
                xr, yr = PO.prep_resampled(img, lab, aff, (1.5, 1.5, 2.0), corner, roi)
                np.testing.assert_array_equal(b["label"][j].cpu().numpy(), yr)
                got = b["image"][j].cpu().numpy()
                if name == "disk":
                    ref = O.fourier_disk(xr, 5.5)
                    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-5
                else:   # salt and pepper: every voxel kept or set to the sample's min/2 or max/2
                    tol = 1e-5 * np.abs(xr).max()
                    keep = np.abs(got - xr) <= tol
                    lo, hi = xr.min() / 2, xr.max() / 2
                    salt = np.abs(got - lo) <= tol
                    pepper = np.abs(got - hi) <= tol
                    assert np.all(keep | salt | pepper) and 0.8 < keep.mean() < 0.97
                    assert len(np.unique(got[~keep])) <= 2   # the two sample-wide values only
    assert names == ["disk", "sap"]
    # the per-sample view and the evaluation harness on a named set
    one = BratsValIterDataset(src, tr, split=(4, 4), roi=roi)["disk"]
    assert len(one) == 4 and one[0]["image"].shape == (4,) + roi
    ev = ModelEvaluation(model=reference_model(4, 3), instance_name="val")
    ev.add_eval("disk", ds["disk"])
    assert set(ev.eval_dict["disk"]) == {"mean", "et", "tc", "wt"}


def test_load_gibbs_and_spikes_unet(gpu, tmp_path):
    """ModelEvaluation(model_path, gibbs_unet=True / spikes_unet=True) loads like utils.py:286-297;
    a reference-style Gibbs_UNet state dict (no alpha entry) loads with alpha 0.5."""
    import stylization_layers as SL
    from texbias.evaluation import ModelEvaluation
    torch.manual_seed(0)
    g = SL.Gibbs_UNet()
    sd = {k: v for k, v in g.state_dict().items() if k != "gibbs.alpha"}
    torch.save(sd, tmp_path / "g.pth")
    ev = ModelEvaluation(str(tmp_path / "g.pth"), gibbs_unet=True, in_channels=1, out_channels=1)
    assert isinstance(ev.model, SL.Gibbs_UNet) and float(ev.model.gibbs.alpha) == 0.5
    for k, v in sd.items():
        assert torch.equal(ev.model.state_dict()[k].cpu(), v.cpu()), k
    s = SL.Spikes_UNet()
    torch.save(s.state_dict(), tmp_path / "s.pth")
    ev2 = ModelEvaluation(str(tmp_path / "s.pth"), spikes_unet=True, in_channels=1, out_channels=1)
    assert isinstance(ev2.model, SL.Spikes_UNet)
