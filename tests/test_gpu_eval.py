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
