"""DataLoader(num_workers=4) with the reference's Compose order (127_.../..._3modalities.py:171-175:
disk -> plane wave -> wrap -> salt-and-pepper -> MultimodalSlicesd): the workers defer, the batches
run on the GPU (texbias.deferred.DeferredLoader), and every sample equals the eager per-sample
result of the same transforms replayed in the main process (same draws, same Philox keys).

Tolerance: max|y - y_eager| / max|y_eager| <= 1e-6 (batched vs single-sample launches sum the band
spectrum in a different grouping); the salt-and-pepper positions are identical (a mismatch would be
an error of the order of max|y|); labels bit-exact."""
import pytest
import torch

from _deferred_case import DictSet, emulate, make_transforms, worker_seed

pytestmark = pytest.mark.gpu


def test_deferred_loader_matches_eager(gpu):
    from texbias.deferred import DeferredLoader, deferred_collate
    ts = make_transforms()
    loader = torch.utils.data.DataLoader(DictSet(ts), batch_size=2, num_workers=4, collate_fn=deferred_collate,
                                         worker_init_fn=worker_seed)
    got = {}
    for bi, batch in enumerate(DeferredLoader(loader, torch.device("cuda"))):
        assert "image_texbias_plan" not in batch and batch["image"].is_cuda
        assert batch["image"].shape == (2, 1, 24, 20, 16)
        for j in range(2):
            got[2 * bi + j] = (batch["image"][j].cpu(), batch["label"][j])

    def eager(d):   # in the main process the transforms compute at once (no deferral)
        return d["image"].cpu(), d["label"]

    ref = emulate(make_transforms(), 4, 2, eager)
    for i in range(len(ref)):
        y, lab = got[i]
        yr, labr = ref[i]
        assert y.shape == yr.shape == (1, 24, 20, 16)
        assert torch.equal(lab, labr)
        err = (y - yr).abs().max().item() / yr.abs().max().item()
        assert err <= 1e-6, (i, err)
