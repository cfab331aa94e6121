"""Strided residual units keep [unit0; residual] weights in one storage only after the explicit
``pack_parameters`` setup (TrainStep calls it); ``forward`` never rebinds parameter data, so an
inference-mode forward, ``torch.func.functional_call`` and saving all see plain parameters."""
import io

import pytest
import torch

from texbias.train import TrainStep, reference_model
from texbias.unet import ResidualUnit, _adjacent, pack_parameters


def _strided_pairs(model):
    for m in model.modules():
        if isinstance(m, ResidualUnit) and isinstance(m.residual, torch.nn.Conv3d):
            u0 = list(m.conv.children())[0].conv
            if m.residual.stride == u0.stride and m.residual.kernel_size == u0.kernel_size:
                yield u0, m.residual


def _ptrs(model):
    return [p.data_ptr() for p in model.parameters()]


def test_forward_does_not_rebind_and_pack_is_explicit():
    torch.manual_seed(0)
    model = reference_model(4, 3)
    before = _ptrs(model)
    x = torch.randn(1, 4, 32, 32, 32)
    with torch.inference_mode():
        model(x)
    assert _ptrs(model) == before
    with torch.inference_mode():
        assert pack_parameters(model) == 0          # skipped under inference mode
    assert _ptrs(model) == before
    ref = {k: v.clone() for k, v in model.state_dict().items()}
    n = pack_parameters(model)
    assert n == sum(1 for _ in _strided_pairs(model)) and n > 0
    for u0, r in _strided_pairs(model):
        assert _adjacent(u0.weight, r.weight) is not None
        assert _adjacent(u0.bias, r.bias) is not None
    for k, v in model.state_dict().items():             # values unchanged by packing
        assert torch.equal(v, ref[k])
    assert pack_parameters(model) == n and _ptrs(model) == _ptrs(model)  # idempotent
    buf = io.BytesIO()
    torch.save(model.state_dict(), buf)
    buf.seek(0)
    sd = torch.load(buf, weights_only=True)
    assert all(torch.equal(sd[k], ref[k]) for k in ref)


def test_packed_model_saves_with_safetensors(tmp_path):
    st = pytest.importorskip("safetensors.torch")
    torch.manual_seed(0)
    model = reference_model(4, 3)
    pack_parameters(model)
    path = str(tmp_path / "m.safetensors")
    st.save_model(model, path)
    fresh = reference_model(4, 3)
    st.load_model(fresh, path)
    for (k, a), b in zip(model.state_dict().items(), fresh.state_dict().values()):
        assert torch.equal(a, b), k


def test_functional_call_leaves_caller_tensors_alone():
    torch.manual_seed(0)
    model = reference_model(4, 3)
    params = {k: v.clone() for k, v in model.named_parameters()}
    ptrs = {k: v.data_ptr() for k, v in params.items()}
    torch.func.functional_call(model, params, (torch.randn(1, 4, 32, 32, 32),))
    assert {k: v.data_ptr() for k, v in params.items()} == ptrs


@pytest.mark.gpu
def test_inference_forward_then_train_and_save(gpu):
    """The fused HIP path: an inference-mode forward before any packing (unpacked weights are
    concatenated per call), then TrainStep packs, trains two steps and the model saves."""
    torch.manual_seed(0)
    model = reference_model(4, 3).to(gpu)
    x = torch.randn(2, 4, 32, 32, 32, device=gpu)
    y = (torch.rand(2, 3, 32, 32, 32, device=gpu) > 0.5).float()
    with torch.inference_mode():
        out0 = model(x)
    ts = TrainStep(model, gpu)
    for u0, r in _strided_pairs(model):
        assert _adjacent(u0.weight, r.weight) is not None
    with torch.no_grad():
        out1 = model(x)
    torch.testing.assert_close(out1, out0, rtol=1e-5, atol=1e-5)  # packing changed no values
    l0 = ts(x, y)
    l1 = ts(x, y)
    assert torch.isfinite(l0) and torch.isfinite(l1)
    buf = io.BytesIO()
    torch.save(model.state_dict(), buf)
    st = pytest.importorskip("safetensors.torch")
    blob = st.save(dict((k, v.detach().clone()) for k, v in model.state_dict().items()))
    assert len(blob) > 0
