"""CPU checks of the custom-operator boundary (texbias/ops.py): the op-program records survive the
uint8 tensor round trip byte for byte, and the ops trace under fake tensors (what torch.compile /
torch.export see) with the right output shapes -- no GPU needed, no kernel launched."""
import ctypes as C

import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from texbias import kprog as K
from texbias import ops


def _progs():
    geo = K.geometry((32, 30, 16))
    return [[K.disk_op(12.5, False), K.spike_op((3, 4, 5), geo, 9.0, phase=0.25, chan=1), K.wrap_op(0.5)],
            [K.gibbs_op(0.7, (32, 30, 16))], []]


def test_program_records_round_trip():
    progs = _progs()
    t = ops.pack_programs(progs)
    assert t.dtype == torch.uint8 and t.shape == (3, 304)
    recs = ops.unpack_programs(t)
    assert [r.n for r in recs] == [3, 1, 0]
    for r, p in zip(recs, progs):
        for j, op in enumerate(p):
            assert bytes(r.op[j]) == bytes(op)
            assert C.sizeof(r.op[j]) == 48


def test_fake_tensor_shapes_and_trace():
    progs = ops.pack_programs(_progs()[:2])
    thr = torch.tensor([[0.025, 0.05]] * 2)

    def f(x):
        y, mm = torch.ops.texbias.kspace_filter(x, 3, progs, 4, 5)
        torch.ops.texbias.salt_and_pepper_(y[..., :16], mm, thr, 1, 0, 4)
        return y

    with FakeTensorMode(allow_non_fake_inputs=True):
        x = torch.empty((2, 4, 32, 30, 16), device="cuda")
        y, mm = torch.ops.texbias.kspace_filter(x, 3, progs, 4, 5)
        assert y.shape == (2, 4, 32, 30, 21) and y.device.type == "cuda"
        assert mm.shape == (2, 2) and mm.dtype == torch.int32
        a = torch.empty((1,), device="cuda")
        img = torch.empty((2, 1, 8, 8, 4), device="cuda")
        assert torch.ops.texbias.gibbs_layer(img, a).shape == img.shape
        gm = torch.fx.experimental.proxy_tensor.make_fx(f, tracing_mode="fake")(x)
    targets = [n.target for n in gm.graph.nodes if n.op == "call_function"]
    assert torch.ops.texbias.kspace_filter.default in targets
    assert torch.ops.texbias.salt_and_pepper_.default in targets
