"""Filters launched from two streams at once (per-(device, stream) workspaces, texbias/runtime.py):
the band route (whose passes keep an arrival counter and min/max partials in the workspace) and the
closed-form route on two side streams, overlapping, equal the same calls made one after the other."""
import pytest
import torch

from texbias import kprog as K

pytestmark = pytest.mark.gpu


def test_two_streams_band_and_point(gpu):
    from texbias import runtime as rt
    torch.manual_seed(21)
    shape = (2, 4, 64, 60, 31)
    sp = shape[2:]
    xs = [torch.randn(shape, device="cuda") for _ in range(4)]
    band = [[K.disk_op(7.5, False), K.wrap_op(0.5)]] * 2
    point = [[K.spike_op((40, 9, 20), K.geometry(sp), 11.0)]] * 2
    progs = [band, point, band, point]
    ref = []
    for x, p in zip(xs, progs):
        mm = torch.empty((2, 2), dtype=torch.int32, device="cuda")
        ref.append((rt.kspace_filter(x, 3, p, 4, pad=1, minmax=mm), mm))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    got = [None] * 4
    for rep in range(3):  # several rounds so the two streams' launches interleave on the device
        for i, (x, p) in enumerate(zip(xs, progs)):
            with torch.cuda.stream(streams[i % 2]):
                mm = torch.empty((2, 2), dtype=torch.int32, device="cuda")
                got[i] = (rt.kspace_filter(x, 3, p, 4, pad=1, minmax=mm), mm)
    torch.cuda.synchronize()
    for (y, mm), (yr, mmr) in zip(got, ref):
        torch.testing.assert_close(y, yr, rtol=0, atol=0)
        assert torch.equal(mm, mmr)
