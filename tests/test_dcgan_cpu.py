"""DCGAN (BASELINE config 5) on CPU: the networks reproduce the reference's outputs for the same
seed (golden vectors from 50_reconstruction/networks.py, tests/golden/make_golden_dcgan.py), the
full-size parameter counts match, the reference iteration runs, and the data-parallel form keeps
two gloo replicas identical."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from texbias import dcgan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "golden_dcgan.npz")


def test_networks_match_reference_vectors():
    g = np.load(GOLD, allow_pickle=False)
    torch.manual_seed(7)
    G = dcgan.Generator(nz=100, ngf=16, nc=1)
    D = dcgan.Discriminator(nc=1, ndf=16)
    G.apply(dcgan.weights_init)
    D.apply(dcgan.weights_init)
    with torch.no_grad():
        go = G(torch.from_numpy(g["z"])).numpy()
        do = D(torch.from_numpy(g["x"])).numpy()
    np.testing.assert_allclose(go, g["g_out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(do, g["d_out"], rtol=1e-5, atol=1e-6)
    assert sum(p.numel() for p in dcgan.Generator().parameters()) == int(g["n_params_g_full"])
    assert sum(p.numel() for p in dcgan.Discriminator().parameters()) == int(g["n_params_d_full"])


def test_step_runs_and_learns_on_cpu():
    torch.manual_seed(0)
    step = dcgan.DCGANStep(torch.device("cpu"), ngf=8, ndf=8, bf16=False)
    real = torch.tanh(torch.randn(4, 1, 128, 128))
    p0 = [p.detach().clone() for p in step.G_module.parameters()]
    errD, errG, dx, dgz1, dgz2 = step(real)
    assert all(torch.isfinite(t).item() for t in (errD, errG, dx, dgz1, dgz2))
    assert any(not torch.equal(a, b) for a, b in zip(p0, step.G_module.parameters()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "medical-vision-textural-bias_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from texbias import dcgan as DG
    from texbias.train import init_distributed
    torch.set_num_threads(1)
    init_distributed("gloo")
    torch.manual_seed(0)                     # identical init on every rank
    step = DG.DCGANStep(torch.device("cpu"), ngf=8, ndf=8, bf16=False, distributed=True)
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(2):
        real = torch.tanh(torch.randn(4, 1, 128, 128, generator=g))
        noise = torch.randn(4, 100, 1, 1, generator=g)
        step(real, noise)
    flat = torch.cat([p.detach().reshape(-1) for m in (step.G_module, step.D_module) for p in m.parameters()])
    got = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(got, flat)
    if rank == 0:
        out.put(float((got[0] - got[1]).abs().max()))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dcgan_ddp_two_ranks_stay_in_sync():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
    assert all(p.exitcode == 0 for p in ps)
    assert q.get(timeout=5) == 0.0
