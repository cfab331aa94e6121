"""The data-parallel train step over torch.distributed (gloo on CPU, world size 2): replicas start
identical, all-reduced gradients keep them identical after optimizer steps on different data."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    from texbias.train import TrainStep, init_distributed, reference_model
    torch.set_num_threads(1)
    init_distributed("gloo")
    torch.manual_seed(0)                      # identical init on every rank
    model = reference_model(4, 3)
    step = TrainStep(model, torch.device("cpu"), distributed=True, bucket_cap_mb=0.5)
    g = torch.Generator().manual_seed(100 + rank)   # different data per rank
    for _ in range(2):
        x = torch.randn((1, 4, 32, 32, 32), generator=g)
        lab = (torch.rand((1, 3, 32, 32, 32), generator=g) > 0.7).float()
        step(x, lab)
    flat = torch.cat([p.detach().reshape(-1) for p in step.module.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        out.put(float((gathered[0] - gathered[1]).abs().max()))
        out.put(float((gathered[0] - torch.cat([p.detach().reshape(-1) for p in reference_model(4, 3).parameters()])).abs().max()))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_two_ranks_stay_in_sync():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs)
    diff, moved = q.get(timeout=5), q.get(timeout=5)
    assert diff == 0.0          # replicas bit-identical
    assert moved > 0.0          # and they actually trained
