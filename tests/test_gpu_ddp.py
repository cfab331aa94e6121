"""Data-parallel train step WITH the HIP backward kernels in the loop (DESIGN (e)).

Two ranks share cuda:0 (spawned child processes, each initialising the GPU itself), process group over
gloo (the RCCL path cannot put two ranks on one device; DDP's bucketing, static graph and
``gradient_as_bucket_view`` -- texbias/train.py:55-68 -- are the same code either way).  Every rank runs
``TrainStep(distributed=True)`` on the reference U-Net(4 -> 3) with the texbias conv / InstanceNorm+PReLU /
Dice kernels, its own batch of 2.  Checked:
  * after 3 steps the replicas are bit-identical (every parameter and Adam state);
  * the first step's averaged gradients equal ONE process's batch-of-4 step (the two ranks' batches
    concatenated) -- the whole-step bar of tests/test_gpu_norm.py (per tensor, vs the largest gradient
    scale: conv biases in front of an InstanceNorm have an exactly-zero true gradient);
  * ``gibbs_gd`` (the Gibbs layer driver's finite-difference alpha step) leaves alpha identical on both ranks.
"""
import os
import socket
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "medical-vision-textural-bias_amd")
SHAPE = (32, 32, 32)


def _batch(rank: int, dev):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn((2, 4) + SHAPE, generator=g)
    lab = (torch.rand((2, 3) + SHAPE, generator=g) > 0.8).float()
    return x.to(dev), lab.to(dev)


def _rank_main(rank: int, world: int, port: int, out_dir: str):
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch.distributed as dist

    import stylization_layers as SL
    from texbias.losses import DiceLoss
    from texbias.train import TrainStep, gibbs_gd, reference_model
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    step = TrainStep(reference_model(4, 3), dev, distributed=True)
    x, lab = _batch(rank, dev)
    # step 1 by hand to capture the averaged gradients before the optimizer moves the weights
    step.opt.zero_grad(set_to_none=True)
    loss = step.loss_fn(step.model(x), lab)
    loss.backward()
    grads = [p.grad.detach().clone().cpu() for p in step.module.parameters()]
    step.opt.step()
    for _ in range(2):
        step(x, lab)
    torch.cuda.synchronize()
    params = [p.detach().cpu() for p in step.module.parameters()]
    st = step.opt.state_dict()["state"]
    adam = [(v["exp_avg"].cpu(), v["exp_avg_sq"].cpu(), v["max_exp_avg_sq"].cpu()) for v in st.values()]
    # the Gibbs layer driver: a DDP Gibbs_UNet, one train step and one gibbs_gd alpha update
    torch.manual_seed(0)
    gm = SL.Gibbs_UNet()
    gm.gibbs.alpha.fill_(0.7)
    gstep = TrainStep(gm, dev, distributed=True)
    x1 = x[:, :1].contiguous()
    l1 = lab[:, :1].contiguous()
    gstep(x1, l1)
    gibbs_gd(x1, l1, gstep.model, DiceLoss(sigmoid=True, squared_pred=True))
    torch.cuda.synchronize()
    alpha = gm.gibbs.alpha.detach().cpu().clone()
    torch.save({"grads": grads, "params": params, "adam": adam, "alpha": alpha},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_ddp_two_ranks_hip_kernels(gpu, heartbeat):
    import torch.multiprocessing as mp
    sys.path[:0] = [PKG, ROOT]
    from texbias.train import TrainStep, reference_model
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    with tempfile.TemporaryDirectory() as td:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_rank_main, args=(r, 2, port, td)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=540)
        codes = [p.exitcode for p in procs]
        for p in procs:
            if p.is_alive():
                p.kill()
        assert codes == [0, 0], f"rank exit codes {codes}"
        r0 = torch.load(os.path.join(td, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(td, "rank1.pt"), weights_only=True)
    # replicas bit-identical after 3 steps (parameters and Adam moments)
    for a, b in zip(r0["params"], r1["params"]):
        assert torch.equal(a, b)
    for ta, tb in zip(r0["adam"], r1["adam"]):
        for a, b in zip(ta, tb):
            assert torch.equal(a, b)
    for a, b in zip(r0["grads"], r1["grads"]):
        assert torch.equal(a, b)
    # the averaged first-step gradients == one process's batch-of-4 step
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    single = TrainStep(reference_model(4, 3), dev)
    x0, l0 = _batch(0, dev)
    x1, l1 = _batch(1, dev)
    single.opt.zero_grad(set_to_none=True)
    loss = single.loss_fn(single.model(torch.cat([x0, x1])), torch.cat([l0, l1]))
    loss.backward()
    g4 = [p.grad.detach().cpu() for p in single.module.parameters()]
    scale = max(g.abs().max().item() for g in g4)
    for a, b in zip(r0["grads"], g4):
        err = (a.double() - b.double()).abs().max().item()
        assert err <= 2e-3 * max(b.abs().max().item(), 1e-4 * scale), (err, b.abs().max().item())
    # gibbs_gd: one alpha on every replica, moved from 0.7
    assert torch.equal(r0["alpha"], r1["alpha"])
    assert abs(r0["alpha"].item() - 0.7) > 0.0
