"""Data-parallel train step WITH the HIP backward kernels in the loop (DESIGN (e)).

Two ranks share cuda:0 (spawned child processes, each initialising the GPU itself), process group over
gloo (the RCCL path cannot put two ranks on one device; DDP's bucketing, static graph and
``gradient_as_bucket_view`` -- texbias/train.py:55-68 -- are the same code either way).  Every rank runs
BASELINE config 4's workload at the reference drivers' crop size (2 x 4 x 128 x 128 x 64,
…_3modalities.py:163-165,231): its own ``reference_c3_chain(rank)`` with bench.py's per-batch random
filter draws (r, I, wrap alpha, S&P p) on its own batch, then ``TrainStep(distributed=True)`` on the
reference U-Net(4 -> 3) with the texbias conv / InstanceNorm+PReLU / Dice kernels.  Checked:
  * the ranks' filter draws differ, and every non-transposed 3x3x3 convolution routed to a texbias
    kernel (no ``aten`` route), with the direct kernels' weight gradients on texbias too;
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
SHAPE = (128, 128, 64)


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
    import numpy as np
    from texbias.pipeline import reference_c3_chain
    torch.manual_seed(0)
    step = TrainStep(reference_model(4, 3), dev, distributed=True)
    x_raw, lab = _batch(rank, dev)
    chain, tr = reference_c3_chain(rank)
    prs = np.random.RandomState(12345 + rank)
    draws = []

    def filtered():  # bench.py randomize_filters(), then the fused chain on this rank's batch
        tr["disk"].r = float(prs.uniform(10.0, 25.1))
        tr["planes"].intensity_value = float(prs.uniform(10.0, 17.0))
        tr["wrap"].transform.alpha = float(prs.choice([0.0, 0.25, 0.5, 0.75]))
        tr["sap"].p = float(prs.uniform(0.05, 0.35))
        draws.append((tr["disk"].r, tr["planes"].intensity_value, tr["wrap"].transform.alpha, tr["sap"].p))
        return chain(x_raw)

    x = filtered()
    # step 1 by hand to capture the averaged gradients before the optimizer moves the weights
    step.opt.zero_grad(set_to_none=True)
    loss = step.loss_fn(step.model(x), lab)
    loss.backward()
    grads = [p.grad.detach().clone().cpu() for p in step.module.parameters()]
    step.opt.step()
    x1st = x.cpu()
    for _ in range(2):
        step(filtered(), lab)
    torch.cuda.synchronize()
    routes = [(key[1] if key[0] == "stacked" else key[0], r.k, r.transposed, r.kind, r.dx, r.fast_w)
              for m in step.module.modules()
              for key, r in m.__dict__.get("_tb_routes", {}).items()]
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
    torch.save({"grads": grads, "params": params, "adam": adam, "alpha": alpha, "x": x1st, "draws": draws,
                "routes": routes},
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
    # C4: each rank drew its own filters and filtered its own batch
    assert r0["draws"] != r1["draws"] and len(r0["draws"]) == 3
    assert not torch.equal(r0["x"], r1["x"])
    # the HIP kernels ran: no non-transposed 3x3x3 convolution on ATen; the top two resolutions' weight
    # gradients on the texbias MFMA kernels
    print("routes:", r0["routes"])
    assert r0["routes"] and r0["routes"] == r1["routes"]
    conv3 = [r for r in r0["routes"] if r[1] == 3 and not r[2]]
    assert conv3 and all(r[3] != "aten" for r in conv3), conv3
    # the direct / z-march kernels take their layers' weight gradients too (the stacked stride-2 and
    # transposed GEMM-route layers keep MIOpen's, as in the C3 step)
    direct = [r for r in r0["routes"] if r[3] in ("fwd16", "mfma", "small", "fewin", "fewout")]
    assert direct and all(r[5] for r in direct), direct
    kinds = {(r[0][1:], r[2]): r[3] for r in r0["routes"]}
    assert kinds[((4,) + SHAPE, False)] == "fewin" and kinds[((3,) + SHAPE, False)] == "small"
    assert kinds[((16,) + tuple(n // 2 for n in SHAPE), False)] in ("fwd16", "gemm")
    # the averaged first-step gradients == one process's batch-of-4 step on the ranks' filtered batches
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    single = TrainStep(reference_model(4, 3), dev)
    _, l0 = _batch(0, dev)
    _, l1 = _batch(1, dev)
    x0, x1 = r0["x"].to(dev), r1["x"].to(dev)
    single.opt.zero_grad(set_to_none=True)
    loss = single.loss_fn(single.model(torch.cat([x0, x1])), torch.cat([l0, l1]))
    loss.backward()
    g4 = [p.grad.detach().cpu() for p in single.module.parameters()]
    scale = max(g.abs().max().item() for g in g4)
    for a, b in zip(r0["grads"], g4):
        err = (a.double() - b.double()).abs().max().item()
        # + floor: tensors whose true gradient is exactly zero (conv biases in front of an InstanceNorm) hold
        # float32 rounding sums whose order differs between the two runs -- up to ~5e-6 of the largest
        # gradient at 2 x 4 x 128 x 128 x 64
        assert err <= 2e-3 * b.abs().max().item() + 1e-5 * scale, (err, b.abs().max().item(), scale)
    # gibbs_gd: one alpha on every replica, moved from 0.7
    assert torch.equal(r0["alpha"], r1["alpha"])
    assert abs(r0["alpha"].item() - 0.7) > 0.0
