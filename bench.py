#!/usr/bin/env python3
"""Headline benchmark: BraTS 4-ch 240x240x155 volumes/s, filter chain + U-Net train step.

One step = one batch of ``--batch`` (default 2, the reference's batch size) synthetic
volumes per GPU, resident in HBM:
  1. host RNG draws of the reference's chain (127_.../..._3modalities.py:171-174):
     RandFourierDiskMaskd(r=12.5) -> RandPlaneWaves_ellipsoid(55,55,30, I=15) ->
     WrapArtifactd(0.5) -> SaltAndPepper(0.05)  (``--random-filters``: per-batch random
     r~U(10,25.1), I~U(10,17), alpha in {0,.25,.5,.75}, p~U(.05,.35) -- BASELINE config 4)
  2. ONE fused k-space pass (3 kernels) writing the U-Net input with D padded 155 -> 160,
     then the sparse salt-and-pepper kernel;
  3. U-Net(4->3) forward, DiceLoss, backward, Adam -- DDP over RCCL when N > 1.
Timing: W warmup steps, then K steps between barrier+synchronize pairs; max over ranks.
Rank 0 prints one JSON line (see README / task contract), with the dominant filter kernel's
HBM roofline (HIP events on the launch stream) and a CPU baseline of the reference's filter
path (the numpy oracle, test infrastructure) on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "medical-vision-textural-bias_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "BraTS 4ch 240^3 vols/sec filtered+train-step @1/2/4/8 GPU; filter HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2, help="volumes per GPU per step")
    ap.add_argument("--shape", type=str, default="240,240,155")
    ap.add_argument("--pad-to", type=int, default=160, help="U-Net D extent (G10: 155 is not /16)")
    ap.add_argument("--random-filters", action="store_true")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--no-cudnn-benchmark", action="store_true",
                    help="skip MIOpen Find (its exhaustive solver search makes the first step slow, the rest fast)")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-vols", type=int, default=1)
    ap.add_argument("--filter-only", action="store_true", help="diagnostic: time the filter chain alone")
    return ap.parse_args()


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r2", "traffic.json")


def pmc_traffic(kernel: str, launch_bytes: int):
    """HBM bytes per launch of a filter kernel from the committed rocprofv3 PMC passes (FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction), or None when not measured for launches of
    this size (the record carries the kernel name and the algorithmic bytes of the launches it measured)."""
    try:
        with open(TRAFFIC_FILE) as f:
            rec = json.load(f)["kernels"].get(kernel)
        if not rec or abs(int(rec.get("algorithmic_bytes_per_launch", -1)) - int(launch_bytes)) > 0.001 * launch_bytes:
            return None
        return int(rec["traffic_bytes"])
    except (OSError, ValueError, KeyError):
        return None


def maybe_launch_ranks(args) -> None:
    """``bench.py --gpus N`` without a torchrun environment: start N ranks (one process per GPU)
    under torch.distributed.run as a CHILD process -- nothing here has touched the GPU -- and exit
    with its status.  Under torchrun (WORLD_SIZE set) this returns and the rank runs."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    sys.exit(subprocess.call(cmd))


def cpu_baseline(x0: np.ndarray, args) -> dict:
    """The reference's CPU filter path restated op for op (oracle/, numpy complex64, 1 thread)."""
    from oracle import filters_oracle as O
    n = max(1, args.cpu_sample_vols)
    rs = np.random.RandomState(0)
    coords = O.ellipsoid_shell(x0.shape[1:], 55.0, 55.0, 30.0)
    t0 = time.perf_counter()
    for _ in range(n):
        idx = O.ellipsoid_sample(coords, rs)
        u = rs.random_sample(x0.shape).astype(np.float32)
        O.chain(x0, 12.5, idx, 15.0, 0.5, 0.05, u)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "vols/s", "cores": 1, "kind": "port",
            "sample": f"{n} volume(s) 4x{'x'.join(map(str, x0.shape[1:]))} through the oracle's op-for-op restatement of "
                      "the reference chain disk(12.5)->planes(55,55,30,I=15)->wrap(0.5)->S&P(0.05) (numpy complex64 "
                      f"FFTs, single thread); filter only, {dt:.1f} s"}


def main():
    args = parse()
    maybe_launch_ranks(args)
    from texbias import runtime as rt
    from texbias.pipeline import FusedChain
    from texbias.synth import brats_labels, brats_like
    from texbias.train import TrainStep, init_distributed, reference_model
    import filters_and_operators as F

    rank, world, local = init_distributed()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} ranks")
    if rank == 0:
        print(f"[bench] world size {world} (backend {dist.get_backend() if world > 1 else 'none'})",
              file=sys.stderr, flush=True)
    dev = torch.device("cuda", local)
    H, W, D = (int(v) for v in args.shape.split(","))
    B, C = args.batch, 4
    pad = max(0, args.pad_to - D)
    torch.manual_seed(1000 + rank)

    # resident synthetic data: two distinct batches per rank, labels pre-padded
    pool = [brats_like(B, C, (H, W, D), seed=rank * 97 + i, device=dev) for i in range(2)]
    labels = [brats_labels(B, (H, W, D), seed=rank * 97 + i, device=dev, pad_to=D + pad) for i in range(2)]

    disk = F.RandFourierDiskMaskd(keys="image", r=12.5, inside_off=False, prob=1.0)
    planes = F.RandPlaneWaves_ellipsoid("image", 55.0, 55.0, 30.0, intensity_value=15.0, prob=1.0)
    wrap = F.WrapArtifactd("image", 0.5)
    sap = F.SaltAndPepper(0.05)
    for j, t in enumerate((disk, planes, sap)):
        t.set_random_state(10 * rank + j)
    planes.ellipsoid.set_random_state(10 * rank + 7)
    chain = FusedChain([disk, planes, wrap, sap])
    prs = np.random.RandomState(12345 + rank)

    def randomize_filters():
        disk.r = float(prs.uniform(10.0, 25.1))
        planes.intensity_value = float(prs.uniform(10.0, 17.0))
        wrap.transform.alpha = float(prs.choice([0.0, 0.25, 0.5, 0.75]))
        sap.p = float(prs.uniform(0.05, 0.35))

    step_fn = None
    if not args.filter_only:
        torch.backends.cudnn.benchmark = not args.no_cudnn_benchmark
        step_fn = TrainStep(reference_model(C, 3), dev, distributed=world > 1, bucket_cap_mb=args.bucket_mb,
                            channels_last=args.channels_last)

    def one_step(i):
        if args.random_filters:
            randomize_filters()
        y = chain(pool[i % 2], pad=pad)
        if step_fn is not None:
            return step_fn(y, labels[i % 2])
        return y

    for i in range(args.warmup):
        t_w = time.perf_counter()
        one_step(i)
        torch.cuda.synchronize(dev)
        if rank == 0:
            print(f"[bench] warmup step {i}: {time.perf_counter() - t_w:.3f} s", file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    rt.set_pass_timing(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        last = one_step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms, cnt, nbytes, kernels = rt.pass_stats()
    rt.set_pass_timing(False)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    if rank == 0:
        vols = B * world * args.steps
        names = ["forward", "kspace", "inverse", "salt_pepper"]
        passes = {}
        for i, nm in enumerate(names):
            if cnt[i]:
                avg = ms[i] / cnt[i]
                passes[nm] = {"kernel": kernels[i], "avg_ms": round(avg, 4), "launches": cnt[i]}
                if nbytes[i] > 0:
                    per_launch = nbytes[i] / cnt[i]
                    passes[nm]["algorithmic_bytes"] = int(round(per_launch))
                    passes[nm]["algorithmic_MB"] = round(per_launch / 1e6, 2)
                    passes[nm]["GB_s"] = round(per_launch / (avg * 1e-3) / 1e9, 1)
        # the dominant (longest) k-space pass, its bytes and time both measured live on its stream
        dom = max((n for n in names[:3] if n in passes and "GB_s" in passes[n]), key=lambda n: passes[n]["avg_ms"])
        ach = passes[dom]["GB_s"]
        dom_bytes = passes[dom]["algorithmic_bytes"]
        line = {
            "metric": METRIC,
            "value": round(vols / elapsed, 4),
            "unit": "vols/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic BraTS-like z-scored 4-ch volumes resident in HBM; random-init U-Net",
            "config": {
                "workload": ("C3 full filter chain (disk 12.5 -> plane wave (55,55,30) I=15 -> wrap 0.5 -> S&P 0.05) "
                             "+ 3D U-Net(4->3, 16..256, 2 res units) fwd/bwd/Adam(amsgrad), DiceLoss")
                            + (" [random per-batch filter params, config 4]" if args.random_filters else "")
                            + (" [FILTER ONLY diagnostic]" if args.filter_only else ""),
                "volume": [C, H, W, D],
                "unet_input": [B, C, H, W, D + pad],
                "per_gpu_batch": B,
                "global_batch": B * world,
                "parallelism": f"dp{world}",
            },
            "roofline": {"kernel": passes[dom]["kernel"], "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(passes[dom]["kernel"], dom_bytes),
                         "traffic_unit": "bytes per launch (rocprofv3 PMC, profiles/r2/traffic.json)",
                         "algorithmic_bytes_per_launch": dom_bytes},
            "filter_passes": passes,
            "filter_ms_per_step": round(sum(ms) / args.steps, 4),
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(pool[0][0].cpu().numpy(), args)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
