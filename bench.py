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

# MIOpen's find-db / perf-db (seeded in the tree: miopen_db/, gfx950 + this image's MIOpen) and its
# compiled-kernel cache: MIOpen's Find (cudnn.benchmark) then runs once per cache, not once per process
# and rank (first step 12.9 s cold -> 0.8 s seeded; texbias/__init__ also keeps MIOpen's naive solvers out
# of Find, which was 140 s).  Set before torch initialises MIOpen; TEXBIAS_MIOPEN_DIR overrides, an
# existing MIOPEN_* setting wins.
_MIOPEN_DIR = os.environ.get("TEXBIAS_MIOPEN_DIR", os.path.join(ROOT, "miopen_db"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", _MIOPEN_DIR)
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_MIOPEN_DIR, "kcache"))

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
    ap.add_argument("--config", choices=("c3", "c2", "c5"), default="c3",
                    help="c3: full filter chain + U-Net train step on 4x240x240x155 (the headline); "
                         "c2: Gibbs truncation (disk low-pass r=12.5) alone on 4x128x128x128 (BASELINE config 2); "
                         "c5: DCGAN step on filtered 1x128x128 BraTS slices, bf16 (BASELINE config 5)")
    ap.add_argument("--batch", type=int, default=None, help="volumes (c5: slices) per GPU per step (c3: 2, c2: 16, c5: 64)")
    ap.add_argument("--fp32", action="store_true", help="c5: run the networks in fp32 instead of bf16 autocast")
    ap.add_argument("--shape", type=str, default=None, help="c3: 240,240,155; c2: 128,128,128")
    ap.add_argument("--pad-to", type=int, default=None, help="U-Net D extent (c3: 160, G10: 155 is not /16)")
    ap.add_argument("--random-filters", action="store_true")
    ap.add_argument("--chain", choices=("ref", "planes", "wrap", "gibbs-aug", "spikes-aug"), default="ref",
                    help="c3: which of the reference's chains runs -- ref: disk -> planes -> wrap -> S&P "
                         "(127_.../..._3modalities.py:171-174); planes: RandPlaneWaves_ellipsoid alone "
                         "(30_plane_waves_filters/stylized_planes15.py:133); wrap: WrapArtifactd(0.5) alone "
                         "(50_wraparound/stylized_wrap0__test.py); gibbs-aug: RandGibbsNoised(alpha=(0, 0.4)) "
                         "(300_.../30_augmentation/baseline_domain_augment_alpha0p4.py:118); spikes-aug: "
                         "RandKSpaceSpikeNoised(intensity_ranges=(10, 11)) (..._spikes10-11.py:120); the two "
                         "augmentations at prob 1 (the drivers' 0.1 would time mostly identity copies)")
    ap.add_argument("--model", choices=("unet", "gibbs-layer", "spike-layer"), default="unet",
                    help="c3 only.  unet: the filter chain + U-Net(4->3) train step (the headline); gibbs-layer: "
                         "the in-model Gibbs layer drivers (350_stylized_layers/gibbs0p7_layer_domain_GD.py:252-301): "
                         "Gibbs_UNet(1->1) with the device-resident GibbsNoiseLayer at alpha 0.7, train step + "
                         "Gibbs_GD (2 no-grad forwards) per step; spike-layer: Spikes_UNet(I=11) + the intensity "
                         "finite-difference step (spikes11_layer_domain_GD.py:260-300).  Layer models default to "
                         "the drivers' 1 x 128 x 128 x 64 crops (--shape 240,240,160 for BraTS size)")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--no-cudnn-benchmark", action="store_true",
                    help="skip MIOpen Find (its exhaustive solver search makes the first step slow, the rest fast)")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-vols", type=int, default=None,
                    help="volumes per process in the CPU baseline's multi-process modes (c3: 1, c2: 8)")
    ap.add_argument("--cpu-cores", type=int, default=None, help="CPU baseline core count (default: the job's share)")
    ap.add_argument("--filter-only", action="store_true", help="diagnostic: time the filter chain alone")
    ap.add_argument("--graph", action="store_true",
                    help="c3, one GPU: replay the train step as a captured HIP graph (TrainStep(capturable=True)); "
                         "unet: the filter chain still runs eagerly every step (fresh host draws) and writes the "
                         "graph's static input; gibbs-layer: the whole step incl. Gibbs_GD is one graph (the "
                         "layer reads its alpha from device memory)")
    a = ap.parse_args()
    c2, c5 = a.config == "c2", a.config == "c5"
    layer = a.model != "unet"
    if layer and a.config != "c3":
        ap.error("--model gibbs-layer / spike-layer run with --config c3")
    a.batch = a.batch or (16 if c2 else 64 if c5 else 2)
    a.shape = a.shape or ("128,128,128" if c2 else "1,128,128" if c5 else "128,128,64" if layer else "240,240,155")
    if a.pad_to is None:
        a.pad_to = 0 if (c2 or c5 or layer) else 160
    if layer:
        a.no_cpu_baseline = True  # the layers run inside the model on the GPU in the reference too
    if c5:
        a.no_cpu_baseline = True  # the reference trains its DCGAN on the GPU; no CPU path to time
        a.channels_last = True    # NHWC: 4.89k vs 4.60k slices/s at batch 64 (profiles/r2/bench/c5_variants.txt)
    if a.chain != "ref":
        a.no_cpu_baseline = True  # the CPU restatement times the reference chain only
    a.cpu_sample_vols = a.cpu_sample_vols or (8 if c2 else 1)
    if c2:
        a.filter_only = True  # config 2 is the filter kernel alone
    if a.graph and (a.config != "c3" or a.filter_only or a.model == "spike-layer" or a.gpus != 1):
        ap.error("--graph: c3 train step on one GPU, --model unet or gibbs-layer (spike_gd reads its slope "
                 "on the host every step)")
    return a


# traffic_<config or chain>.json (scripts/make_traffic.py), newest round first
TRAFFIC_DIRS = [os.path.join(ROOT, "profiles", r) for r in ("r6", "r5", "r4", "r3")]


def pmc_traffic(kernel: str, launch_bytes: int, key: str = "c3"):
    """(HBM bytes per launch of a filter kernel from the committed rocprofv3 PMC passes (FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction), the file) or (None, None) when not measured for
    launches of this size (a record carries the kernel name and the algorithmic bytes it measured)."""
    for d in TRAFFIC_DIRS:
        path = os.path.join(d, f"traffic_{key}.json")
        try:
            with open(path) as f:
                rec = json.load(f)["kernels"].get(kernel)
        except (OSError, ValueError, KeyError):
            continue
        if rec and abs(int(rec.get("algorithmic_bytes_per_launch", -1)) - int(launch_bytes)) <= 0.001 * launch_bytes:
            return int(rec["traffic_bytes"]), os.path.relpath(path, ROOT)
    return None, None


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


def cpu_baseline(args, shape) -> dict:
    """The reference's CPU filter path on this host's cores (oracle/cpu_bench.py, test/baseline
    infrastructure): the torch-CPU restatement in the three BASELINE.md modes plus the numpy oracle.
    ``value`` is the best mode (the strongest CPU baseline); every mode is listed."""
    from oracle import cpu_bench
    n = args.cpu_sample_vols
    rep = cpu_bench.three_modes(args.config, shape, vols_single=2 * n, vols_multi=n, cores=args.cpu_cores,
                                numpy_vols=n)
    torch_modes = [m for m in rep["modes"] if m["kind"] == "torch"]
    best = max(torch_modes, key=lambda m: m["vols_per_s"])
    chain = ("disk(12.5)->planes(55,55,30,I=15)->wrap(0.5)->S&P(0.05)" if args.config == "c3"
             else "disk low-pass r=12.5 (RandFourierDiskMaskd)")
    return {"value": best["vols_per_s"], "unit": "vols/s", "cores": best["cores"], "kind": "port",
            "sample": f"{best['volumes']} volume(s) 4x{'x'.join(map(str, shape))} in mode '{best['mode']}' through the "
                      f"torch-CPU restatement of the reference's {chain} (oracle/torch_chain.py), {best['seconds']} s; "
                      f"filter only; best of the modes listed",
            "cpu_model": rep["cpu_model"], "job_cores": rep["job_cores"], "modes": rep["modes"]}


def main():
    args = parse()
    maybe_launch_ranks(args)
    H, W, D = (int(v) for v in args.shape.split(","))
    cpu_line = None
    if args.gpus == 1 and "WORLD_SIZE" not in os.environ and not args.no_cpu_baseline:
        # before anything touches the GPU: the CPU workers are fresh interpreters and the host is idle
        t_c = time.perf_counter()
        cpu_line = cpu_baseline(args, (4, H, W, D))
        print(f"[bench] cpu baseline {time.perf_counter() - t_c:.1f} s", file=sys.stderr, flush=True)
    from texbias import runtime as rt
    from texbias.pipeline import FusedChain, reference_c3_chain
    from texbias.synth import brats_labels, brats_like
    from texbias.train import TrainStep, init_distributed, reference_model

    rank, world, local = init_distributed()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} ranks")
    if rank == 0:
        print(f"[bench] world size {world} (backend {dist.get_backend() if world > 1 else 'none'})",
              file=sys.stderr, flush=True)
    dev = torch.device("cuda", local)
    layer_model = args.model != "unet"
    B, C = args.batch, (1 if (args.config == "c5" or layer_model) else 4)
    pad = max(0, args.pad_to - D)
    torch.manual_seed(1000 + rank)

    # resident synthetic data: two distinct batches per rank, labels pre-padded
    pool = [brats_like(B, C, (H, W, D), seed=rank * 97 + i, device=dev) for i in range(2)]
    labels = [] if args.filter_only else \
        [brats_labels(B, (H, W, D), seed=rank * 97 + i, device=dev, pad_to=D + pad) for i in range(2)]
    if layer_model:  # the layer drivers segment one class (whole tumour) from one modality
        labels = [lab[:, :1].contiguous() for lab in labels]

    chain, tr = reference_c3_chain(rank)  # per-rank seeded transform streams
    disk, planes, wrap, sap = tr["disk"], tr["planes"], tr["wrap"], tr["sap"]
    if args.config == "c2":
        chain = FusedChain([disk])
    elif args.config == "c5":  # 2-D slices [B, 1, 1, 128, 128]: the plane-wave shell does not fit
        chain = FusedChain([disk, wrap, sap])
    if args.config == "c3" and args.chain != "ref":
        import filters_and_operators as F
        if args.chain == "planes":
            chain = FusedChain([planes])
        elif args.chain == "wrap":
            chain = FusedChain([wrap])
        elif args.chain == "gibbs-aug":
            g = F.RandGibbsNoised("image", prob=1.0, alpha=(0.0, 0.4))
            g.set_random_state(100 + rank)
            chain = FusedChain([g])
        else:
            g = F.RandKSpaceSpikeNoised("image", global_prob=1.0, prob=1.0, intensity_ranges={"image": (10.0, 11.0)})
            g.set_random_state(100 + rank)
            chain = FusedChain([g])
    prs = np.random.RandomState(12345 + rank)

    def randomize_filters():
        disk.r = float(prs.uniform(10.0, 25.1))
        planes.intensity_value = float(prs.uniform(10.0, 17.0))
        wrap.transform.alpha = float(prs.choice([0.0, 0.25, 0.5, 0.75]))
        sap.p = float(prs.uniform(0.05, 0.35))

    step_fn = None
    if args.config == "c5":
        from texbias.dcgan import DCGANStep
        torch.backends.cudnn.benchmark = not args.no_cudnn_benchmark
        torch.manual_seed(0)  # identical network init on every rank
        step_fn = DCGANStep(dev, distributed=world > 1, bf16=not args.fp32, channels_last=args.channels_last)
        torch.manual_seed(1000 + rank)
    elif layer_model:
        import stylization_layers as SL
        from texbias.train import gibbs_gd, spike_gd
        torch.backends.cudnn.benchmark = not args.no_cudnn_benchmark
        torch.manual_seed(0)
        if args.model == "gibbs-layer":
            lm = SL.Gibbs_UNet()
            lm.gibbs.alpha.fill_(0.7)  # the driver's GibbsNoiseLayer(0.7) (gibbs0p7_layer_domain_GD.py)
        else:
            lm = SL.Spikes_UNet(11.0)
        torch.manual_seed(1000 + rank)
        step_fn = TrainStep(lm, dev, distributed=world > 1, bucket_cap_mb=args.bucket_mb, capturable=args.graph)
        gd = gibbs_gd if args.model == "gibbs-layer" else spike_gd
        train_step = step_fn

        def step_fn(x, y):  # noqa: F811 - train step, then the layer's finite-difference update
            loss = train_step(x, y)
            gd(x, y, train_step.model, train_step.loss_fn)
            return loss
    elif not args.filter_only:
        torch.backends.cudnn.benchmark = not args.no_cudnn_benchmark
        step_fn = TrainStep(reference_model(C, 3), dev, distributed=world > 1, bucket_cap_mb=args.bucket_mb,
                            channels_last=args.channels_last, capturable=args.graph)

    def one_step(i):
        if args.random_filters:
            randomize_filters()
        if layer_model:  # the filter is the model's first layer
            return step_fn(pool[i % 2], labels[i % 2])
        y = chain(pool[i % 2], pad=pad)
        if args.config == "c5":
            return step_fn(y.view(B, 1, W, D))
        if step_fn is not None:
            return step_fn(y, labels[i % 2])
        return y

    graphs = None
    if args.graph:
        # static input of the U-Net step: the eager chain writes it every step (fresh draws)
        xs = None if layer_model else torch.zeros((B, C, H, W, D + pad), device=dev)

        def body(i):  # the captured part: everything but the filter chain's host draws
            return step_fn(pool[i % 2] if layer_model else xs, labels[i % 2])

        def fill(i):
            if args.random_filters:
                randomize_filters()
            if not layer_model:
                chain(pool[i % 2], pad=pad, out=xs)

        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm up off the capture stream: plans, workspaces, solver choice, optimizer state
            for i in range(max(args.warmup, 2)):
                t_w = time.perf_counter()
                fill(i)
                body(i)
                torch.cuda.synchronize(dev)
                if rank == 0:
                    print(f"[bench] warmup step {i}: {time.perf_counter() - t_w:.3f} s", file=sys.stderr, flush=True)
        torch.cuda.current_stream(dev).wait_stream(side)
        graphs = []
        for k in range(2):  # one graph per resident batch; one memory pool, replayed in capture order
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=graphs[0].pool() if graphs else None):
                body(k)
            graphs.append(g)
        torch.cuda.synchronize(dev)

        def one_step(i):  # noqa: F811
            fill(i)
            graphs[i % 2].replay()
    else:
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
    stat_steps = args.steps
    if graphs is not None and not any(cnt[:3]):
        # the filter launches sit inside the graph: time them on eager steps after the timed region
        stat_steps = min(args.steps, 5)
        rt.set_pass_timing(True)
        for i in range(stat_steps):
            body(i)
        torch.cuda.synchronize(dev)
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
        if layer_model:
            workload = f"LAYER DRIVER {args.model}: " + (
                "Gibbs_UNet(1->1) with GibbsNoiseLayer alpha 0.7 (device-resident), train step + Gibbs_GD "
                "(2 no-grad forwards) per step (350_stylized_layers/gibbs0p7_layer_domain_GD.py:252-301)"
                if args.model == "gibbs-layer" else
                "Spikes_UNet(1->1, I=11), train step + intensity finite-difference step (2 no-grad forwards) "
                "(350_stylized_layers/spikes11_layer_domain_GD.py:260-300)") + (
                " [whole step replayed as a HIP graph]" if args.graph else "")
        elif args.config == "c3":
            workload = ("C3 full filter chain (disk 12.5 -> plane wave (55,55,30) I=15 -> wrap 0.5 -> S&P 0.05) "
                        "+ 3D U-Net(4->3, 16..256, 2 res units) fwd/bwd/Adam(amsgrad), DiceLoss"
                        + (" [random per-batch filter params, config 4]" if args.random_filters else "")
                        + (f" [CHAIN {args.chain}: see bench.py --help]" if args.chain != "ref" else "")
                        + (" [FILTER ONLY diagnostic]" if args.filter_only else "")
                        + (" [train step replayed as a HIP graph]" if args.graph else ""))
        else:
            workload = "C2 Gibbs truncation: RandFourierDiskMaskd(r=12.5) low-pass alone, batched 4x128^3 volumes"
        traffic, traffic_file = pmc_traffic(passes[dom]["kernel"], dom_bytes,
                                            args.chain if args.config == "c3" and args.chain != "ref" else args.config)
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
                "workload": workload,
                "volume": [C, H, W, D],
                "unet_input": [B, C, H, W, D + pad],
                "per_gpu_batch": B,
                "global_batch": B * world,
                "parallelism": f"dp{world}",
            },
            "roofline": {"kernel": passes[dom]["kernel"], "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_unit": f"bytes per launch (rocprofv3 PMC, {traffic_file})",
                         "algorithmic_bytes_per_launch": dom_bytes},
            "filter_passes": passes,
            "filter_ms_per_step": round(sum(ms) / stat_steps, 4),
        }
        if args.config == "c3" and not layer_model and not args.filter_only:
            from texbias.train import step_conv_flops
            fl = step_conv_flops(lambda: reference_model(C, 3), (B, C, H, W, D + pad))
            tfs = fl / (elapsed / args.steps) / 1e12
            line["unet_compute"] = {"analytic_tflop_per_step": round(fl / 1e12, 4), "tflop_s": round(tfs, 2),
                                    "peak_f32_matrix_tflop_s": 157.3, "frac": round(tfs / 157.3, 4),
                                    "note": "per rank: the U-Net's conv layers (fwd + weight grad + input grad except "
                                            "the network input's), texbias.train.step_conv_flops / measured step time "
                                            "(the whole step, filter chain included)"}
        if args.config == "c5":
            from texbias.dcgan import step_flops
            fl = step_flops() * B  # per rank and step (analytic: 3x forward per backward pass)
            tfs = fl / (elapsed / args.steps) / 1e12
            line.update({
                "unit": "slices/s", "dtype": "f32" if args.fp32 else "bf16",
                "data": "synthetic BraTS-like 1x128x128 slices resident in HBM, filtered on the GPU each step; "
                        "random-init DCGAN (N(0, 0.02) init)",
            })
            line["config"] = {
                "workload": "C5 DCGAN (50_reconstruction/networks.py, nz=100, ngf=ndf=128) step: D on real + D on G(z) "
                            "+ Adam(2e-4, 0.5), G through the updated D + Adam; input slices filtered by disk 12.5 -> "
                            "wrap 0.5 -> S&P 0.05 on the GPU" + (" [fp32]" if args.fp32 else " [bf16 autocast]")
                            + (" [channels_last]" if args.channels_last else ""),
                "slice": [1, W, D], "per_gpu_batch": B, "global_batch": B * world, "parallelism": f"dp{world}"}
            line["roofline"] = {"kernel": "DCGAN step (MIOpen/hipBLASLt convolutions)", "bound": "mfma",
                                "achieved": round(tfs, 2), "peak": 2500.0 if not args.fp32 else 157.3,
                                "unit": "TFLOP/s", "frac": round(tfs / (2500.0 if not args.fp32 else 157.3), 4),
                                "traffic": None, "algorithmic_flops_per_step": fl,
                                "note": "analytic conv flops / measured step time (whole step, not one kernel)"}
        if cpu_line is not None:
            line["cpu_baseline"] = cpu_line
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
