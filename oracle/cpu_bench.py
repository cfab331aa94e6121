"""CPU baseline runner: the reference's filter path timed on the host cores in three modes.

TEST / BASELINE INFRASTRUCTURE ONLY (used by ``bench.py``'s ``cpu_baseline`` leg and tests).

Modes:
  (i)   1 thread per process x 4 processes   -- the reference's DataLoader(num_workers=4) setting
  (ii)  1 thread per process x `cores` processes
  (iii) 1 process x `cores` threads
``cores`` = the CPUs this job may use: OMP_NUM_THREADS when set (the GPU box pins it to the job's
share, 16), else the affinity mask.  Workers are fresh interpreters (multiprocessing "spawn": no
inherited GPU state, thread counts fixed before torch loads); each builds its own synthetic volume,
runs one untimed warm-up volume of a small shape, waits on a barrier, then times its volumes.
Throughput = all volumes / (last worker end - first worker start).

Kinds: "torch" -- oracle/torch_chain.py (the reference's own torch-CPU arithmetic); "numpy" --
oracle/filters_oracle.py (the parity oracle's numpy restatement, pocketfft, single-threaded).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import platform
import time
from typing import Dict, List, Sequence


def job_cores() -> int:
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _volume(shape: Sequence[int], seed: int):
    """BraTS-like synthetic volume (zero background outside a centred ellipsoid, smooth field + noise)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    C, D, H, W = shape
    zz, yy, xx = np.meshgrid(*[np.linspace(-1, 1, n, dtype=np.float32) for n in (D, H, W)], indexing="ij")
    brain = (zz / 0.8) ** 2 + (yy / 0.9) ** 2 + (xx / 0.7) ** 2 < 1.0
    x = rng.standard_normal((C, D, H, W), dtype=np.float32)
    x += np.float32(0.5) * np.sin(3 * zz + 2 * yy)[None] * np.cos(2 * xx)[None]
    x *= brain[None]
    return x


def _worker(kind: str, config: str, shape, nvols: int, threads: int, seed: int, barrier, q) -> None:
    try:
        _work(kind, config, shape, nvols, threads, seed, barrier, q)
    except BaseException as e:  # report instead of leaving the parent waiting
        barrier.abort()
        q.put(("error", f"{type(e).__name__}: {e}", 0))


def _work(kind: str, config: str, shape, nvols: int, threads: int, seed: int, barrier, q) -> None:
    os.environ["OMP_NUM_THREADS"] = str(threads)
    os.environ["MKL_NUM_THREADS"] = str(threads)
    import numpy as np
    rs = np.random.RandomState(seed)
    x = _volume(shape, seed)
    if kind == "torch":
        import torch
        torch.set_num_threads(threads)
        from oracle import torch_chain as T
        fn = T.chain_c3 if config == "c3" else T.chain_c2
        gen = torch.Generator().manual_seed(seed)
        xt = torch.from_numpy(x)
        T.disk(torch.from_numpy(_volume((shape[0], 16, 16, 16), seed)), 4.0)  # warm-up (FFT plans, allocator)

        def run():
            fn(xt, rs, gen)
    else:
        from oracle import filters_oracle as O
        coords = O.ellipsoid_shell(shape[1:], 55.0, 55.0, 30.0)

        def run():
            if config == "c3":
                idx = O.ellipsoid_sample(coords, rs)
                u = rs.random_sample(shape).astype(np.float32)
                O.chain(x, 12.5, idx, 15.0, 0.5, 0.05, u)
            else:
                O.fourier_disk(x, 12.5)
    barrier.wait(timeout=600)
    t0 = time.time()
    for _ in range(nvols):
        run()
    q.put((t0, time.time(), nvols))


def run_mode(kind: str, config: str, shape, procs: int, threads: int, vols_per_proc: int, timeout: float = 600.0) -> Dict:
    ctx = mp.get_context("spawn")
    barrier = ctx.Barrier(procs)
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(kind, config, tuple(shape), vols_per_proc, threads, 1000 + i, barrier, q),
                      daemon=True) for i in range(procs)]
    for p in ps:
        p.start()
    res = []
    try:
        for _ in range(procs):
            r = q.get(timeout=timeout)
            if r[0] == "error":
                raise RuntimeError(f"CPU baseline worker failed: {r[1]}")
            res.append(r)
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    t0 = min(r[0] for r in res)
    t1 = max(r[1] for r in res)
    n = sum(r[2] for r in res)
    return {"kind": kind, "processes": procs, "threads_per_process": threads, "cores": procs * threads,
            "volumes": n, "seconds": round(t1 - t0, 3), "vols_per_s": round(n / (t1 - t0), 5)}


def three_modes(config: str, shape, vols_single: int = 1, vols_multi: int = 1, kinds: Sequence[str] = ("torch",),
                cores: int = None, numpy_vols: int = 1) -> Dict:
    """The three BASELINE.md modes for the torch restatement, plus the numpy oracle single-threaded."""
    cores = cores or job_cores()
    modes: List[Dict] = []
    for kind in kinds:
        modes.append(dict(mode="i: 1 thread x 4 processes", **run_mode(kind, config, shape, 4, 1, vols_multi)))
        modes.append(dict(mode=f"ii: 1 thread x {cores} processes", **run_mode(kind, config, shape, cores, 1, vols_multi)))
        modes.append(dict(mode=f"iii: 1 process x {cores} threads", **run_mode(kind, config, shape, 1, cores, vols_single)))
    if numpy_vols > 0:
        modes.append(dict(mode="numpy oracle, 1 thread x 1 process", **run_mode("numpy", config, shape, 1, 1, numpy_vols)))
    return {"cpu_model": cpu_model(), "job_cores": cores, "modes": modes}
