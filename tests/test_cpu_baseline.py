"""The CPU baseline's torch restatement (oracle/torch_chain.py) agrees with the numpy parity oracle
stage by stage, and the three-mode runner (oracle/cpu_bench.py) produces a well-formed report."""
import numpy as np
import torch

from oracle import cpu_bench
from oracle import filters_oracle as O
from oracle import torch_chain as T


def _x(shape=(4, 24, 20, 18), seed=0):
    return cpu_bench._volume(shape, seed)


def rel(a, b):
    return np.abs(np.asarray(a, np.float64) - b).max() / np.abs(b).max()


def test_torch_restatement_matches_numpy_oracle():
    x = _x()
    xt = torch.from_numpy(x)
    y1 = T.disk(xt, 12.5)
    assert rel(y1.numpy(), O.fourier_disk(x, 12.5)) < 1e-5
    np.testing.assert_array_equal(T.disk_mask(xt.shape, 5.0).numpy(), O.disk_mask(xt.shape, 5.0, 3, False))
    coords_t = T.ellipsoid_coords((24, 20, 18), 8.0, 7.0, 6.0).numpy()
    np.testing.assert_array_equal(coords_t, O.ellipsoid_shell((24, 20, 18), 8.0, 7.0, 6.0))
    y2, idx = T.planes(y1, 8.0, 7.0, 6.0, 9.0, np.random.RandomState(3))
    idx_o = O.ellipsoid_sample(O.ellipsoid_shell((24, 20, 18), 8.0, 7.0, 6.0), np.random.RandomState(3))
    assert idx == idx_o
    # the spiked coefficient's phase after the low-pass is rounding noise: take it from torch's own FFT
    k = T._fwd(y1)
    ph = k[:, idx[0], idx[1], idx[2]].angle().numpy()
    assert rel(y2.numpy(), O.plane_waves(y1.numpy(), idx, 9.0, phase=ph)) < 1e-5
    y3 = T.wrap(y2, 0.5)
    assert rel(y3.numpy(), O.wrap_artifact(y2.numpy(), 0.5)) < 1e-5


def test_torch_sap_semantics():
    x = torch.from_numpy(_x((4, 32, 32, 32), 1))
    y = T.sap(x, 0.2, torch.Generator().manual_seed(0))
    mn, mx = x.min() / 2, x.max() / 2
    pep, salt, keep = y == mn, (y == mx) & (x != mx), y == x
    assert torch.all(pep | salt | keep)
    frac = 1.0 - keep.double().mean().item()
    assert 0.17 < frac < 0.23


def test_run_mode_report():
    r = cpu_bench.run_mode("torch", "c2", (4, 16, 16, 16), procs=2, threads=1, vols_per_proc=2, timeout=300)
    assert r["volumes"] == 4 and r["cores"] == 2 and r["vols_per_s"] > 0
    # the C3 chain needs the (55, 55, 30) ellipsoid shell inside the grid: 4 x 116 x 116 x 64
    r = cpu_bench.run_mode("torch", "c3", (4, 116, 116, 64), procs=1, threads=2, vols_per_proc=1, timeout=300)
    assert r["volumes"] == 1 and r["cores"] == 2
    r = cpu_bench.run_mode("numpy", "c2", (4, 24, 24, 24), procs=1, threads=1, vols_per_proc=1, timeout=300)
    assert r["volumes"] == 1
    try:  # a worker error surfaces as an exception, not a hang (no shell point fits 24^3)
        cpu_bench.run_mode("numpy", "c3", (4, 24, 24, 24), procs=2, threads=1, vols_per_proc=1, timeout=300)
        raise AssertionError("expected a worker error")
    except RuntimeError as e:
        assert "worker failed" in str(e)
    assert cpu_bench.job_cores() >= 1 and isinstance(cpu_bench.cpu_model(), str)
