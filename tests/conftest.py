import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "medical-vision-textural-bias_amd")
for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def heartbeat(request):
    """Print a progress line every 30 s while a long GPU test runs (fresh boxes compile MIOpen kernels
    for minutes; the line shows the test is alive, not hung)."""
    import threading
    import time
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(30.0):
            print(f"[heartbeat] {request.node.name} {time.time() - t0:.0f} s", flush=True)

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
    th.join(timeout=1.0)
