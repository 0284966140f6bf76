import base64
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def b64d(s):
    return base64.b64decode(s)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def has_gpu():
    from swarm_amd import device_count
    return device_count() > 0


@pytest.fixture(scope="module", autouse=True)
def _release_device_memory():
    """After each test module: drop its tensors and return torch's cached device memory, so
    one pytest process running every GPU module does not carry one module's buffers into the
    next (no effect on CPU-only runs: CUDA is never initialised here)."""
    yield
    import gc
    gc.collect()
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():  # never initialises HIP itself
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
