import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    workers = os.environ.get("PYTEST_XDIST_WORKER_COUNT")
    if workers:
        # pytest -n N: split the CPUs between the workers. Each torch process otherwise spins
        # os.cpu_count() intra-op threads, and the epoch-loop tests (UMAP) slow down ~100x.
        import torch

        torch.set_num_threads(max(1, (os.cpu_count() or 1) // int(workers)))
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "compat: Spark-API compatibility test (oracle values from Spark docs/tests)")
    config.addinivalue_line("markers", "dist: multi-process (gloo) distributed test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    return torch.device("cuda", 0)
