import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels); run with -m gpu")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs (RCCL P2P over xGMI)")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_count():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def pytest_collection_modifyitems(config, items):
    n = _gpu_count()
    skip_gpu = pytest.mark.skip(reason="no GPU visible")
    skip_multi = pytest.mark.skip(reason="needs >= 2 GPUs")
    for it in items:
        if "gpu" in it.keywords and n < 1:
            it.add_marker(skip_gpu)
        if "multigpu" in it.keywords and n < 2:
            it.add_marker(skip_multi)
