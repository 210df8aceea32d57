import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) GPU")
    config.addinivalue_line("markers", "slow: multi-process / long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _restore_environ():
    """Every test sees (and leaves) the session's environment: nothing a test or the code under
    test writes into os.environ leaks into a later test or the subprocesses it starts."""
    saved = dict(os.environ)
    yield
    if dict(os.environ) != saved:
        os.environ.clear()
        os.environ.update(saved)


@pytest.fixture(scope="session", autouse=True)
def _teardown_process_group():
    """Tests that initialise the default process group in-process (engine, graph impl, native RCCL)
    share it; tear it down once at the end, as the reference's train.py:138 does."""
    yield
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
