import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE-size batches)")
    config.addinivalue_line("markers", "multigpu: needs two or more GPUs in one process")


def pytest_collection_modifyitems(config, items):
    """Tests marked multigpu are deselected (not skipped) where fewer than two
    GPUs are visible -- the one-GPU round-end box included.  Counting devices
    does not initialise the GPU on this image."""
    if not any(it.get_closest_marker("multigpu") for it in items):
        return
    import torch
    if torch.cuda.device_count() >= 2:
        return
    keep = [it for it in items if not it.get_closest_marker("multigpu")]
    dropped = [it for it in items if it.get_closest_marker("multigpu")]
    config.hook.pytest_deselected(items=dropped)
    items[:] = keep


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(HERE, "golden")


@pytest.fixture
def aes_engine():
    """Selects the AES-GCM engine for one test ("bs" or "table",
    BSSL_AMD_set_aes_gcm_engine) and restores the previous one afterwards."""
    import boringssl_amd as ba
    prev = ba.aes_gcm_engine()
    yield ba.set_aes_gcm_engine
    ba.set_aes_gcm_engine(prev)
