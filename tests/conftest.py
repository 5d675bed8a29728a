import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ml_music_style_transfer_amd import _lib
    _lib.load()
    return torch.device("cuda")


@pytest.fixture(autouse=True)
def _sync_device_after_gpu_test(request):
    """Every GPU test ends with a device-wide synchronize, so an asynchronous kernel fault is
    raised in the test that launched the kernel (including work left on side streams), not at
    the first HIP call of the next test (round 3's unexplained hipErrorLaunchFailure surfaced that
    way)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
