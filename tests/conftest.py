import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# tests pin the low-bit-only footprint; the resident prefill shadow (auto on
# large-HBM devices) is exercised by its own test (test_gpu_model.py)
os.environ.setdefault("ILLM_PREFILL_DENSE_GB", "0")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ipex_llm_amd.ops as ops
    ops.require()
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _no_stray_kernel_errors(request):
    """every GPU test leaves the device-side bounds-check word clean: an
    out-of-range index a kernel skipped (ops.check_kernel_errors) is charged
    to the test that caused it, not to whichever test checks next"""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if not torch.cuda.is_available():
        return
    import ipex_llm_amd.ops as ops
    ops.check_kernel_errors(torch.device("cuda", 0))
