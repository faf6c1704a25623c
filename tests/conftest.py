import os
import sys

import pytest

# PyTorch ships its own libamdhip64 under the SONAME /opt/rocm's has: import
# it before anything loads the engine library (tests that only touch the
# host-side ABI, e.g. spf_table_layout, load it too), so the engine binds to
# torch's already-loaded HIP runtime (see gpu_ready).
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)"
    )


@pytest.fixture(scope="session")
def gpu_ready():
    # PyTorch ships its own libamdhip64 (same SONAME as /opt/rocm's, which
    # the engine links): initialise torch's HIP runtime first so the engine
    # binds to the already-loaded one, as bench.py does.  Loaded the other
    # way round, torch later reports "No HIP GPUs are available".
    import torch

    torch.cuda.init()
    from openr_amd import abi

    n = abi.device_count()
    if n <= 0:
        pytest.fail("no HIP device visible: the -m gpu tests need an MI355X")
    return n
