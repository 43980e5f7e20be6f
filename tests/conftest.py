import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP kernels)")


def pytest_sessionstart(session):
    """A fresh checkout (no built library) in the build container (hipcc, no
    GPU) builds it first.  On a GPU box the prebuilt library travels with the
    tree and nothing is built: a missing one makes the product fail loudly."""
    import shutil

    lib = os.path.join(ROOT, "parameter_server_amd", "libpskv.so")
    if (not os.path.exists(lib) and not os.path.exists("/dev/kfd")
            and shutil.which(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"))):
        import __graft_entry__ as g

        g.build()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda:0")
