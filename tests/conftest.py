import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, "--h.264-by-zhaodongyu_amd")
for p in (HERE, PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu():
    """The HIP product path must run: fail loudly (never skip) without a GPU."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test on a machine without a visible MI355X")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def built_lib():
    from jmme import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    return _lib.lib()
