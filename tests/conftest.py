import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "llama-fft_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def built_lib():
    """Path of libbcfft.so, building it in-tree (hipcc cross-compiles without a GPU) if absent."""
    import subprocess
    lib = os.path.join(PKG, "lib", "libbcfft.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", PKG], check=True, stdout=subprocess.DEVNULL)
    return lib
