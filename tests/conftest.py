import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through librsgpu.so's HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    """The CPU oracle (test infrastructure only), built on demand."""
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def ref_vectors():
    with open(os.path.join(GOLDEN, "reference_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def derived_vectors():
    with open(os.path.join(GOLDEN, "derived_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def rsgpu_lib():
    lib = os.path.join(ROOT, "rustfs_amd", "librsgpu.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "rustfs_amd", "csrc")], check=True)
    from rustfs_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(rsgpu_lib):
    """A live rsg_ctx on device 0.  GPU tests fail loudly (no CPU fallback)."""
    import torch  # noqa: F401  (shares the HIP runtime; see rustfs_amd/_lib.py)
    from rustfs_amd import _lib
    return _lib.context(0)


def compat_data(n: int) -> bytes:
    return bytes((i * 7 + 13) % 256 for i in range(n))
