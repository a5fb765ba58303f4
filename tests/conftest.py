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


SLOT_FILL = 0xA5  # what the in-place GET's slots hold before the call


def decode_get(e, files, S, n, form, **kw):
    """One GET through either form of the engine, as (data (n, k*S), status).
    "gather": rsg_decode_records_dev.  "into": rsg_decode_records_into_dev
    (reconstruct_into's contract), with the data assembled the way
    write_data_blocks reads it (decode.rs:1390): shard i of stripe s from
    files[i]'s record where src says it was served from there, else from slot
    i — and checked that the call left every served shard's slot untouched and
    never claimed to serve an absent file."""
    import torch
    if form == "gather":
        return e.decode_records_batch(files, S, n, **kw)
    k = e.data_shards
    slots = torch.full((n, k * S), SLOT_FILL, dtype=torch.uint8, device="cuda")
    slots_, src, status = e.decode_records_into_batch(files, S, n, targets=slots, **kw)
    assert slots_ is slots and src.shape == (k, n)
    out = slots.clone().view(n, k, S)
    for i in range(k):
        if files[i] is None:
            assert not src[i].any(), f"absent shard {i} reported as served from its record"
            continue
        served = torch.from_numpy(src[i].copy()).cuda()
        if bool(served.any()):
            assert bool((slots.view(n, k, S)[:, i][served] == SLOT_FILL).all()), f"slot {i} written though served"
            body = files[i][: n * (32 + S)].view(n, 32 + S)[:, 32:]
            out[:, i][served] = body[served]
    return out.view(n, k * S), status


def compat_data(n: int) -> bytes:
    return bytes((i * 7 + 13) % 256 for i in range(n))
