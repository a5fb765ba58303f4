"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/rsgpu.h declares, and its host-only entry points (matrix
construction, geometry validation, error strings) match the oracle / reference."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_symbols():
    src = open(os.path.join(ROOT, "include", "rsgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rsg_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported(rsgpu_lib):
    from rustfs_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(rsgpu_lib, s), f"{s} declared in include/rsgpu.h but not exported"
    assert sorted(_lib.EXPORTED) == syms


def test_exported_symbols_have_c_linkage():
    out = os.popen(f"nm -D --defined-only {os.path.join(ROOT, 'rustfs_amd', 'librsgpu.so')}").read()
    for s in header_symbols():
        assert re.search(rf"\bT {s}$", out, flags=re.M), s


def test_abi_version(rsgpu_lib):
    assert rsgpu_lib.rsg_abi_version() == 5


@pytest.mark.parametrize("k,m", [(1, 1), (2, 2), (3, 1), (4, 2), (6, 3), (8, 4), (12, 4), (16, 4), (10, 10),
                                 (17, 3), (32, 8), (200, 56)])
def test_matrix_matches_oracle(rsgpu_lib, oracle, k, m):
    out = np.zeros((k + m, k), dtype=np.uint8)
    assert rsgpu_lib.rsg_matrix(k, m, out.ctypes.data) == 0
    assert (out == oracle.matrix(k, m)).all()


def test_matrix_pins_reference_rows(rsgpu_lib, derived_vectors):
    for key, rows in derived_vectors["parity_rows"].items():
        k, m = map(int, key.split(","))
        out = np.zeros((k + m, k), dtype=np.uint8)
        assert rsgpu_lib.rsg_matrix(k, m, out.ctypes.data) == 0
        assert [bytes(r).hex() for r in out[k:]] == rows


def test_geometry_errors(rsgpu_lib):
    from rustfs_amd import _lib
    assert rsgpu_lib.rsg_check_geometry(0, 2) == _lib.RSG_ERR_ZERO_DATA_SHARDS
    assert rsgpu_lib.rsg_check_geometry(255, 2) == _lib.RSG_ERR_TOO_MANY_SHARDS
    assert rsgpu_lib.rsg_check_geometry(254, 2) == _lib.RSG_OK
    assert rsgpu_lib.rsg_check_geometry(4, 0) == _lib.RSG_OK
    buf = np.zeros(16, dtype=np.uint8)
    assert rsgpu_lib.rsg_matrix(4, 0, buf.ctypes.data) == _lib.RSG_ERR_ZERO_PARITY_SHARDS


def test_strerror_fragments(rsgpu_lib):
    from rustfs_amd import _lib
    assert _lib.strerror(_lib.RSG_ERR_INCONSISTENT_SOURCES) == "inconsistent read source shards"
    assert _lib.strerror(_lib.RSG_ERR_BITROT_MISMATCH) == "bitrot hash mismatch"
    assert "inconsistent shard length" in _lib.strerror(_lib.RSG_ERR_INCONSISTENT_LENGTH)
    assert "invalid shard count" in _lib.strerror(_lib.RSG_ERR_INVALID_SHARD_COUNT)
    assert "Reed-Solomon reconstruct failed" in _lib.strerror(_lib.RSG_ERR_TOO_FEW_SHARDS)
    assert _lib.strerror(999) == "unknown rsgpu status"


def test_null_args_rejected_without_device(rsgpu_lib):
    from rustfs_amd import _lib
    assert rsgpu_lib.rsg_create(0, None) == _lib.RSG_ERR_INVALID_ARG
    assert rsgpu_lib.rsg_encode(None, 4, 2, 16, None) == _lib.RSG_ERR_INVALID_ARG
    assert rsgpu_lib.rsg_device_count(None) == _lib.RSG_ERR_INVALID_ARG
    rsgpu_lib.rsg_destroy(None)  # no-op
