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
    assert rsgpu_lib.rsg_abi_version() == 6


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


def test_tuning_knobs_default_and_settable(rsgpu_lib):
    """rsg_get_tuning reports every knob's default; rsg_set_tuning changes one
    knob, refuses unknown names and values out of range without changing
    anything, and NULL value / NULL name restore the defaults (no GPU)."""
    from rustfs_amd import _lib
    for k, v in _lib.TUNING_DEFAULTS.items():
        assert _lib.get_tuning(k) == v, k
    with _lib.tuned(RSG_DECODE_NET="0", RSG_FUSED_KIND="dma", RSG_HASH_DEPTH="3"):
        assert (_lib.get_tuning("RSG_DECODE_NET"), _lib.get_tuning("RSG_FUSED_KIND"),
                _lib.get_tuning("RSG_HASH_DEPTH")) == ("0", "dma", "3")
    assert _lib.get_tuning("RSG_DECODE_NET") == "1" and _lib.get_tuning("RSG_FUSED_KIND") == "auto"
    # RSG_NET12_RD=4: its kernels are compiled into measurement builds only
    for name, bad in (("RSG_NET12_RD", b"3"), ("RSG_NET12_RD", b"4"), ("RSG_DECODE_NET", b"yes"), ("RSG_HASH_DEPTH", b"4"),
                      ("RSG_FUSED_KIND", b"fast"), ("RSG_NO_SUCH_KNOB", b"1")):
        assert rsgpu_lib.rsg_set_tuning(name.encode(), bad) == _lib.RSG_ERR_INVALID_ARG
    assert _lib.get_tuning("RSG_HASH_DEPTH") == "2"
    _lib.set_tuning("RSG_HASH_DEPTH", "3")
    _lib.set_tuning("RSG_HASH_DEPTH", None)
    assert _lib.get_tuning("RSG_HASH_DEPTH") == "2"
    _lib.set_tuning("RSG_VEC_OCC", "4")
    _lib.set_tuning(None, None)
    assert _lib.get_tuning("RSG_VEC_OCC") == "-1"
    buf = ctypes.create_string_buffer(2)
    assert rsgpu_lib.rsg_get_tuning(b"RSG_FUSED_KIND", buf, 2) == _lib.RSG_ERR_INVALID_ARG


def test_environment_changes_no_kernel_choice():
    """The production library ignores the RSG_* environment variables (only
    measurement builds read them): a process with every knob set to a
    non-default value in its environment still sees the defaults."""
    import subprocess
    import sys
    from rustfs_amd import _lib
    env = dict(os.environ)
    nondefault = {"RSG_FUSED": "0", "RSG_LOST_DISK_FAST": "0", "RSG_ZERO_COPY": "0", "RSG_VEC_BLOCK": "256",
                  "RSG_VEC_OCC": "3", "RSG_ROLLED": "1", "RSG_HASH_COPY": "1", "RSG_HASH_DEPTH": "3",
                  "RSG_FUSED_KIND": "dma", "RSG_FUSED_SPW1": "1", "RSG_ENC_PRIO": "3", "RSG_DMA_EW": "4",
                  "RSG_DMA_NT": "0", "RSG_DMA_SPW": "4", "RSG_DMA_PRIO": "0", "RSG_DECODE_NET": "0",
                  "RSG_NET12_RD": "4", "RSG_HASH_UNAL": "0", "RSG_GET_CACHED": "0"}
    assert set(nondefault) == set(_lib.TUNING_DEFAULTS)
    env.update(nondefault)
    code = ("import json, sys; sys.path.insert(0, %r); from rustfs_amd import _lib; "
            "print(json.dumps({k: _lib.get_tuning(k) for k in _lib.TUNING_DEFAULTS}))" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    import json
    assert json.loads(out.stdout.strip().splitlines()[-1]) == _lib.TUNING_DEFAULTS
