"""ctypes view of the CPU oracle (oracle/build/librs_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package ``rustfs_amd``.
The C restatement and its reference anchors are in oracle/rs_oracle.c.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "librs_oracle.so")
_lib = None

MAGIC_KEY = bytes.fromhex("4be734fa8e238acd263e83e6bb968552040f935da39f441497e09d1322de36a0")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.ro_gf_mul.restype = ctypes.c_uint8
        L.ro_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.ro_build_matrix.argtypes = [ctypes.c_int, ctypes.c_int, P]
        L.ro_invert.argtypes = [ctypes.c_int, P]
        L.ro_encode.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_size_t]
        L.ro_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_size_t, ctypes.c_int]
        L.ro_verify.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_size_t]
        L.ro_hh256.argtypes = [P, P, ctypes.c_size_t, P]
        L.ro_hh256s.argtypes = [P, ctypes.c_size_t, P]
        L.ro_hh256s_legacy.argtypes = [P, ctypes.c_size_t, P]
        L.ro_encode_batch_mt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, P, P, ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _ptr_array(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def gf_mul(a: int, b: int) -> int:
    return int(lib().ro_gf_mul(a, b))


def matrix(k: int, m: int) -> np.ndarray:
    out = np.zeros((k + m, k), dtype=np.uint8)
    if lib().ro_build_matrix(k, m, _ptr(out)) != 0:
        raise ValueError(f"bad geometry k={k} m={m}")
    return out


def invert(mat: np.ndarray) -> np.ndarray:
    m = np.ascontiguousarray(mat, dtype=np.uint8).copy()
    if lib().ro_invert(m.shape[0], _ptr(m)) != 0:
        raise ValueError("singular matrix")
    return m


def encode(k: int, m: int, shards: np.ndarray) -> np.ndarray:
    """shards: (k+m, S) uint8; parity rows are overwritten in place (returned)."""
    assert shards.shape[0] == k + m and shards.dtype == np.uint8 and shards.flags.c_contiguous
    rows = [shards[i] for i in range(k + m)]
    if lib().ro_encode(k, m, _ptr_array(rows), shards.shape[1]) != 0:
        raise ValueError("encode failed")
    return shards


def reconstruct(k: int, m: int, shards: np.ndarray, present, data_only: bool = False) -> np.ndarray:
    rows = [shards[i] for i in range(k + m)]
    pres = np.asarray([1 if p else 0 for p in present], dtype=np.uint8)
    rc = lib().ro_reconstruct(k, m, _ptr_array(rows), _ptr(pres), shards.shape[1], 1 if data_only else 0)
    if rc == -2:
        raise ValueError("too few shards present")
    if rc != 0:
        raise ValueError("reconstruct failed")
    return shards


def verify(k: int, m: int, shards: np.ndarray) -> bool:
    rows = [shards[i] for i in range(k + m)]
    return lib().ro_verify(k, m, _ptr_array(rows), shards.shape[1]) == 1


def hh256(key32: bytes, data) -> bytes:
    d = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)
    k = np.frombuffer(key32, dtype=np.uint64).copy()
    out = np.zeros(32, dtype=np.uint8)
    lib().ro_hh256(_ptr(k), _ptr(d) if d.size else None, d.size, _ptr(out))
    return out.tobytes()


def hh256s(data) -> bytes:
    return hh256(MAGIC_KEY, data)


def hh256s_legacy(data) -> bytes:
    key = np.array([3, 4, 2, 1], dtype=np.uint64).tobytes()
    return hh256(key, data)


def encode_batch_mt(k: int, m: int, S: int, stripes: np.ndarray, digests: np.ndarray | None = None, threads: int = 0) -> None:
    n = stripes.size // ((k + m) * S)
    rc = lib().ro_encode_batch_mt(k, m, S, n, _ptr(stripes), _ptr(digests) if digests is not None else None, threads)
    if rc != 0:
        raise ValueError("encode_batch_mt failed")


def xorshift_payload(n: int, seed: int = 0x9E3779B97F4A7C15) -> np.ndarray:
    """bitrot_self_test_payload (bitrot.rs:861-871) generalised to n bytes."""
    out = np.empty(n, dtype=np.uint8)
    s = seed
    M = (1 << 64) - 1
    for i in range(n):
        s ^= s >> 12
        s ^= (s << 25) & M
        s ^= s >> 27
        out[i] = (s * 0x2545F4914F6CDD1D) & 0xFF
    return out
