"""Loader for the in-tree C-ABI library ``rustfs_amd/librsgpu.so`` (include/rsgpu.h).

The product path has no CPU fallback: if the library is missing, importing the
codec raises.  torch is imported first when available so the process has ONE
HIP runtime: torch's bundled ``libamdhip64.so`` carries the SONAME
``libamdhip64.so.7`` that librsgpu.so depends on, so the loader reuses it.
"""
from __future__ import annotations

import ctypes
import os
import threading

try:  # share torch's HIP runtime (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C ABI itself
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
# RSG_LIB_PATH: an experiment build of the same library (tools/ab_*.sh A/B
# runs); the default is the in-tree build.
LIB_PATH = os.environ.get("RSG_LIB_PATH") or os.path.join(HERE, "librsgpu.so")

# rsg_status (include/rsgpu.h)
RSG_OK = 0
RSG_ERR_INVALID_ARG = 1
RSG_ERR_ZERO_DATA_SHARDS = 2
RSG_ERR_ZERO_PARITY_SHARDS = 3
RSG_ERR_TOO_MANY_SHARDS = 4
RSG_ERR_INVALID_SHARD_COUNT = 5
RSG_ERR_INCONSISTENT_LENGTH = 6
RSG_ERR_EMPTY_SHARD = 7
RSG_ERR_TOO_FEW_SHARDS = 8
RSG_ERR_NO_VALID_SHARDS = 9
RSG_ERR_INCONSISTENT_SOURCES = 10
RSG_ERR_BITROT_MISMATCH = 11
RSG_ERR_NO_DEVICE = 12
RSG_ERR_DEVICE = 13
RSG_ERR_OUT_OF_MEMORY = 14
RSG_ERR_UNSUPPORTED = 15
RSG_ERR_FILE_SIZE_MISMATCH = 16
RSG_ERR_UNEXPECTED_EOF = 17
RSG_ERR_TRAILING_DATA = 18

RSG_HASH_NONE = 0
RSG_HASH_HIGHWAY256S = 1
RSG_HASH_HIGHWAY256S_LEGACY = 2

RSG_RECONSTRUCT_DATA = 0
RSG_RECONSTRUCT_MISSING = 1
RSG_RECONSTRUCT_REENCODE_PARITY = 2

RSG_RECORD_ENGINE_AUTO = 0
RSG_RECORD_ENGINE_ONE_PASS = 1
RSG_RECORD_ENGINE_TWO_PASS = 2

# Every symbol include/rsgpu.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "rsg_abi_version", "rsg_strerror", "rsg_device_count", "rsg_create", "rsg_destroy",
    "rsg_matrix", "rsg_check_geometry", "rsg_encode", "rsg_reconstruct", "rsg_verify",
    "rsg_hash", "rsg_encode_batch_dev", "rsg_reconstruct_batch_dev", "rsg_verify_batch_dev",
    "rsg_hash_batch_dev", "rsg_sync", "rsg_encode_batch_host", "rsg_pin", "rsg_unpin",
    "rsg_decode_records_dev", "rsg_heal_records_dev", "rsg_bitrot_verify_dev",
    "rsg_encode_batch_host_submit", "rsg_poll", "rsg_wait", "rsg_set_kernel_timing", "rsg_last_kernel_ms",
    "rsg_set_record_engine", "rsg_decode_records_into_dev", "rsg_decode_records_submit",
    "rsg_heal_records_submit", "rsg_test_fail_subbatch", "rsg_set_tuning", "rsg_get_tuning",
)

# Kernel-choice knobs (rsg_set_tuning, include/rsgpu.h) and their defaults:
# set only through the ABI (the production library ignores RSG_* variables).
TUNING_DEFAULTS = {
    "RSG_FUSED": "1", "RSG_LOST_DISK_FAST": "1", "RSG_ZERO_COPY": "1", "RSG_VEC_BLOCK": "0",
    "RSG_VEC_OCC": "-1", "RSG_ROLLED": "0", "RSG_HASH_COPY": "0", "RSG_HASH_DEPTH": "2",
    "RSG_FUSED_KIND": "auto", "RSG_FUSED_SPW1": "0", "RSG_ENC_PRIO": "0", "RSG_DMA_EW": "2",
    "RSG_DMA_NT": "3", "RSG_DMA_SPW": "8", "RSG_DMA_PRIO": "2", "RSG_DECODE_NET": "1",
    "RSG_NET12_RD": "2", "RSG_HASH_UNAL": "1", "RSG_GET_CACHED": "1",
}


class RsgError(IOError):
    """io::Error::other(...) equivalent carrying the rsg_status code."""

    def __init__(self, code: int, context: str = ""):
        self.code = code
        msg = strerror(code)
        super().__init__(f"{context}: {msg}" if context else msg)


class InvalidDataError(RsgError):
    """io::ErrorKind::InvalidData (inconsistent sources / bitrot mismatch)."""


_lib = None
_lock = threading.Lock()


def load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: the HIP extension is not built "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
        L = ctypes.CDLL(LIB_PATH)
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.rsg_abi_version.restype = I
        L.rsg_strerror.restype = ctypes.c_char_p
        L.rsg_strerror.argtypes = [I]
        L.rsg_device_count.argtypes = [ctypes.POINTER(I)]
        L.rsg_create.argtypes = [I, ctypes.POINTER(P)]
        L.rsg_destroy.argtypes = [P]
        L.rsg_destroy.restype = None
        L.rsg_matrix.argtypes = [I, I, P]
        L.rsg_check_geometry.argtypes = [I, I]
        L.rsg_encode.argtypes = [P, I, I, S, P]
        L.rsg_reconstruct.argtypes = [P, I, I, S, P, P, I]
        L.rsg_verify.argtypes = [P, I, I, S, P, ctypes.POINTER(I)]
        L.rsg_hash.argtypes = [P, I, P, S, P]
        L.rsg_encode_batch_dev.argtypes = [P, I, I, S, S, P, S, S, P, I, P]
        L.rsg_reconstruct_batch_dev.argtypes = [P, I, I, S, S, P, S, S, P, I, P]
        L.rsg_verify_batch_dev.argtypes = [P, I, I, S, S, P, S, S, P, P]
        L.rsg_hash_batch_dev.argtypes = [P, I, P, S, S, S, P, P]
        L.rsg_sync.argtypes = [P, P]
        L.rsg_encode_batch_host.argtypes = [P, I, I, S, S, P, S, S, P, I]
        L.rsg_encode_batch_host_submit.argtypes = [P, I, I, S, S, P, S, S, P, I, ctypes.POINTER(ctypes.c_uint64)]
        L.rsg_poll.argtypes = [P, ctypes.c_uint64, ctypes.POINTER(I)]
        L.rsg_wait.argtypes = [P, ctypes.c_uint64]
        L.rsg_decode_records_dev.argtypes = [P, I, I, S, S, P, I, I, P, P, P]
        L.rsg_heal_records_dev.argtypes = [P, I, I, S, S, P, P, I, P, P, P]
        L.rsg_decode_records_into_dev.argtypes = [P, I, I, S, S, P, I, I, P, S, P, P, P]
        L.rsg_decode_records_submit.argtypes = [P, I, I, S, S, P, I, I, P, P, S, P, P, P,
                                                ctypes.POINTER(ctypes.c_uint64)]
        L.rsg_heal_records_submit.argtypes = [P, I, I, S, S, P, P, I, P, P, ctypes.POINTER(ctypes.c_uint64)]
        L.rsg_bitrot_verify_dev.argtypes = [P, I, S, P, P, S, S, S, P, P]
        L.rsg_pin.argtypes = [P, S]
        L.rsg_unpin.argtypes = [P]
        L.rsg_set_kernel_timing.argtypes = [P, I]
        L.rsg_last_kernel_ms.argtypes = [P, ctypes.POINTER(ctypes.c_float)]
        L.rsg_set_record_engine.argtypes = [P, I]
        L.rsg_test_fail_subbatch.argtypes = [P, I]
        L.rsg_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.rsg_get_tuning.argtypes = [ctypes.c_char_p, ctypes.c_char_p, S]
        _lib = L
        return L


def status_list(status, n: int) -> list:
    """Per-stripe status codes of a ctypes int array as a list, in one C-level
    pass (indexing the ctypes array element by element costs ~0.1 us each:
    0.4 ms per 4096-stripe call, a fifth of a GET call's kernel time)."""
    return memoryview(status).cast("B").cast("i")[:n].tolist() if n else []


def strerror(code: int) -> str:
    return load().rsg_strerror(code).decode()


def check(code: int, context: str = "") -> None:
    if code == RSG_OK:
        return
    if code in (RSG_ERR_INCONSISTENT_SOURCES, RSG_ERR_BITROT_MISMATCH):
        raise InvalidDataError(code, context)
    raise RsgError(code, context)


def get_tuning(name: str) -> str:
    """A kernel-choice knob's current value (rsg_get_tuning)."""
    buf = ctypes.create_string_buffer(32)
    check(load().rsg_get_tuning(name.encode(), buf, len(buf)), f"rsg_get_tuning({name})")
    return buf.value.decode()


def set_tuning(name: str | None, value: str | None) -> None:
    """Set one knob process-wide (value None: its default; name None: every
    knob's default) through rsg_set_tuning."""
    check(load().rsg_set_tuning(name.encode() if name is not None else None,
                                str(value).encode() if value is not None else None),
          f"rsg_set_tuning({name}={value})")


class tuned:
    """`with tuned(RSG_DECODE_NET="0"): ...` — knobs set for the block, every
    one of them back to its previous value afterwards (tests, A/B runs)."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.saved = {}

    def __enter__(self):
        try:
            for k, v in self.knobs.items():
                self.saved[k] = get_tuning(k)
                set_tuning(k, v)
        except Exception:  # a bad name or value: undo the knobs already set, then raise
            self.__exit__()
            raise
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_tuning(k, v)
        return False


class Context:
    """One rsg_ctx (device, stream, scratch).  Thread-safe."""

    def __init__(self, device: int = 0):
        self.device = device
        h = ctypes.c_void_p()
        check(load().rsg_create(device, ctypes.byref(h)), f"rsg_create(device={device})")
        self.handle = h

    def close(self):
        if self.handle:
            load().rsg_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_contexts: dict[int, Context] = {}


def context(device: int | None = None) -> Context:
    if device is None:
        device = int(os.environ.get("RSG_DEVICE", "0"))
    with _lock:
        ctx = _contexts.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _contexts.setdefault(device, ctx)
            ctx = _contexts[device]
    return ctx


def device_count() -> int:
    n = ctypes.c_int(0)
    load().rsg_device_count(ctypes.byref(n))
    return n.value
