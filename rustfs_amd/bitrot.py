"""Per-shard bitrot framing over the GPU HighwayHash-256 kernels.

Mirrors:
  * ``HashAlgorithm`` / ``hash_encode``   crates/utils/src/hash.rs:52-141
  * ``bitrot_shard_file_size``            crates/ecstore/src/erasure/coding/bitrot.rs:593-601
  * ``BitrotWriter.write``                bitrot.rs:464-510  ([hash][block] per block)
  * ``split_and_verify`` / ``BitrotReader.read``   bitrot.rs:139-157, 227-247
  * ``bitrot_verify``                     bitrot.rs:616-655

Digests are computed by librsgpu.so (rsg_hash / rsg_hash_batch_dev).
"""
from __future__ import annotations

import ctypes
import enum
import io

import numpy as np

from . import _lib
from ._lib import InvalidDataError, check


class HashAlgorithm(enum.Enum):
    """Streaming HighwayHash variants used for interleaved bitrot (hash.rs:52-68)."""

    HighwayHash256S = _lib.RSG_HASH_HIGHWAY256S
    HighwayHash256SLegacy = _lib.RSG_HASH_HIGHWAY256S_LEGACY
    NONE = _lib.RSG_HASH_NONE

    def size(self) -> int:
        return 0 if self is HashAlgorithm.NONE else 32

    def hash_encode(self, data, device=None) -> bytes:
        if self is HashAlgorithm.NONE:
            return b""
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else \
            np.ascontiguousarray(data, dtype=np.uint8)
        out = (ctypes.c_uint8 * 32)()
        check(_lib.load().rsg_hash(_lib.context(device).handle, self.value, a.ctypes.data if a.size else None,
                                   a.size, out), "bitrot hash")
        return bytes(out)


def bitrot_shard_file_size(size: int, shard_size: int, algo: HashAlgorithm) -> int:
    if algo not in (HashAlgorithm.HighwayHash256S, HashAlgorithm.HighwayHash256SLegacy):
        return size
    return -(-size // shard_size) * algo.size() + size


class BitrotWriter:
    """Writes ``[hash][block]`` per block to a binary sink (bitrot.rs:464-510)."""

    def __init__(self, sink, shard_size: int, algo: HashAlgorithm = HashAlgorithm.HighwayHash256S):
        self.sink = sink
        self.shard_size = shard_size
        self.algo = algo
        self.finished = False

    def write(self, buf) -> int:
        if len(buf) == 0:
            return 0
        if self.finished:
            raise ValueError("bitrot writer already finished")
        if len(buf) > self.shard_size:
            raise ValueError(f"data size {len(buf)} exceeds shard size {self.shard_size}")
        if len(buf) < self.shard_size:
            self.finished = True
        if self.algo.size():
            self.sink.write(self.algo.hash_encode(buf))
        self.sink.write(bytes(buf))
        return len(buf)


def split_and_verify(algo: HashAlgorithm, block: bytes, skip_verify: bool = False) -> bytes:
    h, data = block[: algo.size()], block[algo.size():]
    if not skip_verify and algo.hash_encode(data) != h:
        raise InvalidDataError(_lib.RSG_ERR_BITROT_MISMATCH)
    return data


class BitrotReader:
    """Reads ``[hash][block]`` blocks and verifies before returning (bitrot.rs:139-157)."""

    def __init__(self, src, shard_size: int, algo: HashAlgorithm = HashAlgorithm.HighwayHash256S,
                 skip_verify: bool = False):
        self.src = src
        self.shard_size = shard_size
        self.algo = algo
        self.skip_verify = skip_verify

    def read(self, want: int) -> bytes:
        if want > self.shard_size:
            raise ValueError(f"read size {want} exceeds shard size {self.shard_size}")
        need = self.algo.size() + want
        block = self.src.read(need)
        if len(block) < need:
            raise EOFError("bitrot short shard read")
        return split_and_verify(self.algo, block, self.skip_verify)


def bitrot_verify(r, want_size: int, part_size: int, algo: HashAlgorithm, shard_size: int) -> None:
    """Whole-shard-file verification (bitrot.rs:616-655)."""
    if want_size != bitrot_shard_file_size(part_size, shard_size, algo):
        raise IOError("bitrot shard file size mismatch")
    left = want_size
    hs = algo.size()
    while left > 0:
        h = r.read(hs)
        if len(h) < hs:
            raise EOFError("unexpected eof")
        left -= hs
        shard_size = min(shard_size, left)
        buf = r.read(shard_size)
        if len(buf) < shard_size:
            raise EOFError("unexpected eof")
        if algo.hash_encode(buf) != h:
            raise IOError("bitrot hash mismatch")
        left -= shard_size
    if r.read(1):
        raise IOError("bitrot shard file has trailing data")


def bitrot_verify_batch(files, want_size: int, part_size: int, algo: HashAlgorithm, shard_size: int,
                        stream=None) -> list:
    """Device-batch whole-shard-file verification (rsg_bitrot_verify_dev):
    `files` are cuda uint8 tensors holding complete shard files of one part.
    Returns one rsg_status per file with bitrot_verify's decision order
    (bitrot.rs:616-655): size mismatch, first bad record, early EOF, trailing
    data.  `raise_for_status` turns a status into the reference's error."""
    import torch
    n = len(files)
    dev = None
    for f in files:
        if f.dtype != torch.uint8 or not f.is_cuda or not f.is_contiguous():
            raise TypeError("files must be contiguous cuda uint8 tensors")
        dev = f.device
    if n == 0:
        return []
    ptrs = (ctypes.c_void_p * n)(*[f.data_ptr() if f.numel() else None for f in files])
    lens = (ctypes.c_size_t * n)(*[f.numel() for f in files])
    status = (ctypes.c_int * n)()
    s = stream.cuda_stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.load().rsg_bitrot_verify_dev(
        _lib.context(dev.index or 0).handle, algo.value, n, ptrs, lens, want_size, part_size, shard_size, status,
        s), "bitrot_verify")
    return _lib.status_list(status, n)


def raise_for_status(code: int) -> None:
    """bitrot_verify's error for an rsg_bitrot_verify_dev status."""
    if code == _lib.RSG_OK:
        return
    if code == _lib.RSG_ERR_UNEXPECTED_EOF:
        raise EOFError("unexpected eof")
    raise IOError(_lib.strerror(code))


def frame_shards(shards, digests) -> list:
    """encode_inline_shards layout: one ``[hash][shard]`` bytes object per shard
    (encode.rs:601-628), from shard bytes and their 32-byte digests."""
    return [bytes(d) + bytes(s) for s, d in zip(shards, digests)]


__all__ = ["HashAlgorithm", "bitrot_shard_file_size", "BitrotWriter", "BitrotReader", "split_and_verify",
           "bitrot_verify", "bitrot_verify_batch", "raise_for_status", "frame_shards", "io"]
