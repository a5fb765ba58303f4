"""Host-side mirror of rustfs's erasure codec surface, running on librsgpu.so.

Mirrors, name for name and error for error:
  * ``Erasure``            crates/ecstore/src/erasure/coding/erasure.rs:617-1095
  * ``ReedSolomonEncoder`` erasure.rs:358-446
  * ``calc_shard_size``    erasure.rs:655
  * ``RustfsCodecDecodeEngine.reconstruct_into``  crates/ecstore/src/erasure/codec/bridge.rs:274-307

Every GF(2^8) byte is computed by the HIP kernels behind include/rsgpu.h; this
module only validates, marshals pointers and maps status codes to exceptions.
The device-batch entry points (``*_batch``) take torch uint8 tensors resident
on the GPU and run asynchronously on the current torch stream.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import InvalidDataError, RsgError, check

MODERN_MAX_TOTAL_SHARDS = 256  # galois_8::Field::ORDER, erasure.rs:72


# ---------------------------------------------------------------------------
# ErasureConstructionError (erasure.rs:87-121)

class ErasureConstructionError(ValueError):
    pass


class ZeroDataShards(ErasureConstructionError):
    def __init__(self):
        super().__init__("data_shards must be greater than zero")


class ZeroBlockSize(ErasureConstructionError):
    def __init__(self):
        super().__init__("block_size must be greater than zero")


class UnsupportedModernShardCount(ErasureConstructionError):
    def __init__(self, data_shards: int, parity_shards: int):
        super().__init__(f"modern codec does not support {data_shards} data shards and {parity_shards} parity shards")


def calc_shard_size(block_size: int, data_shards: int) -> int:
    """erasure.rs:655 — plain ceiling division (MinIO-compatible sizing)."""
    return -(-block_size // data_shards)


def _as_array(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return buf
    return np.frombuffer(buf, dtype=np.uint8)


def _ptrs(arrs: Sequence[np.ndarray]):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data if a.size else 0 for a in arrs])


def _writable(buf) -> np.ndarray:
    a = _as_array(buf)
    if not a.flags.writeable:
        raise TypeError("shard buffer is read-only; pass bytearray / numpy arrays")
    return a


def _shard_view(buf) -> np.ndarray:
    """A shard as the flat uint8 byte run the C ABI reads and writes through
    one pointer: a strided view (buf[:, i]) or another dtype would make the
    library touch bytes outside the caller's shard, so those are rejected."""
    a = _as_array(buf)
    if a.dtype != np.uint8 or not a.flags.c_contiguous:
        raise TypeError("shard buffers must be C-contiguous uint8 (bytes, bytearray or numpy uint8 arrays)")
    return a


# ---------------------------------------------------------------------------

class ReedSolomonEncoder:
    """ReedSolomonEncoder (erasure.rs:358-446) over the GPU codec."""

    def __init__(self, data_shards: int, parity_shards: int, device: Optional[int] = None):
        st = _lib.load().rsg_check_geometry(data_shards, parity_shards)
        if st != _lib.RSG_OK:
            raise RsgError(st, "Failed to create Reed-Solomon encoder")
        self.data_shards = data_shards
        self.parity_shards = parity_shards
        self._device = device

    @property
    def total(self) -> int:
        return self.data_shards + self.parity_shards

    def _ctx(self):
        return _lib.context(self._device)

    def encode(self, shards: List) -> None:
        """In place: shards[k..k+m) overwritten with parity (erasure.rs:396-408)."""
        if len(shards) == 0 or self.parity_shards == 0:
            return
        if len(shards) != self.total:
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT, "Reed-Solomon encode failed")
        arrs = [_shard_view(s) for s in shards]
        n = arrs[0].size
        if any(a.size != n for a in arrs):
            raise RsgError(_lib.RSG_ERR_INCONSISTENT_LENGTH, "Reed-Solomon encode failed")
        for a in arrs[self.data_shards:]:
            _writable(a)
        check(_lib.load().rsg_encode(self._ctx().handle, self.data_shards, self.parity_shards, n, _ptrs(arrs)),
              "Reed-Solomon encode failed")

    def _reconstruct(self, shards: List, mode: int) -> None:
        if len(shards) != self.total:
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT,
                           f"invalid shard count: got {len(shards)}, expected {self.total}")
        present = [s is not None for s in shards]
        lens = {len(s) for s in shards if s is not None}
        if len(lens) > 1:
            raise RsgError(_lib.RSG_ERR_INCONSISTENT_LENGTH, "Reed-Solomon reconstruct failed")
        n = lens.pop() if lens else 0
        if n == 0:
            # recover_empty_payload_data_shards (erasure.rs:563-594 / bridge.rs:54-84)
            st = _lib.load().rsg_reconstruct(self._ctx().handle, self.data_shards, self.parity_shards, 0,
                                             None, (ctypes.c_uint8 * self.total)(*present), mode)
            check(st, "Reed-Solomon reconstruct failed")
            fill = range(self.data_shards) if mode == _lib.RSG_RECONSTRUCT_DATA else range(self.total)
            for i in fill:
                if shards[i] is None and (i < self.data_shards or mode != _lib.RSG_RECONSTRUCT_DATA):
                    shards[i] = bytearray()
            return
        if self.parity_shards == 0:
            return
        arrs = []
        for i, s in enumerate(shards):
            is_parity = i >= self.data_shards
            if s is None:
                s = bytearray(n)  # Option::None -> freshly allocated Vec (filled by the codec)
                if not is_parity or mode != _lib.RSG_RECONSTRUCT_DATA:
                    shards[i] = s
            elif is_parity and mode == _lib.RSG_RECONSTRUCT_REENCODE_PARITY and not _as_array(s).flags.writeable:
                s = bytearray(s)  # re-encoded parity replaces the present buffer
                shards[i] = s
            arrs.append(_shard_view(s))
        st = _lib.load().rsg_reconstruct(self._ctx().handle, self.data_shards, self.parity_shards, n,
                                         _ptrs(arrs), (ctypes.c_uint8 * self.total)(*present), mode)
        check(st, "Reed-Solomon reconstruct failed")

    def reconstruct_data(self, shards: List) -> None:
        """erasure.rs:411-422: rebuild missing data shards (parity stays None)."""
        self._reconstruct(shards, _lib.RSG_RECONSTRUCT_DATA)

    def reconstruct(self, shards: List) -> None:
        """erasure.rs:425-428: reconstruct_data then re-encode every parity shard."""
        self._reconstruct(shards, _lib.RSG_RECONSTRUCT_REENCODE_PARITY)

    def reconstruct_opt(self, shards: List) -> None:
        """reconstruct_opt (bridge.rs:296): rebuild every missing shard."""
        self._reconstruct(shards, _lib.RSG_RECONSTRUCT_MISSING)

    def verify(self, shards: Sequence) -> bool:
        """erasure.rs:430-441."""
        if all(len(s) == 0 for s in shards):
            return True
        if self.parity_shards == 0:
            return True
        if len(shards) != self.total:
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT, "Reed-Solomon verify failed")
        arrs = [np.ascontiguousarray(_as_array(s)) for s in shards]
        n = arrs[0].size
        if any(a.size != n for a in arrs):
            raise RsgError(_lib.RSG_ERR_INCONSISTENT_LENGTH, "Reed-Solomon verify failed")
        ok = ctypes.c_int(0)
        check(_lib.load().rsg_verify(self._ctx().handle, self.data_shards, self.parity_shards, n, _ptrs(arrs),
                                     ctypes.byref(ok)), "Reed-Solomon verify failed")
        return bool(ok.value)


# ---------------------------------------------------------------------------

class Erasure:
    """Erasure (erasure.rs:617-1095), modern GF(2^8) backend only."""

    def __init__(self, data_shards: int, parity_shards: int, block_size: int, device: Optional[int] = None):
        if data_shards == 0:
            raise ZeroDataShards()
        if block_size == 0:
            raise ZeroBlockSize()
        if parity_shards > 0 and data_shards + parity_shards > MODERN_MAX_TOTAL_SHARDS:
            raise UnsupportedModernShardCount(data_shards, parity_shards)
        self.data_shards = data_shards
        self.parity_shards = parity_shards
        self.block_size = block_size
        self.encoder = ReedSolomonEncoder(data_shards, parity_shards, device) if parity_shards > 0 else None
        self._device = device

    try_new = classmethod(lambda cls, k, m, b, device=None: cls(k, m, b, device))

    # -- geometry (erasure.rs:1021-1095) --
    def total_shard_count(self) -> int:
        return self.data_shards + self.parity_shards

    def shard_size(self) -> int:
        return calc_shard_size(self.block_size, self.data_shards)

    def has_valid_dimensions(self) -> bool:
        return self.block_size > 0 and self.data_shards > 0

    def shard_file_size(self, total_length: int) -> int:
        if total_length == 0:
            return 0
        if total_length < 0:
            return total_length
        num_shards = total_length // self.block_size
        last = total_length % self.block_size
        return num_shards * self.shard_size() + calc_shard_size(last, self.data_shards)

    def shard_file_offset(self, start_offset: int, length: int, total_length: int) -> int:
        shard_size = self.shard_size()
        shard_file_size = self.shard_file_size(total_length)
        end_shard = (start_offset + length) // self.block_size
        till = end_shard * shard_size + shard_size
        return min(till, shard_file_size)

    # -- encode (erasure.rs:784-887) --
    def encode_buffer(self, data) -> np.ndarray:
        """Copy + zero-pad to (k+m)*S and encode; returns the (k+m, S) stripe."""
        data = _as_array(data)
        per_shard = calc_shard_size(data.size, self.data_shards)
        if per_shard == 0:
            return np.zeros((self.total_shard_count(), 0), dtype=np.uint8)
        buf = np.zeros((self.total_shard_count(), per_shard), dtype=np.uint8)
        buf.reshape(-1)[: data.size] = data
        if self.encoder is not None:
            self.encoder.encode([buf[i] for i in range(self.total_shard_count())])
        return buf

    def encode_data(self, data) -> List[bytes]:
        buf = self.encode_buffer(data)
        return [buf[i].tobytes() for i in range(buf.shape[0])]

    def encode_inline_shards(self, data) -> List[bytes]:
        """encode_inline_shards_with_size_hint (encode.rs:601-628): encode one
        small object and return each shard as its BitrotWriter payload
        ``[HighwayHash256S(shard)][shard]`` (empty list for an empty object).
        Parity and all k+m digests come from one rsg_encode_batch_host call
        (fused encode + hash on the device)."""
        data = _as_array(data)
        if data.size == 0:
            return []
        per_shard = calc_shard_size(data.size, self.data_shards)
        t = self.total_shard_count()
        buf = np.zeros((1, t, per_shard), dtype=np.uint8)
        buf.reshape(-1)[: data.size] = data
        dig = np.zeros((1, t, 32), dtype=np.uint8)
        if self.parity_shards:
            self.encode_batch_host(buf, dig)
        else:
            from .bitrot import HashAlgorithm
            for i in range(t):
                dig[0, i] = np.frombuffer(HashAlgorithm.HighwayHash256S.hash_encode(buf[0, i], self._device), np.uint8)
        return [dig[0, i].tobytes() + buf[0, i].tobytes() for i in range(t)]

    # -- decode (erasure.rs:897-1019) --
    def decode_data(self, shards: List) -> None:
        if self.encoder is not None:
            self.encoder.reconstruct_data(shards)

    def decode_data_and_parity(self, shards: List) -> None:
        if self.encoder is not None:
            self.encoder.reconstruct(shards)

    def decode_data_with_reconstruction_verification(self, shards: List) -> None:
        k = self.data_shards
        missing_data = any(s is None for s in shards[:k])
        available = sum(s is not None for s in shards)
        source_parity = []
        if missing_data and available > k:
            source_parity = [(i, bytes(s)) for i, s in enumerate(shards) if i >= k and s is not None]
        if not source_parity:
            self.decode_data(shards)
            return
        self.decode_data_and_parity(shards)
        for i, src in source_parity:
            if shards[i] is None:
                raise InvalidDataError(_lib.RSG_ERR_INCONSISTENT_SOURCES,
                                       "missing rebuilt parity shard after read verification")
            if bytes(shards[i]) != src:
                raise InvalidDataError(_lib.RSG_ERR_INCONSISTENT_SOURCES)

    def verify_data_and_parity(self, shards: Sequence) -> bool:
        if len(shards) != self.total_shard_count():
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT,
                           f"invalid shard count: got {len(shards)}, expected {self.total_shard_count()}")
        if self.parity_shards == 0:
            return True
        for i, s in enumerate(shards):
            if s is None:
                raise RsgError(_lib.RSG_ERR_INVALID_ARG, f"missing shard {i} for data/parity verification")
        return self.encoder.verify(shards)

    # -- device batches (the GPU dispatch point of encode_batched, encode.rs:795-919) --
    def encode_batch(self, stripes, digests=None, algo: int = _lib.RSG_HASH_HIGHWAY256S, stream=None) -> None:
        """stripes: cuda uint8 tensor (n, k+m, S) in the a3 layout; parity written
        in place.  digests: optional (n, k+m, 32) tensor for the fused HH256S."""
        n, t, S = _check_batch(stripes, self.total_shard_count())
        d = digests.data_ptr() if digests is not None else None
        check(_lib.load().rsg_encode_batch_dev(
            _lib.context(_device_of(stripes)).handle, self.data_shards, self.parity_shards, S, n,
            stripes.data_ptr(), S, t * S, d, algo if d else _lib.RSG_HASH_NONE, _stream_of(stripes, stream)),
            "Reed-Solomon encode failed")

    def encode_batch_host(self, stripes: np.ndarray, digests: Optional[np.ndarray] = None,
                          algo: int = _lib.RSG_HASH_HIGHWAY256S) -> None:
        """Host-memory batch (n, k+m, S) uint8, parity written in place; pipelined
        H2D -> encode(+digests) -> D2H inside librsgpu (rsg_encode_batch_host)."""
        n, t, S, d = self._host_batch_args(stripes, digests)
        check(_lib.load().rsg_encode_batch_host(
            _lib.context(self._device).handle, self.data_shards, self.parity_shards, S, n, stripes.ctypes.data,
            S, t * S, d, algo if d else _lib.RSG_HASH_NONE), "Reed-Solomon encode failed")

    def encode_batch_host_submit(self, stripes: np.ndarray, digests: Optional[np.ndarray] = None,
                                 algo: int = _lib.RSG_HASH_HIGHWAY256S) -> "HostBatchTicket":
        """Asynchronous encode_batch_host (rsg_encode_batch_host_submit): returns
        at once with a ticket; the arrays must stay alive and untouched until
        the ticket is done (poll() / wait()).  Jobs run in submission order and
        overlap each other's copies and kernels (encode_batched's bounded
        in-flight queue, encode.rs:64-72, 795-919)."""
        n, t, S, d = self._host_batch_args(stripes, digests)
        tk = ctypes.c_uint64(0)
        ctx = _lib.context(self._device)
        check(_lib.load().rsg_encode_batch_host_submit(
            ctx.handle, self.data_shards, self.parity_shards, S, n, stripes.ctypes.data, S, t * S, d,
            algo if d else _lib.RSG_HASH_NONE, ctypes.byref(tk)), "Reed-Solomon encode failed")
        return HostBatchTicket(ctx, tk.value, (stripes, digests))

    def _host_batch_args(self, stripes, digests):
        if stripes.dtype != np.uint8 or stripes.ndim != 3 or not stripes.flags.c_contiguous:
            raise TypeError("stripes must be a C-contiguous uint8 array (n, k+m, S)")
        n, t, S = stripes.shape
        if t != self.total_shard_count():
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT, f"invalid shard count: got {t}")
        d = None
        if digests is not None:
            if digests.shape != (n, t, 32) or digests.dtype != np.uint8 or not digests.flags.c_contiguous:
                raise TypeError("digests must be a C-contiguous uint8 array (n, k+m, 32)")
            d = digests.ctypes.data
        return n, t, S, d

    def _record_files(self, files: Sequence, shard_len: int, n: int):
        """Validate the GET's record files; returns (device, ctypes pointer array)."""
        import torch
        t = self.total_shard_count()
        if len(files) != t:
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT, f"invalid shard count: got {len(files)}")
        rec = 32 + shard_len
        dev = None
        for f in files:
            if f is not None:
                if f.dtype != torch.uint8 or not f.is_cuda or not f.is_contiguous() or f.numel() < n * rec:
                    raise TypeError("each file must be a contiguous cuda uint8 tensor of n records")
                dev = f.device
        if dev is None:
            raise RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, "no shard available")
        return dev, (ctypes.c_void_p * t)(*[f.data_ptr() if f is not None else None for f in files])

    def _slots(self, targets, shard_len: int, n: int, dev, target_stride: Optional[int]):
        """The in-place GET's k data-shard slots: None -> a new (n, k*S) block
        tensor (slot i = columns [i*S, (i+1)*S)); a 2-D (n, k*S) tensor, the
        same layout; or k tensors with `target_stride` bytes between stripes
        (default S).  Returns (keep, ctypes pointer array, stride)."""
        import torch
        k = self.data_shards
        if targets is None:
            targets = torch.empty((n, k * shard_len), dtype=torch.uint8, device=dev)
        if isinstance(targets, torch.Tensor):
            if targets.dtype != torch.uint8 or not targets.is_cuda or not targets.is_contiguous() \
                    or targets.numel() < n * k * shard_len:
                raise TypeError("targets must be a contiguous cuda uint8 tensor (n, k*shard_len)")
            base = targets.data_ptr()
            return targets, (ctypes.c_void_p * k)(*[base + i * shard_len for i in range(k)]), k * shard_len
        if len(targets) != k:
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT, f"invalid slot count: got {len(targets)}, expected {k}")
        stride = shard_len if target_stride is None else target_stride
        for tg in targets:
            if tg is None or tg.dtype != torch.uint8 or not tg.is_cuda or not tg.is_contiguous() \
                    or (n and tg.numel() < (n - 1) * stride + shard_len):
                raise TypeError("each slot must be a contiguous cuda uint8 tensor of n strided shards")
        return targets, (ctypes.c_void_p * k)(*[tg.data_ptr() for tg in targets]), stride

    @staticmethod
    def _stream_handle(stream, dev):
        import torch
        if stream is None:
            return torch.cuda.current_stream(dev).cuda_stream
        return stream if isinstance(stream, int) else stream.cuda_stream

    def decode_records_batch(self, files: Sequence, shard_len: int, n: int, verify_surplus: bool = True,
                             algo: int = _lib.RSG_HASH_HIGHWAY256S, out=None, stream=None):
        """GET engine, gather form (rsg_decode_records_dev, deprecated since ABI
        6: decode_records_into_batch is the reference's form): `files[i]` is a
        cuda uint8 tensor holding shard i's n BitrotWriter records ([32-byte
        digest][shard_len]) or None.  Returns (data (n, k*shard_len) tensor,
        per-stripe status list)."""
        import torch
        dev, ptrs = self._record_files(files, shard_len, n)
        if out is None:
            out = torch.empty((n, self.data_shards * shard_len), dtype=torch.uint8, device=dev)
        status = (ctypes.c_int * max(n, 1))()
        check(_lib.load().rsg_decode_records_dev(
            _lib.context(dev.index or 0).handle, self.data_shards, self.parity_shards, shard_len, n, ptrs, algo,
            1 if verify_surplus else 0, out.data_ptr(), status, self._stream_handle(stream, dev)),
            "RustFS codec reconstruct failed")
        return out, _lib.status_list(status, n)

    def decode_records_into_batch(self, files: Sequence, shard_len: int, n: int, targets=None,
                                  target_stride: Optional[int] = None, verify_surplus: bool = True,
                                  algo: int = _lib.RSG_HASH_HIGHWAY256S, stream=None):
        """GET engine, in-place form (rsg_decode_records_into_dev): the
        reference's reconstruct_into contract (bridge.rs:274-307) — a data
        shard whose record verifies is served from that record and never
        copied; only the shards no verified record serves (file absent or
        record rotten) are rebuilt, into their slot (`targets`, see _slots).
        Returns (slots, src, status): src is a (k, n) bool array, True where
        data shard i of stripe s is the body of files[i]'s record s, False
        where it was written to slot i."""
        dev, ptrs = self._record_files(files, shard_len, n)
        slots, tptr, stride = self._slots(targets, shard_len, n, dev, target_stride)
        k = self.data_shards
        src = np.ones((k, max(n, 1)), dtype=np.uint8)
        status = (ctypes.c_int * max(n, 1))()
        check(_lib.load().rsg_decode_records_into_dev(
            _lib.context(dev.index or 0).handle, k, self.parity_shards, shard_len, n, ptrs, algo,
            1 if verify_surplus else 0, tptr, stride, src.ctypes.data, status, self._stream_handle(stream, dev)),
            "RustFS codec reconstruct failed")
        return slots, src[:, :n].astype(bool), _lib.status_list(status, n)

    def decode_records_submit(self, files: Sequence, shard_len: int, n: int, out=None, targets=None,
                              target_stride: Optional[int] = None, inplace: bool = False,
                              verify_surplus: bool = True, algo: int = _lib.RSG_HASH_HIGHWAY256S,
                              stream=None) -> "RecordTicket":
        """Asynchronous GET (rsg_decode_records_submit): returns at once; the
        ticket's wait() gives what the synchronous form returns — (data,
        status) for the gather form, (slots, src, status) with inplace=True."""
        import torch
        dev, ptrs = self._record_files(files, shard_len, n)
        k = self.data_shards
        status = (ctypes.c_int * max(n, 1))()
        src = np.ones((k, max(n, 1)), dtype=np.uint8) if inplace else None
        if inplace:
            slots, tptr, stride = self._slots(targets, shard_len, n, dev, target_stride)
            d_out, keep = None, slots
        else:
            if out is None:
                out = torch.empty((n, k * shard_len), dtype=torch.uint8, device=dev)
            d_out, tptr, stride, keep = out.data_ptr(), None, 0, out
        tk = ctypes.c_uint64(0)
        ctx = _lib.context(dev.index or 0)
        check(_lib.load().rsg_decode_records_submit(
            ctx.handle, k, self.parity_shards, shard_len, n, ptrs, algo, 1 if verify_surplus else 0, d_out, tptr,
            stride, src.ctypes.data if inplace else None, status, self._stream_handle(stream, dev),
            ctypes.byref(tk)), "RustFS codec reconstruct failed")

        def result():
            st = _lib.status_list(status, n)
            return (keep, src[:, :n].astype(bool), st) if inplace else (keep, st)
        return RecordTicket(ctx, tk.value, (files, keep, ptrs, tptr, status, src), result,
                            "RustFS codec reconstruct failed")

    def heal_records_submit(self, files: Sequence, targets: Sequence, shard_len: int, n: int,
                            algo: int = _lib.RSG_HASH_HIGHWAY256S, stream=None) -> "RecordTicket":
        """Asynchronous heal (rsg_heal_records_submit); wait() returns the
        per-stripe status list of heal_records_batch."""
        dev, src, dst = self._heal_args(files, targets, shard_len, n)
        status = (ctypes.c_int * max(n, 1))()
        tk = ctypes.c_uint64(0)
        ctx = _lib.context(dev.index or 0)
        check(_lib.load().rsg_heal_records_submit(
            ctx.handle, self.data_shards, self.parity_shards, shard_len, n, src, dst, algo, status,
            self._stream_handle(stream, dev), ctypes.byref(tk)), "erasure heal")
        return RecordTicket(ctx, tk.value, (files, targets, src, dst, status),
                            lambda: _lib.status_list(status, n), "erasure heal")

    def _heal_args(self, files, targets, shard_len, n):
        import torch
        t = self.total_shard_count()
        if len(files) != t or len(targets) != t:
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT,
                           f"invalid shard count: got {len(files)}/{len(targets)}, expected {t}")
        rec = 32 + shard_len
        dev = None
        for f in list(files) + list(targets):
            if f is not None:
                if f.dtype != torch.uint8 or not f.is_cuda or not f.is_contiguous() or f.numel() < n * rec:
                    raise TypeError("files/targets must be contiguous cuda uint8 tensors of n records")
                dev = f.device
        if dev is None:
            raise RsgError(_lib.RSG_ERR_INVALID_ARG, "invalid argument")
        src = (ctypes.c_void_p * t)(*[f.data_ptr() if f is not None else None for f in files])
        dst = (ctypes.c_void_p * t)(*[f.data_ptr() if f is not None else None for f in targets])
        return dev, src, dst

    def heal_records_batch(self, files: Sequence, targets: Sequence, shard_len: int, n: int,
                           algo: int = _lib.RSG_HASH_HIGHWAY256S, work=None, stream=None):
        """Batched heal (rsg_heal_records_dev; Erasure::heal, heal.rs:112-206).
        `work` is accepted for compatibility and unused (ABI 3).

        `files[i]`: cuda uint8 tensor with shard i's n BitrotWriter records, or
        None (no reader).  `targets[i]`: cuda uint8 tensor of n*(32+shard_len)
        bytes that receives the rebuilt records of shard i, or None (no
        writer).  Returns the per-stripe status list (RSG_OK,
        RSG_ERR_TOO_FEW_SHARDS = read quorum, RSG_ERR_INCONSISTENT_SOURCES)."""
        dev, src, dst = self._heal_args(files, targets, shard_len, n)
        status = (ctypes.c_int * max(n, 1))()
        check(_lib.load().rsg_heal_records_dev(
            _lib.context(dev.index or 0).handle, self.data_shards, self.parity_shards, shard_len, n, src, dst,
            algo, work.data_ptr() if work is not None else None, status, self._stream_handle(stream, dev)),
            "erasure heal")
        return _lib.status_list(status, n)

    def reconstruct_batch(self, stripes, present: Sequence[bool], mode: int = _lib.RSG_RECONSTRUCT_MISSING,
                          stream=None) -> None:
        n, t, S = _check_batch(stripes, self.total_shard_count())
        pres = (ctypes.c_uint8 * t)(*[1 if p else 0 for p in present])
        check(_lib.load().rsg_reconstruct_batch_dev(
            _lib.context(_device_of(stripes)).handle, self.data_shards, self.parity_shards, S, n,
            stripes.data_ptr(), S, t * S, pres, mode, _stream_of(stripes, stream)),
            "Reed-Solomon reconstruct failed")

    def verify_batch(self, stripes, stream=None):
        import torch
        n, t, S = _check_batch(stripes, self.total_shard_count())
        ok = torch.empty(n, dtype=torch.uint8, device=stripes.device)
        check(_lib.load().rsg_verify_batch_dev(
            _lib.context(_device_of(stripes)).handle, self.data_shards, self.parity_shards, S, n,
            stripes.data_ptr(), S, t * S, ok.data_ptr(), _stream_of(stripes, stream)),
            "Reed-Solomon verify failed")
        return ok


class HostBatchTicket:
    """A submitted host-batch encode (rsg_encode_batch_host_submit).  Holds
    references to the job's arrays until it completes."""

    def __init__(self, ctx, ticket: int, keep):
        self._ctx = ctx
        self.ticket = ticket
        self._keep = keep
        self._done = False

    def poll(self) -> bool:
        """True once the job has finished (raises its error, if any)."""
        if self._done:
            return True
        done = ctypes.c_int(0)
        st = _lib.load().rsg_poll(self._ctx.handle, self.ticket, ctypes.byref(done))
        if done.value:  # finished (successfully or not): nothing writes into the arrays any more
            self._done, self._keep = True, None
        check(st, "Reed-Solomon encode failed")
        return self._done

    def wait(self) -> None:
        if self._done:
            return
        st = _lib.load().rsg_wait(self._ctx.handle, self.ticket)
        self._done, self._keep = True, None
        check(st, "Reed-Solomon encode failed")

    def __del__(self):  # never leave a job writing into freed arrays
        try:
            if not self._done:
                self.wait()
        except Exception:
            pass


class RecordTicket:
    """A submitted GET or heal (rsg_decode_records_submit /
    rsg_heal_records_submit).  Holds the call's buffers and status arrays
    until it completes; wait() returns what the synchronous call returns."""

    def __init__(self, ctx, ticket: int, keep, result, what: str):
        self._ctx = ctx
        self.ticket = ticket
        self._keep = keep
        self._result = result
        self._what = what
        self._done = False
        self._value = None
        self._error = None

    def _complete(self, st: int) -> None:
        self._done = True
        try:
            check(st, self._what)
            self._value = self._result()
        except RsgError as err:
            self._error = err
        self._keep = None

    def poll(self) -> bool:
        if not self._done:
            done = ctypes.c_int(0)
            st = _lib.load().rsg_poll(self._ctx.handle, self.ticket, ctypes.byref(done))
            if not done.value:
                check(st, self._what)
                return False
            self._complete(st)
        return True

    def wait(self):
        if not self._done:
            self._complete(_lib.load().rsg_wait(self._ctx.handle, self.ticket))
        if self._error is not None:
            raise self._error
        return self._value

    def __del__(self):  # never leave a job reading or writing freed buffers
        try:
            if not self._done:
                self._complete(_lib.load().rsg_wait(self._ctx.handle, self.ticket))
        except Exception:
            pass


# ---------------------------------------------------------------------------
# The GET decode-engine seam (crates/ecstore/src/erasure/codec/bridge.rs:33-50):
# a GPU arm beside RustfsCodecDecodeEngine (bridge.rs:137-307), same outcome
# labels, same error messages.

GET_RECONSTRUCT_OUTCOME_SKIP_DATA_COMPLETE = "skip_data_complete"  # bridge.rs:25
GET_RECONSTRUCT_OUTCOME_SKIP_EMPTY_PAYLOAD = "skip_empty_payload"  # bridge.rs:26
GET_RECONSTRUCT_OUTCOME_GPU_CALLED = "rsgpu_called"


class GpuDecodeWorkspace:
    """RustfsCodecDecodeWorkspace's role: carries the shard length the engine
    was prepared for (the device buffers live in the library's context)."""

    def __init__(self, shard_len: int):
        self._shard_len = shard_len

    def shard_len(self) -> int:
        return self._shard_len


class GpuCodecDecodeEngine:
    """ErasureDecodeEngine (bridge.rs:33-50) on librsgpu, with
    RustfsCodecDecodeEngine::reconstruct_into's semantics (bridge.rs:274-307):
    data complete -> skip; all-empty payload -> empty data shards; a missing
    data shard with more than k shards available -> rebuild every missing
    shard and verify the whole set (InvalidData "inconsistent read source
    shards", bridge.rs:202-236); otherwise rebuild the missing data only."""

    def __init__(self, erasure: Erasure):
        self.erasure = erasure
        self._enc = ReedSolomonEncoder(erasure.data_shards, erasure.parity_shards, erasure._device) \
            if erasure.parity_shards else None

    def data_shards(self) -> int:
        return self.erasure.data_shards

    def parity_shards(self) -> int:
        return self.erasure.parity_shards

    def block_size(self) -> int:
        return self.erasure.block_size

    def engine_name(self) -> str:
        return "rsgpu"

    def supports_progressive_decode(self) -> bool:
        return False

    def supports_aligned_shards(self) -> bool:
        return False

    def prepare_workspace(self, shard_len: int) -> GpuDecodeWorkspace:
        return GpuDecodeWorkspace(shard_len)

    def reconstruct_into(self, shards: List, workspace: Optional[GpuDecodeWorkspace] = None) -> str:
        k, m = self.erasure.data_shards, self.erasure.parity_shards
        if len(shards) >= k and all(s is not None for s in shards[:k]):  # data_shards_complete, bridge.rs:52
            return GET_RECONSTRUCT_OUTCOME_SKIP_DATA_COMPLETE
        if len(shards) != k + m:  # recover_empty_payload_data_shards, bridge.rs:56-84
            raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT,
                           f"invalid shard count: got {len(shards)}, expected {k + m}")
        present = [s for s in shards if s is not None]
        if present and all(len(s) == 0 for s in present) and len(present) >= k:
            for i in range(k):
                if shards[i] is None:
                    shards[i] = bytearray()
            return GET_RECONSTRUCT_OUTCOME_SKIP_EMPTY_PAYLOAD
        if self._enc is not None:
            needs_verification = any(s is None for s in shards[:k]) and len(present) > k
            try:
                if needs_verification:
                    self._enc.reconstruct_opt(shards)
                else:
                    self._enc.reconstruct_data(shards)
            except RsgError as err:
                raise RsgError(err.code, "RustFS codec reconstruct failed") from err
            if needs_verification and not self._enc.verify(shards):
                raise InvalidDataError(_lib.RSG_ERR_INCONSISTENT_SOURCES)
        return GET_RECONSTRUCT_OUTCOME_GPU_CALLED


def _check_batch(stripes, total: int):
    if stripes.dtype.__str__() != "torch.uint8" or stripes.dim() != 3 or not stripes.is_contiguous():
        raise TypeError("stripes must be a contiguous uint8 tensor of shape (n, k+m, S)")
    if not stripes.is_cuda:
        raise TypeError("stripes must be device-resident (the batch path is GPU only)")
    n, t, S = stripes.shape
    if t != total:
        raise RsgError(_lib.RSG_ERR_INVALID_SHARD_COUNT, f"invalid shard count: got {t}, expected {total}")
    return int(n), int(t), int(S)


def _device_of(t) -> int:
    return t.device.index if t.device.index is not None else 0


def _stream_of(t, stream):
    if stream is not None:
        return stream if isinstance(stream, int) else stream.cuda_stream
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def matrix(k: int, m: int) -> np.ndarray:
    """The (k+m) x k encoding matrix (host-side, rsg_matrix)."""
    out = np.zeros((k + m, k), dtype=np.uint8)
    check(_lib.load().rsg_matrix(k, m, out.ctypes.data), f"rsg_matrix({k},{m})")
    return out
