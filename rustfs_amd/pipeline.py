"""Batched, pipelined stripe I/O for the loopback erasure set: the GPU arm of
the reference's stripe write/read pipelines.

PUT — ``put_stream`` mirrors ``Erasure::encode_batched``
(crates/ecstore/src/erasure/coding/encode.rs:795-919): a producer reads the
object body block by block into batches of B blocks
(``RUSTFS_ERASURE_ENCODE_BATCH_BLOCKS``, encode.rs:39-43), each batch goes to
the GPU as one asynchronous host-batch job (``rsg_encode_batch_host_submit``:
H2D -> encode + fused HighwayHash256S -> D2H), and a consumer writes the
finished batches' ``[HH256S][shard]`` records to the shard files
(``BitrotWriter::write``, bitrot.rs:464-510), one vectored write per shard
file per batch, the k+m files in parallel (``MultiWriter``, encode.rs:200-330).
The number of batches between producer and consumer is bounded (the
reference bounds its channel by ``RUSTFS_ERASURE_ENCODE_MAX_INFLIGHT_BYTES``,
encode.rs:64-72), so reading batch i+1, encoding batch i and writing batch
i-1 overlap.  The staging buffers are page-locked and reused, so the copies
run at full PCIe rate.

GET — ``get_stream`` mirrors ``Erasure::decode_inner``
(crates/ecstore/src/erasure/coding/decode.rs:1702-1968) for a byte range:
the blocks covering [offset, offset + length) are read from the shard files B
blocks at a time (a read-ahead thread fetches batch i+1 while batch i is
verified and decoded on the GPU by ``rsg_decode_records_into_dev``), and the
requested bytes of each block are yielded in order (the block geometry of
decode.rs:1767-1781).  A short last block goes through the host codec path.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Iterator, List, Optional

import numpy as np

from . import _lib
from .bitrot import HashAlgorithm
from .erasure import Erasure, calc_shard_size

DEFAULT_BATCH_BLOCKS = 64      # blocks per GPU job (the reference batches 4 on the CPU)
DEFAULT_INFLIGHT_BATCHES = 2   # encoded batches queued for the writers
IO_THREADS = 16                # shard-file readers (GET) / writers (PUT), capped at one per shard file


def _pinned(shape) -> np.ndarray:
    import torch
    return torch.zeros(shape, dtype=torch.uint8).pin_memory().numpy()


def _read_into(reader, view: memoryview) -> int:
    got = 0
    while got < len(view):
        n = reader.readinto(view[got:])
        if not n:
            break
        got += n
    return got


def _file_source(reader):
    """(fd, position) when `reader` is a regular file positioned by tell():
    the producer then reads a batch's blocks in parallel with pread."""
    try:
        fd = reader.fileno()
        pos = reader.tell()
        import stat
        if stat.S_ISREG(os.fstat(fd).st_mode):
            return fd, pos
    except (AttributeError, OSError, ValueError):
        pass
    return None


def default_write_quorum(k: int, m: int) -> int:
    """The erasure set's write quorum: the data drive count, plus one when
    data == parity (set_disk/mod.rs:2792-2795, set_disk/metadata.rs:336-340)."""
    return k + (1 if k == m else 0)


class WriteQuorumError(IOError):
    """MultiWriter::write_shards' "Failed to write data: ..." once fewer
    shard writers than the write quorum are still alive (encode.rs:408-429)."""


def _write_all(fd: int, iov: List[memoryview]) -> None:
    want = sum(len(v) for v in iov)
    done = os.writev(fd, iov)
    while done < want:  # short write: finish the rest the plain way
        flat = b"".join(bytes(v) for v in iov)[done:]
        done += os.write(fd, flat)


class PutStage:
    """Reusable page-locked (B, k+m, S) stripe buffers + (B, k+m, 32) digest
    arrays for put_stream.  The bytes between a block's end and k*S are never
    written, so the zero padding of erasure.rs:858-866 holds on reuse."""

    def __init__(self, count: int, blocks: int, t: int, S: int):
        self.shape = (count, blocks, t, S)
        self.stripes = [_pinned((blocks, t, S)) for _ in range(count)]
        self.digests = [_pinned((blocks, t, 32)) for _ in range(count)]  # D2H into pageable memory would block the submit

    def fits(self, count: int, blocks: int, t: int, S: int) -> bool:
        c, b, tt, s = self.shape
        return c >= count and b >= blocks and tt == t and s == S


def put_stream(erasure: Erasure, reader, size: int, fds: List[Optional[int]],
               algo: HashAlgorithm = HashAlgorithm.HighwayHash256S,
               batch_blocks: int = DEFAULT_BATCH_BLOCKS,
               inflight_batches: int = DEFAULT_INFLIGHT_BATCHES,
               stage: Optional[PutStage] = None, read_threads: int = 8,
               write_quorum: Optional[int] = None) -> dict:
    """Encode `size` bytes read from `reader` (``readinto``) and append one
    BitrotWriter record per block to each shard file descriptor in `fds`
    (k data then m parity; None: that disk has no writer).  Returns the
    block/batch counts, the shards whose writers failed and the stage used
    (pass it back in to reuse its page-locked buffers).  A regular-file
    `reader` is read `read_threads` blocks at a time with pread (and left
    positioned after the body, like a sequential read).

    Write quorum (MultiWriter::write_shards, encode.rs:374-430): a shard
    file whose write fails (or short-writes) is dropped — nothing more is
    written to it — and the PUT goes on while at least `write_quorum`
    writers (default: default_write_quorum) are alive; below that it raises
    WriteQuorumError.  The caller must not commit the dropped shards."""
    k, m = erasure.data_shards, erasure.parity_shards
    t = k + m
    if len(fds) != t:
        raise ValueError("one file descriptor per shard")
    wq = default_write_quorum(k, m) if write_quorum is None else write_quorum
    # per-writer error: None = alive (the reference's errs[i] with writer Some)
    werr: List[Optional[BaseException]] = [None if fd is not None else FileNotFoundError("disk not found")
                                           for fd in fds]

    def check_quorum() -> None:
        alive = sum(e is None for e in werr)
        if alive < wq:
            failed = {i: repr(e) for i, e in enumerate(werr) if e is not None}
            raise WriteQuorumError(f"Failed to write data: write quorum {wq} not met: {alive} of {t} shard "
                                   f"writers alive, failed {failed}")

    check_quorum()
    bs = erasure.block_size
    S = erasure.shard_size()
    nfull, tail = divmod(size, bs)
    blocks = max(1, min(batch_blocks, nfull))
    nslots = inflight_batches + 2  # queued + being written + being filled
    if nfull and (stage is None or not stage.fits(nslots, blocks, t, S)):
        stage = PutStage(nslots, blocks, t, S)
    free: "queue.Queue[int]" = queue.Queue()
    for i in range(nslots if nfull else 0):
        free.put(i)
    done: "queue.Queue" = queue.Queue(maxsize=inflight_batches)
    errors: List[BaseException] = []
    pool = ThreadPoolExecutor(max_workers=min(t, IO_THREADS))
    src = _file_source(reader) if read_threads > 1 else None
    rpool = ThreadPoolExecutor(max_workers=read_threads) if src else None
    clock = {"read_s": 0.0, "submit_s": 0.0, "wait_s": 0.0, "write_s": 0.0}

    def write_batch(slot: int, cnt: int) -> None:
        st, dg = stage.stripes[slot], stage.digests[slot]

        def one(i):
            iov = []
            for b in range(cnt):
                iov.append(memoryview(dg[b, i]))
                iov.append(memoryview(st[b, i]))
            try:
                _write_all(fds[i], iov)
            except OSError as exc:  # drop this writer (write_shard, encode.rs:342-362)
                werr[i] = exc

        for f in [pool.submit(one, i) for i in range(t) if werr[i] is None]:
            f.result()
        check_quorum()

    def consumer():
        while True:
            item = done.get()
            if item is None:
                return
            ticket, slot, cnt = item
            try:
                t0 = time.perf_counter()
                ticket.wait()
                t1 = time.perf_counter()
                if not errors:
                    write_batch(slot, cnt)
                clock["wait_s"] += t1 - t0
                clock["write_s"] += time.perf_counter() - t1
            except BaseException as exc:  # surfaced by the producer
                errors.append(exc)
            free.put(slot)

    writer = threading.Thread(target=consumer, daemon=True)
    writer.start()
    batches = 0
    try:
        left = nfull
        while left and not errors:
            slot = free.get()
            st, dg = stage.stripes[slot], stage.digests[slot]
            cnt = min(blocks, left)
            t0 = time.perf_counter()
            if src:  # block b's data at src offset; padding to k*S stays zero
                base = src[1] + (nfull - left) * bs
                got = rpool.map(lambda b: os.preadv(src[0], [memoryview(st[b]).cast("B")[:bs]], base + b * bs),
                                range(cnt))
                if any(n != bs for n in got):
                    raise EOFError("object body shorter than its declared size")
            else:
                for b in range(cnt):
                    if _read_into(reader, memoryview(st[b]).cast("B")[:bs]) != bs:
                        raise EOFError("object body shorter than its declared size")
            t1 = time.perf_counter()
            ticket = erasure.encode_batch_host_submit(st[:cnt], dg[:cnt], algo=algo.value)
            clock["read_s"] += t1 - t0
            clock["submit_s"] += time.perf_counter() - t1
            done.put((ticket, slot, cnt))
            batches += 1
            left -= cnt
    finally:
        done.put(None)
        writer.join()
        pool.shutdown()
        if rpool:
            rpool.shutdown()
    if errors:
        raise errors[0]
    if src:
        reader.seek(src[1] + nfull * bs)
    if tail:  # the short last block: host codec path (encode_data)
        buf = bytearray(tail)
        if _read_into(reader, memoryview(buf)) != tail:
            raise EOFError("object body shorter than its declared size")
        shards = erasure.encode_data(buf)
        for i in range(t):
            if werr[i] is not None:
                continue
            try:
                _write_all(fds[i], [memoryview(algo.hash_encode(shards[i]) + shards[i])])
            except OSError as exc:
                werr[i] = exc
        check_quorum()
    return {"size": size, "full_blocks": nfull, "tail": tail, "batches": batches, "batch_blocks": blocks,
            "failed_shards": [i for i in range(t) if werr[i] is not None], "write_quorum": wq,
            "stage": stage, **clock}


def block_geometry(offset: int, length: int, block_size: int, block: int):
    """(offset in block, bytes) of `block` for the range [offset, offset +
    length): decode_inner's per-block window, decode.rs:1767-1781."""
    start, end = offset // block_size, (offset + length - 1) // block_size
    if start == end:
        return offset % block_size, length
    if block == start:
        return offset % block_size, block_size - offset % block_size
    if block == end:
        r = (offset + length) % block_size
        return 0, r if r else block_size
    return 0, block_size


def get_stream(erasure: Erasure, fds: List[Optional[int]], total_length: int, offset: int = 0,
               length: Optional[int] = None, algo: HashAlgorithm = HashAlgorithm.HighwayHash256S,
               batch_blocks: int = DEFAULT_BATCH_BLOCKS, stage: Optional[GetStage] = None,
               views: bool = False, data_shards_only: bool = False) -> Iterator:
    """Yield bytes [offset, offset + length) of an object whose shard files
    are open at `fds` (None: disk unavailable), verifying every record
    before use and rebuilding missing data on the GPU.  Range errors follow
    decode_inner (decode.rs:1716-1742).  `stage`: reusable buffers
    (GetStage), else allocated for this call.

    views=True: each block's window as a list of memoryviews of the shard
    buffers it lies in (the verified record bodies in the page-locked read
    stage, the rebuilt shards in their page-locked slots), in order, without
    joining them — write_data_blocks' form, which writes straight from the
    per-shard buffers (decode.rs:1390); a writev-ready iovec.  The views stay
    valid until the next block is requested (the stages are reused).

    data_shards_only=True: the reference's optional data-shards-only read
    (RUSTFS_GET_LOCKSTEP_DATA_SHARDS_ONLY_ENABLE, decode.rs:125-143,
    1031-1090; off by default there and here): while every data file is
    readable only the k data files are read; with data files missing, that
    many parity files plus one more (so the surplus check stays on) are
    engaged from the start; a batch whose verify finds a record it cannot
    serve engages every remaining parity file for the rest of the object and
    is read and decoded again with them."""
    if length is None:
        length = total_length - offset
    if offset < 0 or length < 0 or offset + length > total_length:
        raise ValueError("offset + length exceeds total length")
    if length == 0:
        return
    k, m = erasure.data_shards, erasure.parity_shards
    t = k + m
    if len(fds) != t:
        raise ValueError("one file descriptor (or None) per shard")
    bs = erasure.block_size
    S = erasure.shard_size()
    rec = 32 + S
    nfull = total_length // bs
    start, end = offset // bs, (offset + length - 1) // bs
    full_end = min(end, nfull - 1)  # last full block in the range
    if start <= full_end:
        yield from _get_full(erasure, fds, start, full_end, offset, length, algo, batch_blocks, stage, views,
                             data_shards_only)
    if end >= nfull:  # the short last block: host path, verify-before-use
        tl = total_length - nfull * bs
        s_blk = calc_shard_size(tl, k)
        shards: List[Optional[bytes]] = [None] * t
        for i, fd in enumerate(fds):
            if fd is None:
                continue
            r = os.pread(fd, 32 + s_blk, nfull * rec)
            if len(r) == 32 + s_blk and algo.hash_encode(r[32:]) == r[:32]:
                shards[i] = r[32:]
        if sum(x is not None for x in shards) < k:
            raise _lib.RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, "read quorum lost")
        erasure.decode_data_with_reconstruction_verification(shards)
        blk = b"".join(bytes(shards[i]) for i in range(k))[:tl]
        o, n = block_geometry(offset, length, bs, nfull)
        yield [memoryview(blk)[o:o + n]] if views else blk[o:o + n]


class GetStage:
    """Reusable buffers of the GET pipeline: two page-locked record stages
    per shard file, the device record files, the in-place decode's k device
    slots and their page-locked mirrors, and the read pool.  Page-locking
    megabytes costs more than a whole 1 MiB-object GET (the loopback set's
    per-object calls), so a LocalErasureSet keeps one; a call that finds it
    busy (another thread's GET) allocates its own."""

    def __init__(self):
        self.lock = threading.Lock()
        self.key = None
        self.cnt = 0
        self.pool = None

    def ensure(self, t: int, k: int, S: int, bs: int, cnt_max: int, dev) -> None:
        import torch
        rec = 32 + S
        key = (t, k, S, bs, str(dev))
        if self.key != key or self.cnt < cnt_max:
            self.stage = [[_pinned(cnt_max * rec) for _ in range(t)] for _ in range(2)]
            # two sets: batch j+1's records go up while batch j is decoded
            self.files_dev = [[torch.empty(cnt_max * rec, dtype=torch.uint8, device=dev) for _ in range(t)]
                              for _ in range(2)]
            self.copy_stream = torch.cuda.Stream(dev)
            self.landed = [torch.cuda.Event(), torch.cuda.Event()]
            self.slots = [torch.empty(cnt_max * S, dtype=torch.uint8, device=dev) for _ in range(k)]
            self.host_slots = [_pinned(cnt_max * S) for _ in range(k)]
            self.key, self.cnt = key, cnt_max
        if self.pool is None:
            self.pool = ThreadPoolExecutor(max_workers=min(t, IO_THREADS))

    def close(self) -> None:
        if self.pool is not None:
            self.pool.shutdown()
            self.pool = None


def _get_full(erasure, fds, start, full_end, offset, length, algo, batch_blocks, reuse=None, views=False,
              data_only=False):
    """Full blocks start..full_end: B-block batches, read-ahead of batch i+1
    into the other page-locked stage while batch i is decoded on the GPU."""
    import torch
    k, t = erasure.data_shards, erasure.total_shard_count()
    bs, S = erasure.block_size, erasure.shard_size()
    rec = 32 + S
    dev = torch.device("cuda", erasure._device or 0)
    cnt_max = max(1, min(batch_blocks, full_end - start + 1))
    own = reuse is None or not reuse.lock.acquire(blocking=False)
    gs = GetStage() if own else reuse
    if own:
        gs.lock.acquire()
    try:
        gs.ensure(t, k, S, bs, cnt_max, dev)
        yield from _get_batches(erasure, fds, start, full_end, offset, length, algo, cnt_max, gs, views, data_only)
    finally:
        gs.lock.release()
        if own:
            gs.close()


def _get_batches(erasure, fds, start, full_end, offset, length, algo, cnt_max, gs, views=False, data_only=False):
    """The in-place GET (reconstruct_into's contract, bridge.rs:274-307; the
    blocks written straight from the per-shard buffers, decode.rs:1390): the
    records are verified on the device, only the shards no verified record
    serves are rebuilt and copied back, and every other byte of the range is
    served from the page-locked record stage it was read into — so the link
    carries the records in and the rebuilt shards out, nothing else."""
    import torch
    k, t = erasure.data_shards, erasure.total_shard_count()
    bs, S = erasure.block_size, erasure.shard_size()
    rec = 32 + S
    dev = torch.device("cuda", erasure._device or 0)
    stage, files_dev, slots, host_slots, pool = gs.stage, gs.files_dev, gs.slots, gs.host_slots, gs.pool
    batches = [(b0, min(cnt_max, full_end + 1 - b0)) for b0 in range(start, full_end + 1, cnt_max)]
    got: dict = {}
    # the files read (data_only: the data files, plus parity engaged as
    # decode.rs:1069-1090 does; else every available file)
    engaged = [fds[i] is not None and (not data_only or i < k) for i in range(t)]

    def engage_parity(want):
        have = sum(engaged[k:])
        for i in range(k, t):
            if have >= want:
                break
            if fds[i] is not None and not engaged[i]:
                engaged[i] = True
                have += 1

    if data_only:
        missing = sum(fds[i] is None for i in range(k))
        if missing:
            engage_parity(missing + 1)

    def read_one(j, i):
        b0, cnt = batches[j]
        if fds[i] is None:
            return False
        try:
            return os.preadv(fds[i], [memoryview(stage[j & 1][i][: cnt * rec])], b0 * rec) == cnt * rec
        except OSError:
            return False

    def fetch(j):
        """Batch j: one pread per shard file, files in parallel (a failed read
        = shard missing), then its records' H2D on the stage's copy stream
        into device set j & 1 (event landed[j & 1]) — so the copy of batch
        j+1 overlaps the decode of batch j."""
        b0, cnt = batches[j]
        want = list(engaged)
        ok = list(pool.map(lambda i: want[i] and read_one(j, i), range(t)))
        with torch.cuda.stream(gs.copy_stream):
            for i in range(t):
                if ok[i]:
                    files_dev[j & 1][i][: cnt * rec].copy_(torch.from_numpy(stage[j & 1][i][: cnt * rec]),
                                                           non_blocking=True)
            gs.landed[j & 1].record(gs.copy_stream)
        got[j] = ok

    th = threading.Thread(target=fetch, args=(0,))
    th.start()
    try:
        s = torch.cuda.current_stream(dev)
        def read_parity_now(j, ok):
            """data_only: every available parity file not read for batch j,
            read and copied up now (on the compute stream, before its decode)."""
            engage_parity(t)
            cnt = batches[j][1]
            more = [i for i in range(k, t) if fds[i] is not None and not ok[i]]
            for i, r in zip(more, pool.map(lambda i: read_one(j, i), more)):
                ok[i] = r
                if r:
                    files_dev[j & 1][i][: cnt * rec].copy_(torch.from_numpy(stage[j & 1][i][: cnt * rec]),
                                                           non_blocking=True)
            return bool(more)

        for j, (b0, cnt) in enumerate(batches):
            th.join()
            ok = got.pop(j)
            s.wait_event(gs.landed[j & 1])
            if data_only and not all(ok[i] for i in range(k) if fds[i] is not None):
                read_parity_now(j, ok)  # a data file failed to read: its reader is replaced by parity
            if sum(ok) < k:
                raise _lib.RsgError(_lib.RSG_ERR_TOO_FEW_SHARDS, "read quorum lost")
            # batch j+1 goes into the other stage and device set, free since
            # batch j-1 was decoded and its blocks yielded
            if j + 1 < len(batches):
                th = threading.Thread(target=fetch, args=(j + 1,))
                th.start()
            _, src, status = erasure.decode_records_into_batch(
                [files_dev[j & 1][i][: cnt * rec] if ok[i] else None for i in range(t)], S, cnt, targets=slots,
                target_stride=S, algo=algo.value, stream=s)
            bad = [x for x in status if x != _lib.RSG_OK]
            # a record it could not serve: engage every parity file, decode again
            if bad and data_only and read_parity_now(j, ok):
                _, src, status = erasure.decode_records_into_batch(
                    [files_dev[j & 1][i][: cnt * rec] if ok[i] else None for i in range(t)], S, cnt,
                    targets=slots, target_stride=S, algo=algo.value, stream=s)
                bad = [x for x in status if x != _lib.RSG_OK]
            if bad:
                _lib.check(bad[0], "erasure decode")
            for i in range(k):  # only the rebuilt shards cross the link back
                if not src[i].all():
                    torch.from_numpy(host_slots[i][: cnt * S]).copy_(slots[i][: cnt * S], non_blocking=True)
            s.synchronize()
            recs = [stage[j & 1][i][: cnt * rec].reshape(cnt, rec) for i in range(k)]
            for b in range(cnt):
                o, n = block_geometry(offset, length, bs, b0 + b)
                parts, pos, end = [], o, o + n
                while pos < end:  # the window's bytes shard by shard
                    i, off = divmod(pos, S)
                    take = min(S - off, end - pos)
                    if src[i, b]:
                        parts.append(recs[i][b, 32 + off: 32 + off + take])
                    else:
                        parts.append(host_slots[i][b * S + off: b * S + off + take])
                    pos += take
                yield [memoryview(x) for x in parts] if views else b"".join(parts)
    finally:
        th.join()
