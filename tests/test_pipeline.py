"""Streaming PUT (encode_batched, encode.rs:795-919) and range GET
(decode_inner, decode.rs:1702-1968) of the loopback erasure set.

The streamed PUT must write byte-for-byte the shard files the CPU oracle
predicts (the same files as put_object), whatever the batch size; the range
GET must return exactly data[offset:offset+length] for ranges that start and
end inside, on and across block boundaries and the short last block, with
lost drives and corrupted records."""
import io
import os

import numpy as np
import pytest

from rustfs_amd.pipeline import block_geometry

BS = 1 << 16  # small blocks so a few MiB spans many batches


def _ranges(size, bs):
    rng = np.random.default_rng(size)
    out = {(0, size), (0, 0), (size, 0), (0, 1), (size - 1, 1) if size else (0, 0)}
    for b in (bs - 1, bs, bs + 1, 2 * bs, 3 * bs - 5):
        if b <= size:
            out.add((0, b))
            out.add((b, size - b))
    for _ in range(12):
        o = int(rng.integers(0, size + 1))
        out.add((o, int(rng.integers(0, size - o + 1))))
    return sorted(out)


def test_block_geometry_matches_brute_force():
    """decode.rs:1767-1781: the per-block window of a range."""
    bs = 10
    for total in (1, 9, 10, 11, 35):
        for off in range(total):
            for ln in range(1, total - off + 1):
                want = {}
                for x in range(off, off + ln):
                    b = x // bs
                    o, n = want.get(b, (x % bs, 0))
                    want[b] = (o, n + 1)
                for b, (o, n) in want.items():
                    assert block_geometry(off, ln, bs, b) == (o, n), (total, off, ln, b)


def test_range_errors_before_any_io():
    from rustfs_amd.erasure import Erasure
    from rustfs_amd.pipeline import get_stream
    e = Erasure(2, 2, BS)
    with pytest.raises(ValueError, match="offset \\+ length exceeds total length"):
        list(get_stream(e, [None] * 4, 100, 90, 11))
    with pytest.raises(ValueError):
        list(get_stream(e, [None] * 4, 100, -1, 1))
    assert list(get_stream(e, [None] * 4, 100, 40, 0)) == []
    assert list(get_stream(e, [None] * 4, 0)) == []


def _set(tmp_path, k, m, bs=BS):
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(k + m)]
    return LocalErasureSet(dirs, k, m, block_size=bs), dirs


def _files(es, name):
    return [open(es.part_file(i, name), "rb").read() for i in range(len(es.dirs))]


def _reader(kind, data, tmp_path):
    """BytesIO (sequential readinto producer) or a regular file opened at an
    offset (parallel pread producer)."""
    if kind == "bytes":
        return io.BytesIO(data)
    p = tmp_path / "body"
    p.write_bytes(b"HEAD" + data + b"TRAILER")
    f = open(p, "rb")
    f.seek(4)
    return f


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bytes", "file"])
@pytest.mark.parametrize("k,m", [(2, 2), (8, 4), (5, 3)])
@pytest.mark.parametrize("nblk,tail", [(0, 0), (0, 777), (1, 0), (7, 0), (7, 12345), (9, 1)])
def test_put_stream_writes_put_object_files(gpu, oracle, tmp_path, kind, k, m, nblk, tail):
    size = nblk * BS + tail
    es, dirs = _set(tmp_path, k, m)
    data = np.random.default_rng(size + k).integers(0, 256, size, dtype=np.uint8).tobytes()
    r = _reader(kind, data, tmp_path)
    es.put_object_stream("b/s", r, size, batch_blocks=3, inflight_batches=1)
    if kind == "file":
        assert r.read() == b"TRAILER"  # left positioned after the body
    es.put_object("b/o", data)
    got, want = _files(es, "b/s"), _files(es, "b/o")
    assert got == want
    # oracle: block by block [HH256S][shard] records
    if size:
        b0 = (nblk - 1) * BS if nblk else 0
        blk = np.frombuffer(data[b0:b0 + BS], dtype=np.uint8)
        S = -(-blk.size // k)
        st = np.zeros((k + m, S), dtype=np.uint8)
        st.reshape(-1)[: blk.size] = blk
        oracle.encode(k, m, st)
        off = (nblk - 1) * (32 + -(-BS // k)) if nblk else 0
        for i in range(k + m):
            assert got[i][off: off + 32 + S] == oracle.hh256s(st[i]) + st[i].tobytes(), i
    assert es.get_object("b/s") == data


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["bytes", "file"])
def test_put_stream_short_body_raises(gpu, tmp_path, kind):
    es, _ = _set(tmp_path, 2, 2)
    with pytest.raises(EOFError):
        es.put_object_stream("b/s", _reader(kind, b"x" * (3 * BS), tmp_path), 5 * BS, batch_blocks=2)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,lost", [(2, 2, ()), (2, 2, (0,)), (2, 2, (0, 1)), (2, 2, (1, 3)),
                                      (6, 3, (0, 4)), (20, 4, (1, 19)), (20, 4, (0, 21))])
def test_range_get(gpu, tmp_path, k, m, lost):
    """(6,3) and (20,4): shard lengths that are not multiples of 16 (the byte
    tail and unaligned copy-through), k > 16 (chained launches, wide compare)."""
    size = 11 * BS + 4321
    es, dirs = _set(tmp_path, k, m)
    data = np.random.default_rng(5).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(data), size, batch_blocks=4)
    for i in lost:
        os.remove(es.part_file(i, "b/o"))
    for off, ln in _ranges(size, BS):
        got = b"".join(es.get_object_stream("b/o", off, ln, batch_blocks=3))
        assert got == data[off:off + ln], (off, ln)
    with pytest.raises(ValueError):
        es.get_object_range("b/o", size - 3, 4)


@pytest.mark.gpu
@pytest.mark.parametrize("lost", [(0, 3, 7), (0, 1, 2, 5, 9)])
def test_range_get_ec5_many_lost_one_pass(gpu, tmp_path, lost):
    """EC:5 (RS(5,5), 10 drives) with three and with five drives lost, read in
    batches of 1100 blocks (>= 1024: the one-pass table kernel, five rows a
    step with five lost) — the whole object and two ranges."""
    k, m, nblk = 5, 5, 1100
    size = nblk * BS + 999
    es, dirs = _set(tmp_path, k, m)
    data = np.random.default_rng(55).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(data), size, batch_blocks=256)
    for i in lost:
        os.remove(es.part_file(i, "b/o"))
    for off, ln in ((0, size), (3 * BS + 17, 1050 * BS), (size - BS - 5, BS + 5)):
        got = b"".join(es.get_object_stream("b/o", off, ln, batch_blocks=nblk))
        assert got == data[off:off + ln], (off, ln)


@pytest.mark.gpu
@pytest.mark.parametrize("lost", [(), (0, 3), (4,)])
def test_range_get_views(gpu, tmp_path, lost):
    """get_stream(views=True): each block's window as memoryviews of the
    record stage and the rebuilt slots (write_data_blocks' form), the same
    bytes as the joined form, over batches whose device sets alternate
    (records of batch j+1 copied while batch j is decoded)."""
    from rustfs_amd.pipeline import get_stream
    k, m = 4, 2
    size = 9 * BS + 777
    es, dirs = _set(tmp_path, k, m)
    data = np.random.default_rng(9).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(data), size, batch_blocks=4)
    fds = [None if i in lost else os.open(es.part_file(i, "b/o"), os.O_RDONLY) for i in range(k + m)]
    try:
        for off, ln in _ranges(size, BS):
            got = []
            for blk in get_stream(es.erasure, fds, size, off, ln, batch_blocks=2, views=True):
                assert all(isinstance(v, memoryview) for v in blk)
                got.append(b"".join(blk))  # valid until the next block is requested
            assert b"".join(got) == data[off:off + ln], (off, ln)
    finally:
        for fd in fds:
            if fd is not None:
                os.close(fd)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["healthy", "data_lost", "rotten_data", "rotten_and_lost", "truncated_data"])
def test_get_data_shards_only(gpu, tmp_path, case):
    """data_shards_only=True (the reference's RUSTFS_GET_LOCKSTEP_DATA_SHARDS_ONLY
    read, decode.rs:1031-1090): the data files alone while they serve, missing
    + 1 parity files engaged for lost data files, every parity file engaged
    (and the batch decoded again) once a record cannot be served — the same
    bytes as the default read in every case."""
    from rustfs_amd.pipeline import get_stream
    k, m = 4, 2
    size = 9 * BS + 555
    es, dirs = _set(tmp_path, k, m)
    data = np.random.default_rng(11).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(data), size, batch_blocks=4)
    rec = 32 + BS // k
    lost = (1,) if case in ("data_lost", "rotten_and_lost") else ()
    if case in ("rotten_data", "rotten_and_lost"):
        p = es.part_file(2, "b/o")
        raw = bytearray(open(p, "rb").read())
        raw[5 * rec + 32 + 99] ^= 0x10  # block 5, data shard 2's body: its digest no longer matches
        open(p, "wb").write(bytes(raw))
    for i in lost:
        os.remove(es.part_file(i, "b/o"))
    if case == "truncated_data":  # data file 3 ends after 4 records: its later reads fail mid-object
        os.truncate(es.part_file(3, "b/o"), 4 * rec)
    fds = [None if i in lost else os.open(es.part_file(i, "b/o"), os.O_RDONLY) for i in range(k + m)]
    try:
        for off, ln in [(0, size), (3 * BS + 7, 4 * BS), (size - 100, 100)]:
            got = b"".join(b"".join(v) for v in get_stream(es.erasure, fds, size, off, ln, batch_blocks=2, views=True,
                                                           data_shards_only=True))
            assert got == data[off:off + ln], (case, off, ln)
    finally:
        for fd in fds:
            if fd is not None:
                os.close(fd)


@pytest.mark.gpu
def test_range_get_drops_corrupted_records(gpu, tmp_path):
    from rustfs_amd import RsgError
    size = 6 * BS + 100
    es, dirs = _set(tmp_path, 4, 2)
    data = np.random.default_rng(6).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(data), size, batch_blocks=2)
    rec = 32 + BS // 4

    def flip(i, off):
        p = es.part_file(i, "b/o")
        raw = bytearray(open(p, "rb").read())
        raw[off] ^= 0x40
        open(p, "wb").write(bytes(raw))

    flip(0, 3 * rec + 32 + 7)   # block 3, data shard 0 body
    flip(5, 3 * rec + 1)        # block 3, parity shard 5 digest
    flip(1, 6 * rec + 32 + 10)  # tail block (25-byte shards), data shard 1
    assert es.get_object_range("b/o", 2 * BS + 10, 4 * BS) == data[2 * BS + 10: 6 * BS + 10]
    assert es.get_object("b/o") == data
    flip(2, 3 * rec + 40)       # a third bad record in block 3: below read quorum
    with pytest.raises(RsgError):
        es.get_object_range("b/o", 3 * BS, 10)
    assert es.get_object_range("b/o", 0, 3 * BS) == data[: 3 * BS]  # other blocks still read


@pytest.mark.gpu
def test_stream_close_early(gpu, tmp_path):
    size = 20 * BS
    es, _ = _set(tmp_path, 2, 2)
    data = np.random.default_rng(8).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(data), size)
    g = es.get_object_stream("b/o", BS // 2, batch_blocks=4)
    assert next(g) == data[BS // 2: BS]
    g.close()  # joins the read-ahead thread, closes the shard files
    assert es.get_object("b/o") == data


class _BreakWriters(io.BytesIO):
    """A body reader that, once `after` bytes have been read, breaks the
    shard writers in `targets`: their descriptors are replaced (dup2) by a
    read-only one, so every later write to them fails (EBADF) — a shard disk
    that goes away mid-stream."""

    def __init__(self, data, after, es, name, targets):
        super().__init__(data)
        self.after, self.es, self.name, self.targets, self.read_so_far = after, es, name, targets, 0
        self.ro = os.open(os.devnull, os.O_RDONLY)

    def readinto(self, b):
        n = super().readinto(b)
        self.read_so_far += n
        if self.read_so_far >= self.after and self.targets:
            for i in self.targets:
                fd = self._fd_of(i)
                if fd is not None:
                    os.dup2(self.ro, fd)
            self.targets = ()
        return n

    def _fd_of(self, i):
        base = os.path.realpath(os.path.join(self.es.dirs[i], self.name)) + os.sep
        for fd in os.listdir("/proc/self/fd"):
            try:  # the PUT writes <name>/<its version>/part.1 (nothing else is open there)
                p = os.path.realpath(f"/proc/self/fd/{fd}")
                if p.startswith(base) and p.endswith(os.sep + "part.1"):
                    return int(fd)
            except OSError:
                pass
        return None


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,broken,ok", [(4, 2, (1,), True), (4, 2, (0, 5), True), (4, 2, (0, 2, 5), False),
                                           (2, 2, (3,), True), (2, 2, (0, 3), False)])
def test_put_stream_write_quorum(gpu, tmp_path, k, m, broken, ok):
    """MultiWriter::write_shards (encode.rs:374-430): writers that fail
    mid-stream are dropped and the PUT completes while >= write quorum (k, or
    k+1 when k == m) remain; the dropped shards are not committed, GET reads
    the object back and heal rebuilds their files byte for byte.  Below
    quorum the PUT fails with "Failed to write data"."""
    from rustfs_amd.pipeline import WriteQuorumError
    size = 9 * BS + 777
    es, dirs = _set(tmp_path, k, m)
    data = np.random.default_rng(k * 10 + len(broken)).integers(0, 256, size, dtype=np.uint8).tobytes()
    r = _BreakWriters(data, 3 * BS, es, "b/o", broken)
    if not ok:
        with pytest.raises(WriteQuorumError, match="Failed to write data"):
            es.put_object_stream("b/o", r, size, batch_blocks=2, inflight_batches=1)
        return
    es.put_object_stream("b/o", r, size, batch_blocks=2, inflight_batches=1)
    assert es.last_put["failed_shards"] == sorted(broken)
    for i in broken:  # neither a meta.json nor any version's part
        assert es.part_file(i, "b/o") is None and os.listdir(os.path.join(dirs[i], "b/o")) == []
    assert es.get_object("b/o") == data
    es.put_object("b/ref", data)
    es.heal_object("b/o", list(broken))
    assert _files(es, "b/o") == _files(es, "b/ref")


@pytest.mark.gpu
def test_put_stream_disk_missing_from_start(gpu, tmp_path):
    """A disk with no writer at all (None: DiskNotFound) counts against the
    quorum from the first block."""
    from rustfs_amd.pipeline import WriteQuorumError, put_stream
    from rustfs_amd.erasure import Erasure
    k, m = 4, 2
    e = Erasure(k, m, BS)
    size = 5 * BS
    data = np.random.default_rng(1).integers(0, 256, size, dtype=np.uint8).tobytes()
    paths = [tmp_path / f"s{i}" for i in range(k + m)]
    fds = [os.open(p, os.O_WRONLY | os.O_CREAT) for p in paths]
    try:
        info = put_stream(e, io.BytesIO(data), size, [None if i == 4 else fd for i, fd in enumerate(fds)],
                          batch_blocks=2)
        assert info["failed_shards"] == [4] and info["write_quorum"] == 4
        assert os.path.getsize(paths[4]) == 0 and os.path.getsize(paths[0]) == 5 * (32 + BS // k)
        with pytest.raises(WriteQuorumError):
            put_stream(e, io.BytesIO(data), size, [None, None, None] + fds[3:], batch_blocks=2)
    finally:
        for fd in fds:
            os.close(fd)


@pytest.mark.gpu
@pytest.mark.parametrize("old_size,new_size", [(9 * BS + 777, 5 * BS + 3), (3 * BS + 997, 3 * BS + 1000)])
def test_overwrite_with_dropped_writer(gpu, tmp_path, old_size, new_size):
    """overwriting an object while shard 0's writer fails must not
    leave disk 0 with the old version's meta or part (GET would read the old
    size: a length mismatch fails every shard, an equal shard-file length
    returns the wrong byte count); and a PUT below write quorum must leave the
    old version readable.  (997 -> 1000 bytes of tail with k = 4: the same
    shard-file length.)"""
    from rustfs_amd.pipeline import WriteQuorumError
    k, m = 4, 2
    es, dirs = _set(tmp_path, k, m)
    old = np.random.default_rng(1).integers(0, 256, old_size, dtype=np.uint8).tobytes()
    new = np.random.default_rng(2).integers(0, 256, new_size, dtype=np.uint8).tobytes()
    es.put_object_stream("b/o", io.BytesIO(old), old_size, batch_blocks=2, inflight_batches=1)
    assert es.get_object("b/o") == old
    es.put_object_stream("b/o", _BreakWriters(new, BS, es, "b/o", (0,)), new_size, batch_blocks=2,
                         inflight_batches=1)
    assert es.last_put["failed_shards"] == [0]
    assert es.part_file(0, "b/o") is None and os.listdir(os.path.join(dirs[0], "b/o")) == []
    assert es.get_object("b/o") == new
    es.heal_object("b/o", [0])
    assert es.get_object("b/o") == new
    # below quorum: the PUT fails and the committed version stays readable
    with pytest.raises(WriteQuorumError):
        es.put_object_stream("b/o", _BreakWriters(old, BS, es, "b/o", (0, 1, 2)), old_size, batch_blocks=2,
                             inflight_batches=1)
    assert es.get_object("b/o") == new
    # every disk holds its meta.json and the committed version's directory, nothing else
    ver = es._meta("b/o")["version"]
    assert all(sorted(os.listdir(os.path.join(d, "b/o"))) == sorted(["meta.json", ver]) for d in dirs)


@pytest.mark.gpu
def test_meta_by_quorum(gpu, tmp_path):
    """A stale meta.json left on a minority of disks (a version those disks
    missed) is outvoted; their shard files are not read."""
    import json
    k, m = 2, 2
    es, dirs = _set(tmp_path, k, m)
    a = np.random.default_rng(3).integers(0, 256, 2 * BS + 5, dtype=np.uint8).tobytes()
    b = np.random.default_rng(4).integers(0, 256, 2 * BS + 9, dtype=np.uint8).tobytes()
    es.put_object("b/o", a)
    old_part = es.part_file(3, "b/o")
    stale = [open(p, "rb").read() for p in (os.path.join(dirs[3], "b/o", "meta.json"), old_part)]
    es.put_object("b/o", b)
    os.makedirs(os.path.dirname(old_part), exist_ok=True)  # disk 3 rolled back to the old version
    for p, raw in zip((os.path.join(dirs[3], "b/o", "meta.json"), old_part), stale):
        open(p, "wb").write(raw)
    assert json.load(open(os.path.join(dirs[3], "b/o", "meta.json")))["size"] == len(a)
    assert es.get_object("b/o") == b
