"""BASELINE config 1: single-node 4-drive loopback RS(2,2), PUT+GET 1 MiB
objects, through the GPU engine.  The on-disk shard files must be byte-for-byte
what the reference writes ([HH256S][block] records, bitrot.rs:464-510, with
RS(2,2) parity), checked against the CPU oracle; GET must survive 0/1/2 lost
drives and silently corrupted records (bitrot verify-before-use)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expected_shard_file(oracle, data: bytes, k: int, m: int, block: int, i: int) -> bytes:
    out = b""
    for b0 in range(0, len(data), block):
        blk = np.frombuffer(data[b0:b0 + block], dtype=np.uint8)
        S = -(-blk.size // k)
        st = np.zeros((k + m, S), dtype=np.uint8)
        st.reshape(-1)[: blk.size] = blk
        oracle.encode(k, m, st)
        out += oracle.hh256s(st[i]) + st[i].tobytes()
    return out


@pytest.mark.parametrize("size", [1 << 20, (5 << 20) // 2, 1000, 1])
def test_put_writes_reference_shard_files(gpu, oracle, tmp_path, size):
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object("bucket/obj", data)
    for i in range(4):
        got = open(es.part_file(i, "bucket/obj"), "rb").read()
        assert got == _expected_shard_file(oracle, data, 2, 2, 1 << 20, i), i
    assert es.get_object("bucket/obj") == data


@pytest.mark.parametrize("lost", [(), (0,), (3,), (0, 1), (1, 2), (2, 3)])
def test_get_survives_lost_drives(gpu, tmp_path, lost):
    import shutil
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(7).integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
    es.put_object("b/o", data)
    for i in lost:
        shutil.rmtree(os.path.join(dirs[i], "b/o"))
    assert es.get_object("b/o") == data


def test_get_drops_corrupted_records(gpu, tmp_path):
    from rustfs_amd import RsgError
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(9).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    es.put_object("b/o", data)

    def flip(i, off):
        p = es.part_file(i, "b/o")
        raw = bytearray(open(p, "rb").read())
        raw[off] ^= 0x01
        open(p, "wb").write(bytes(raw))

    flip(0, 32 + 12345)  # data byte of shard 0
    flip(2, 5)           # hash byte of shard 2
    assert es.get_object("b/o") == data
    flip(1, 100)         # a third bad shard: below read quorum
    with pytest.raises(RsgError):
        es.get_object("b/o")


@pytest.mark.parametrize("size,lost", [((5 << 20) // 2, (0, 3)), (1 << 20, (1,)), (1000, (2, 3)), (3 << 20, (0, 1))])
def test_heal_rewrites_identical_shard_files(gpu, tmp_path, size, lost):
    """Erasure::heal (heal.rs:112-206) through the GPU heal engine: the healed
    part files are byte-identical to what PUT wrote, and the deep scan passes."""
    import shutil
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    es.put_object("b/o", data)
    before = {i: open(es.part_file(i, "b/o"), "rb").read() for i in lost}
    for i in lost:
        shutil.rmtree(os.path.join(dirs[i], "b/o"))
    es.heal_object("b/o", list(lost))
    for i in lost:
        assert open(es.part_file(i, "b/o"), "rb").read() == before[i], i
    assert es.verify_object("b/o") == [0, 0, 0, 0]
    assert es.get_object("b/o") == data


def test_verify_object_flags_bad_shard_files(gpu, tmp_path):
    from rustfs_amd import _lib
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(1).integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
    es.put_object("b/o", data)
    p1 = es.part_file(1, "b/o")
    raw = bytearray(open(p1, "rb").read())
    raw[2 * (32 + (1 << 19)) + 32 + 1000] ^= 0x20  # third record of shard 1
    open(p1, "wb").write(bytes(raw))
    p3 = es.part_file(3, "b/o")
    open(p3, "ab").write(b"x")  # trailing byte on shard 3
    assert es.verify_object("b/o") == [0, _lib.RSG_ERR_BITROT_MISMATCH, 0, _lib.RSG_ERR_TRAILING_DATA]
    # heal the damaged shards from the healthy ones, then everything verifies
    es.heal_object("b/o", [1, 3])
    assert es.verify_object("b/o") == [0, 0, 0, 0]
    assert es.get_object("b/o") == data


def test_concurrent_put_get_share_stages(gpu, oracle, tmp_path):
    """The set's reusable page-locked PUT/GET stages under concurrent callers:
    the caller that finds a stage busy allocates its own, so objects of
    different sizes PUT and GET from 4 threads at once stay byte-exact (and
    the shard files equal the reference's); a later single-threaded pass
    reuses the stages for sizes that need fewer or more blocks."""
    from concurrent.futures import ThreadPoolExecutor
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    sizes = [1 << 20, 3 << 20, (1 << 20) + 7, 2 << 20, 5000, 4 << 20, 1 << 20, (3 << 20) - 1]
    objs = {f"o{j}": np.random.default_rng(j + 100).integers(0, 256, sz, dtype=np.uint8).tobytes()
            for j, sz in enumerate(sizes)}
    with ThreadPoolExecutor(4) as ex:
        list(ex.map(lambda kv: es.put_object(kv[0], kv[1]), objs.items()))
        got = dict(zip(objs, ex.map(es.get_object, objs)))
    for name, data in objs.items():
        assert got[name] == data, name
    for i in range(4):
        raw = open(es.part_file(i, "o1"), "rb").read()
        assert raw == _expected_shard_file(oracle, objs["o1"], 2, 2, 1 << 20, i), i
    for name in ("o5", "o0", "o3"):  # 4, 1, 2 blocks through the reused stages
        es.put_object(name + "b", objs[name])
        assert es.get_object(name + "b") == objs[name]


@pytest.mark.parametrize("committed", [1, 3])
def test_crash_between_part_and_meta_never_mixes_versions(gpu, tmp_path, monkeypatch, committed):
    """a PUT that dies after writing every disk's part but before
    switching every disk's meta.json leaves some disks on the new version and
    the rest on the old one.  Each disk's part lives in its version's own
    directory, so a disk still naming the old version reads the old part: GET
    returns one version whole (the one on more disks), never a mix — even with
    every data disk present, when parity is never read."""
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    old = np.random.default_rng(21).integers(0, 256, (3 << 20) + 5, dtype=np.uint8).tobytes()
    new = np.random.default_rng(22).integers(0, 256, (3 << 20) + 5, dtype=np.uint8).tobytes()
    es.put_object("b/o", old)
    real = es._write_meta_file
    calls = []

    def crashing(i, name, meta):
        if len(calls) == committed:
            raise OSError("crash")
        calls.append(i)
        real(i, name, meta)

    monkeypatch.setattr(es, "_write_meta_file", crashing)
    with pytest.raises(OSError):
        es.put_object("b/o", new)
    monkeypatch.setattr(es, "_write_meta_file", real)
    assert es.get_object("b/o") == (new if committed > 2 else old)
    # heal brings the disks behind onto the served version
    lag = [i for i in range(4) if (i in calls) != (committed > 2)]
    es.heal_object("b/o", lag)
    assert es.get_object("b/o") == (new if committed > 2 else old)
    assert es.verify_object("b/o") == [0, 0, 0, 0]


def test_read_quorum_required(gpu, tmp_path):
    """a metadata version held by fewer than k disks is never
    served: with the disks split 1 / 1 / 2 dropped (k = 2 of RS(2,2)) no
    version reaches read quorum and GET is a read-quorum error, whatever the
    disk order."""
    import shutil
    from rustfs_amd import RsgError
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(5).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    es.put_object("b/o", data)
    for i in (2, 3):
        shutil.rmtree(os.path.join(dirs[i], "b/o"))
    assert es.get_object("b/o") == data  # two disks: read quorum
    shutil.rmtree(os.path.join(dirs[1], "b/o"))
    with pytest.raises(RsgError, match="read quorum"):
        es.get_object("b/o")
