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
        got = open(os.path.join(dirs[i], "bucket/obj", "part.1"), "rb").read()
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
        p = os.path.join(dirs[i], "b/o", "part.1")
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
    before = {i: open(os.path.join(dirs[i], "b/o", "part.1"), "rb").read() for i in lost}
    for i in lost:
        shutil.rmtree(os.path.join(dirs[i], "b/o"))
    es.heal_object("b/o", list(lost))
    for i in lost:
        assert open(os.path.join(dirs[i], "b/o", "part.1"), "rb").read() == before[i], i
    assert es.verify_object("b/o") == [0, 0, 0, 0]
    assert es.get_object("b/o") == data


def test_verify_object_flags_bad_shard_files(gpu, tmp_path):
    from rustfs_amd import _lib
    from rustfs_amd.loopback import LocalErasureSet
    dirs = [str(tmp_path / f"disk{i}") for i in range(4)]
    es = LocalErasureSet(dirs, 2, 2)
    data = np.random.default_rng(1).integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
    es.put_object("b/o", data)
    p1 = os.path.join(dirs[1], "b/o", "part.1")
    raw = bytearray(open(p1, "rb").read())
    raw[2 * (32 + (1 << 19)) + 32 + 1000] ^= 0x20  # third record of shard 1
    open(p1, "wb").write(bytes(raw))
    p3 = os.path.join(dirs[3], "b/o", "part.1")
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
        raw = open(os.path.join(dirs[i], "o1", "part.1"), "rb").read()
        assert raw == _expected_shard_file(oracle, objs["o1"], 2, 2, 1 << 20, i), i
    for name in ("o5", "o0", "o3"):  # 4, 1, 2 blocks through the reused stages
        es.put_object(name + "b", objs[name])
        assert es.get_object(name + "b") == objs[name]
