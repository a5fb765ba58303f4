"""Heal (rsg_heal_records_dev; Erasure::heal, heal.rs:112-206) and whole-file
bitrot verification (rsg_bitrot_verify_dev; bitrot_verify, bitrot.rs:616-655)
on the GPU, checked against the CPU oracle and the reference's semantics."""
import io

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("engine_path")]


@pytest.fixture(params=["one_pass", "two_pass"], autouse=False)
def engine_path(request, gpu):
    """Every test runs through both lost-disk engines: the one-pass kernel
    (forced at any batch size where the geometry has one) and the two-pass
    path, selected on the device-0 context with rsg_set_record_engine (by
    default the one-pass kernel takes >= 1024 stripes)."""
    from rustfs_amd import _lib
    L = _lib.load()
    want = _lib.RSG_RECORD_ENGINE_ONE_PASS if request.param == "one_pass" else _lib.RSG_RECORD_ENGINE_TWO_PASS
    _lib.check(L.rsg_set_record_engine(gpu.handle, want))
    yield request.param
    _lib.check(L.rsg_set_record_engine(gpu.handle, _lib.RSG_RECORD_ENGINE_AUTO))


def _records(torch, oracle, k, m, S, n, seed):
    """n stripes of random data, parity from the oracle, BitrotWriter records
    ([HH256S][shard]) per shard file, built entirely on the host (oracle)."""
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    shards = np.zeros((n, k + m, S), dtype=np.uint8)
    recs = np.zeros((k + m, n, 32 + S), dtype=np.uint8)
    for s in range(n):
        shards[s, :k] = data[s]
        oracle.encode(k, m, shards[s])
        for i in range(k + m):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    files = [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(k + m)]
    return shards, recs, files


@pytest.mark.parametrize("k,m,S,n", [(8, 4, 4096, 7), (4, 2, 3001, 5), (12, 4, 1040, 3), (2, 2, 65536, 2)])
def test_heal_rebuilds_target_records(gpu, oracle, k, m, S, n):
    import torch
    from rustfs_amd import Erasure
    shards, recs, files = _records(torch, oracle, k, m, S, n, seed=k * 100 + S)
    e = Erasure(k, m, k * S)
    rec = 32 + S
    lost = [1, k] if m >= 2 else [1]  # one data and one parity disk replaced
    src = [None if i in lost else files[i] for i in range(k + m)]
    tgt = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(k + m)]
    status = e.heal_records_batch(src, tgt, S, n)
    assert status == [0] * n
    for i in lost:
        got = tgt[i].cpu().numpy().reshape(n, rec)
        assert np.array_equal(got, recs[i]), f"shard {i}"
    # heal a readable shard too: targets are written from the rebuilt set
    tgt2 = [None] * (k + m)
    tgt2[0] = torch.zeros(n * rec, dtype=torch.uint8, device="cuda")
    tgt2[k + m - 1] = torch.zeros(n * rec, dtype=torch.uint8, device="cuda")
    assert e.heal_records_batch(files, tgt2, S, n) == [0] * n
    assert np.array_equal(tgt2[0].cpu().numpy().reshape(n, rec), recs[0])
    assert np.array_equal(tgt2[k + m - 1].cpu().numpy().reshape(n, rec), recs[k + m - 1])


def test_heal_bitrot_and_quorum(gpu, oracle):
    import torch
    from rustfs_amd import Erasure, _lib
    k, m, S, n = 8, 4, 4096, 6
    shards, recs, files = _records(torch, oracle, k, m, S, n, seed=11)
    e = Erasure(k, m, k * S)
    rec = 32 + S
    f = [x.clone() for x in files]
    f[2][3 * rec + 32 + 5] ^= 0x10           # bitrot in stripe 3, shard 2: not a usable source
    for i in range(m + 1):                   # stripe 5 loses more than m shards: read quorum
        f[k - 1 - i][5 * rec + 40] ^= 0x01
    tgt = [None] * (k + m)
    tgt[2] = torch.zeros(n * rec, dtype=torch.uint8, device="cuda")
    status = e.heal_records_batch(f, tgt, S, n)
    assert status[:5] == [0] * 5 and status[5] == _lib.RSG_ERR_TOO_FEW_SHARDS
    got = tgt[2].cpu().numpy().reshape(n, rec)
    assert np.array_equal(got[:5], recs[2][:5])  # including the stripe whose shard-2 record rotted


def test_heal_detects_inconsistent_parity_with_all_data_present(gpu, oracle):
    """heal.rs:180-196 compares every source parity with the re-encoded parity,
    even when no data shard is missing (decode only does so when rebuilding)."""
    import torch
    from rustfs_amd import Erasure, _lib
    k, m, S, n = 4, 2, 2048, 4
    shards, recs, files = _records(torch, oracle, k, m, S, n, seed=3)
    e = Erasure(k, m, k * S)
    rec = 32 + S
    bad = recs[k + 1].copy()
    bad[2, 32 + 77] ^= 0xFF
    bad[2, :32] = np.frombuffer(oracle.hh256s(bad[2, 32:].tobytes()), dtype=np.uint8)  # digest matches the rot
    f = list(files)
    f[k + 1] = torch.from_numpy(bad.reshape(-1).copy()).cuda()
    tgt = [None] * (k + m)
    tgt[k] = torch.zeros(n * rec, dtype=torch.uint8, device="cuda")
    status = e.heal_records_batch(f, tgt, S, n)
    assert status == [0, 0, _lib.RSG_ERR_INCONSISTENT_SOURCES, 0]
    got = tgt[k].cpu().numpy().reshape(n, rec)
    for s in (0, 1, 3):
        assert np.array_equal(got[s], recs[k][s])


def _shard_file(oracle, part: bytes, S: int, legacy=False) -> bytes:
    out = bytearray()
    for o in range(0, len(part), S):
        blk = part[o:o + S]
        out += (oracle.hh256s_legacy(blk) if legacy else oracle.hh256s(blk)) + blk
    return bytes(out)


# S = 4096: records at 0 mod 16 (the quad hash kernel); 4102 and 4099: at 6
# mod 16 and odd pitches (HH256S: the LDS-DMA ring verify, rs_verify.hip)
@pytest.mark.parametrize("legacy,S", [(False, 4096), (True, 4096), (False, 4102), (False, 4099)])
def test_bitrot_verify_batch(gpu, oracle, legacy, S):
    import torch
    from rustfs_amd import _lib
    from rustfs_amd.bitrot import HashAlgorithm, bitrot_shard_file_size, bitrot_verify, bitrot_verify_batch
    algo = HashAlgorithm.HighwayHash256SLegacy if legacy else HashAlgorithm.HighwayHash256S
    rng = np.random.default_rng(7)
    part = rng.integers(0, 256, 3 * S + 100, dtype=np.uint8).tobytes()
    good = _shard_file(oracle, part, S, legacy)
    want = bitrot_shard_file_size(len(part), S, algo)
    assert len(good) == want
    rot = bytearray(good)
    rot[(32 + S) + 32 + 9] ^= 0x04           # record 1 body
    tail_rot = bytearray(good)
    tail_rot[-3] ^= 0x80                     # short last record
    cases = {
        "ok": (good, _lib.RSG_OK),
        "rot": (bytes(rot), _lib.RSG_ERR_BITROT_MISMATCH),
        "tail_rot": (bytes(tail_rot), _lib.RSG_ERR_BITROT_MISMATCH),
        "short": (good[:-50], _lib.RSG_ERR_UNEXPECTED_EOF),
        "short_in_header": (good[:3 * (32 + S) + 10], _lib.RSG_ERR_UNEXPECTED_EOF),
        "rot_then_short": (bytes(rot)[:-50], _lib.RSG_ERR_BITROT_MISMATCH),
        "trailing": (good + b"\x00", _lib.RSG_ERR_TRAILING_DATA),
        "empty": (b"", _lib.RSG_ERR_UNEXPECTED_EOF),
    }
    files = [torch.tensor(list(v[0]), dtype=torch.uint8).cuda() if v[0] else torch.empty(0, dtype=torch.uint8).cuda()
             for v in cases.values()]
    status = bitrot_verify_batch(files, want, len(part), algo, S)
    assert status == [v[1] for v in cases.values()], dict(zip(cases, status))
    # the host mirror (bitrot.rs:616-655 read loop) agrees case by case
    for (name, (blob, code)) in cases.items():
        try:
            bitrot_verify(io.BytesIO(blob), want, len(part), algo, S)
            got = _lib.RSG_OK
        except EOFError:
            got = _lib.RSG_ERR_UNEXPECTED_EOF
        except IOError as exc:
            got = {"bitrot hash mismatch": _lib.RSG_ERR_BITROT_MISMATCH,
                   "bitrot shard file has trailing data": _lib.RSG_ERR_TRAILING_DATA}[str(exc)]
        assert got == code, name
    # size mismatch decided before any read
    assert bitrot_verify_batch(files[:1], want + 1, len(part), algo, S) == [_lib.RSG_ERR_FILE_SIZE_MISMATCH]
    # exact multiple of the shard size, and an empty part
    part2 = part[:2 * S]
    f2 = _shard_file(oracle, part2, S, legacy)
    assert bitrot_verify_batch([torch.tensor(list(f2), dtype=torch.uint8).cuda()], len(f2), len(part2), algo, S) == [0]
    assert bitrot_verify_batch([torch.empty(0, dtype=torch.uint8).cuda()], 0, 0, algo, S) == [0]


@pytest.mark.parametrize("k,m,S,n", [(8, 4, 512, 9), (8, 4, 4608, 3), (8, 4, 1024, 1)])
def test_heal_one_pass_short_walks(gpu, oracle, k, m, S, n):
    """One-pass heal over a single 512-byte step, a step count that is not a
    power of two, and a single stripe (seven dead stripes in the workgroup)."""
    import torch
    from rustfs_amd import Erasure
    shards, recs, files = _records(torch, oracle, k, m, S, n, seed=S + n)
    e = Erasure(k, m, k * S)
    rec = 32 + S
    for lost in ((3,), (0, 11), (1, 2, 9, 10)):
        src = [None if i in lost else files[i] for i in range(k + m)]
        tgt = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(k + m)]
        assert e.heal_records_batch(src, tgt, S, n) == [0] * n
        for i in lost:
            assert np.array_equal(tgt[i].cpu().numpy().reshape(n, rec), recs[i]), (lost, i)


@pytest.mark.parametrize("k,m,lost", [(8, 4, (1, 8)), (8, 4, (0,)), (8, 4, (0, 1, 2, 3)), (8, 4, (9, 10, 11)),
                                      (8, 4, (2, 5, 10)), (16, 4, (3, 16)), (16, 4, (0, 7, 15, 19)),
                                      (16, 4, (18,)), (2, 2, (2,)), (2, 2, (0,)), (4, 2, (3,)), (4, 4, (0, 5, 6))])
def test_heal_one_pass_many_workgroups(gpu, oracle, k, m, lost):
    """Heal through the one-pass kernel (verify every source record, write
    every target record with its digest, compare the surplus parity) over
    many workgroups (8 stripes each, 4 for RS(16,4)) and a ragged last one,
    for every geometry with a one-pass kernel: the healed files are
    byte-identical to the originals; a rotten source record is redone from
    other survivors; a re-hashed inconsistent surplus parity fails its stripe
    alone, whose target digests are zeroed."""
    import torch
    from rustfs_amd import Erasure, _lib
    S, n = 4096, 2051
    rec = 32 + S
    e = Erasure(k, m, k * S)
    g = torch.Generator(device="cuda").manual_seed(len(lost) * 7 + lost[0])
    st = torch.zeros((n, k + m, S), dtype=torch.uint8, device="cuda")
    st[:, :k] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    e.encode_batch(st, dig)
    files = [torch.cat([dig[:, i], st[:, i]], dim=1).contiguous().reshape(-1) for i in range(k + m)]
    # the encoded records match the oracle on a sample (so "identical to the originals" is the reference's bytes)
    for s in (0, n - 1):
        ref = st[s].cpu().numpy().copy()
        ref[k:] = 0
        oracle.encode(k, m, ref)
        assert np.array_equal(st[s].cpu().numpy(), ref)
    src = [None if i in lost else files[i].clone() for i in range(k + m)]
    present = [i for i in range(k + m) if i not in lost]
    rot = present[2]
    src[rot][700 * rec + 32 + 5] ^= 0x04            # rotten source record, stripe 700
    bad_stripe = None
    surplus = [i for i in present if i >= k][max(0, k - len([i for i in present if i < k])):]
    if surplus:                                     # a surplus parity, inconsistent but re-hashed, stripe 1500
        f = surplus[-1]
        body = src[f][1500 * rec + 32: 1501 * rec].cpu().numpy().copy()
        body[11] ^= 0x20
        src[f][1500 * rec + 32: 1501 * rec] = torch.from_numpy(body).cuda()
        src[f][1500 * rec: 1500 * rec + 32] = torch.from_numpy(
            np.frombuffer(oracle.hh256s(body.tobytes()), dtype=np.uint8).copy()).cuda()
        bad_stripe = 1500
    tgt = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(k + m)]
    status = e.heal_records_batch(src, tgt, S, n)
    # with exactly k sources the rotten record costs stripe 700 its read quorum
    want = {1500: _lib.RSG_ERR_INCONSISTENT_SOURCES} if bad_stripe is not None else {}
    if len(present) == k:
        want[700] = _lib.RSG_ERR_TOO_FEW_SHARDS
    assert {i: x for i, x in enumerate(status) if x != 0} == want
    for i in lost:
        got = tgt[i].reshape(n, rec)
        ref = files[i].reshape(n, rec)
        ok = torch.ones(n, dtype=torch.bool, device="cuda")
        for b in want:
            ok[b] = False
            assert not bool(got[b, :32].any())  # digest zeroed: never verifies
        assert torch.equal(got[ok], ref[ok]), f"shard {i}"
