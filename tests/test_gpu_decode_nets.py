"""Every erasure pattern of one or two lost shards through the one-pass GET /
heal kernels: the compile-time XOR-network kernels (k_decode_records_net for
RS(8,4), one kernel per pattern, rs84_decode_nets.h; RS(4,4), RS(6,4),
RS(10,4), RS(12,4) likewise — the patterns read from the generated tables)
and the run-time-table kernel k_decode_records_dma for every other geometry
of at most 16 shards (the odd data counts of 5-, 9-, 15-drive sets and the
reduced-redundancy class: RS(5,4), RS(11,4), RS(15,1), ...; the patterns
generated here).  RS(16,4) (20 shards, more than rustfs stores,
fileinfo.rs:38) has no one-pass kernel: its GET and heal run the two-pass
path, forced or not, and are checked here as that path): GET (a data shard lost) and heal (every lost shard a target), on
oracle-built BitrotWriter records, over a ragged batch (RS(8,4): 19 stripes
= two full 8-stripe workgroups and a partial one, so every 4-stripe network
group meets live and dead stripes; RS(16,4): 11 stripes), bit-exact against the oracle's shards and
digests; then the same pattern with one
surplus parity record of one stripe altered and re-hashed must report
"inconsistent sources" for that stripe only (erasure.rs:935-973,
heal.rs:179-197).  The CPU test test_decode_nets.py pins the networks
themselves."""
import itertools
import os
import re

import numpy as np
import pytest

from conftest import decode_get

pytestmark = pytest.mark.gpu

FORMS = ["gather", "into"]  # rsg_decode_records_dev / rsg_decode_records_into_dev

K, M, T = 8, 4, 12
S, N = 1024, 19
REC = 32 + S
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rustfs_amd", "csrc")


def _listed(header, t):
    """(heal, lost tuple) of every pattern in a generated network table."""
    src = open(os.path.join(CSRC, header)).read()
    out = []
    for m in re.finditer(r"\{0x([0-9a-f]+), (\d), \d+, \d, \d, \{", src):
        mask = int(m.group(1), 16)
        out.append((int(m.group(2)), tuple(i for i in range(t) if mask >> i & 1)))
    return out


@pytest.fixture(scope="module")
def records(gpu, oracle):
    """n stripes of random data, parity and digests from the oracle."""
    import torch
    rng = np.random.default_rng(355)
    shards = np.zeros((N, T, S), dtype=np.uint8)
    recs = np.zeros((T, N, REC), dtype=np.uint8)
    for s in range(N):
        shards[s, :K] = rng.integers(0, 256, (K, S), dtype=np.uint8)
        oracle.encode(K, M, shards[s])
        for i in range(T):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    files = [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(T)]
    return shards, recs, files


@pytest.fixture
def one_pass(gpu):
    from rustfs_amd import _lib
    L = _lib.load()
    _lib.check(L.rsg_set_record_engine(gpu.handle, _lib.RSG_RECORD_ENGINE_ONE_PASS))
    yield
    _lib.check(L.rsg_set_record_engine(gpu.handle, _lib.RSG_RECORD_ENGINE_AUTO))


def _surplus(lost):
    """Present parity beyond the 8 survivors (the compared rows)."""
    files = [i for i in range(T) if i not in lost]
    return files[K:]


def _rehashed(torch, oracle, f, stripe, pos):
    bad = f.clone()
    body = bad[stripe * REC + 32:(stripe + 1) * REC].cpu().numpy().copy()
    body[pos] ^= 0x20
    bad[stripe * REC + 32:(stripe + 1) * REC] = torch.from_numpy(body).cuda()
    bad[stripe * REC:stripe * REC + 32] = torch.from_numpy(
        np.frombuffer(oracle.hh256s(body.tobytes()), dtype=np.uint8).copy()).cuda()
    return bad


LOSSES = [(a,) for a in range(T)] + list(itertools.combinations(range(T), 2))


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("lost", [x for x in LOSSES if min(x) < K], ids=str)
def test_get_every_pattern(gpu, oracle, records, one_pass, lost, form):
    import torch
    from rustfs_amd import Erasure, _lib
    shards, recs, files = records
    e = Erasure(K, M, K * S)
    want = torch.from_numpy(shards[:, :K].reshape(N, K * S).copy()).cuda()
    f = [None if i in lost else files[i] for i in range(T)]
    out, status = decode_get(e, f, S, N, form)
    assert status == [0] * N and torch.equal(out, want)
    sur = _surplus(lost)
    if sur:
        stripe = sum(lost) % N
        f2 = list(f)
        f2[sur[-1]] = _rehashed(torch, oracle, files[sur[-1]], stripe, 3 * sum(lost) % S)
        out, status = decode_get(e, f2, S, N, form)
        assert [i for i, x in enumerate(status) if x] == [stripe]
        assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
        ok = torch.ones(N, dtype=torch.bool, device="cuda")
        ok[stripe] = False
        assert torch.equal(out[ok], want[ok])


@pytest.mark.parametrize("lost", LOSSES, ids=str)
def test_heal_every_pattern(gpu, oracle, records, one_pass, lost):
    import torch
    from rustfs_amd import Erasure, _lib
    shards, recs, files = records
    e = Erasure(K, M, K * S)
    src = [None if i in lost else files[i] for i in range(T)]
    tgt = [torch.zeros(N * REC, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T)]
    status = e.heal_records_batch(src, tgt, S, N)
    assert status == [0] * N
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(N, REC), recs[i]), f"shard {i}"
    sur = _surplus(lost)
    if sur:
        stripe = (5 * sum(lost) + 1) % N
        src2 = list(src)
        src2[sur[0]] = _rehashed(torch, oracle, files[sur[0]], stripe, 7 * sum(lost) % S)
        tgt2 = [torch.zeros(N * REC, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T)]
        status = e.heal_records_batch(src2, tgt2, S, N)
        assert [i for i, x in enumerate(status) if x] == [stripe]
        assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
        for i in lost:
            got = tgt2[i].cpu().numpy().reshape(N, REC)
            keep = [s for s in range(N) if s != stripe]
            assert np.array_equal(got[keep], recs[i][keep]), f"shard {i}"


def _every_pattern(k, m):
    """(heal, lost) of every one- and two-shard loss: GET needs a data shard
    among the lost (else nothing is rebuilt), heal takes every loss."""
    t = k + m
    losses = [(i,) for i in range(t)] + (list(itertools.combinations(range(t), 2)) if m >= 2 else [])
    return [(0, lost) for lost in losses if min(lost) < k] + [(1, lost) for lost in losses]


# ---------------------------------------------------------------- RS(16,4)
# no one-pass kernel since round 5 (rustfs cannot store 20 shards,
# fileinfo.rs:38; one_pass_geometry requires k + m <= 16): GET and heal run
# the two-pass path whatever the record-engine setting
K16, T16, N16 = 16, 20, 11
LISTED16 = _every_pattern(16, 4)


@pytest.fixture(scope="module")
def records16(gpu, oracle):
    import torch
    rng = np.random.default_rng(164)
    shards = np.zeros((N16, T16, S), dtype=np.uint8)
    recs = np.zeros((T16, N16, REC), dtype=np.uint8)
    for s in range(N16):
        shards[s, :K16] = rng.integers(0, 256, (K16, S), dtype=np.uint8)
        oracle.encode(K16, 4, shards[s])
        for i in range(T16):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    files = [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(T16)]
    return shards, recs, files


@pytest.mark.parametrize("heal,lost", LISTED16, ids=lambda x: str(x))
def test_rs16_every_listed_pattern(gpu, oracle, records16, one_pass, heal, lost):
    for form in FORMS if not heal else [None]:
        _rs16_pattern(oracle, records16, heal, lost, form)


def _rs16_pattern(oracle, records16, heal, lost, form):
    import torch
    from rustfs_amd import Erasure, _lib
    shards, recs, files = records16
    e = Erasure(K16, 4, K16 * S)
    present = [i for i in range(T16) if i not in lost]
    sur = present[K16:]
    if not heal:
        want = torch.from_numpy(shards[:, :K16].reshape(N16, K16 * S).copy()).cuda()
        f = [None if i in lost else files[i] for i in range(T16)]
        out, status = decode_get(e, f, S, N16, form)
        assert status == [0] * N16 and torch.equal(out, want)
        if sur:
            stripe = sum(lost) % N16
            f2 = list(f)
            f2[sur[-1]] = _rehashed(torch, oracle, files[sur[-1]], stripe, 3 * sum(lost) % S)
            out, status = decode_get(e, f2, S, N16, form)
            assert [i for i, x in enumerate(status) if x] == [stripe]
            assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
            ok = torch.ones(N16, dtype=torch.bool, device="cuda")
            ok[stripe] = False
            assert torch.equal(out[ok], want[ok])
        return
    src = [None if i in lost else files[i] for i in range(T16)]
    tgt = [torch.zeros(N16 * REC, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T16)]
    assert e.heal_records_batch(src, tgt, S, N16) == [0] * N16
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(N16, REC), recs[i]), f"shard {i}"
    if sur:
        stripe = (5 * sum(lost) + 1) % N16
        src2 = list(src)
        src2[sur[0]] = _rehashed(torch, oracle, files[sur[0]], stripe, 7 * sum(lost) % S)
        tgt2 = [torch.zeros(N16 * REC, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T16)]
        status = e.heal_records_batch(src2, tgt2, S, N16)
        assert [i for i, x in enumerate(status) if x] == [stripe]
        assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
        keep = [s for s in range(N16) if s != stripe]
        for i in lost:
            assert np.array_equal(tgt2[i].cpu().numpy().reshape(N16, REC)[keep], recs[i][keep]), f"shard {i}"


# ---------------------------------------------------------------- RS(12,4)
# the default geometry of a 16-drive set (storageclass.rs:24-31); S12 = 1000:
# a ragged walk (one whole 512-byte step and 488 bytes), records at every
# alignment (pitch 1032)
K12, T12, N12, S12 = 12, 16, 11, 1000
REC12 = 32 + S12
LISTED12 = _listed("rs124_decode_nets.h", T12)


@pytest.fixture(scope="module")
def records12(gpu, oracle):
    import torch
    rng = np.random.default_rng(124)
    shards = np.zeros((N12, T12, S12), dtype=np.uint8)
    recs = np.zeros((T12, N12, REC12), dtype=np.uint8)
    for s in range(N12):
        shards[s, :K12] = rng.integers(0, 256, (K12, S12), dtype=np.uint8)
        oracle.encode(K12, 4, shards[s])
        for i in range(T12):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    files = [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(T12)]
    return shards, recs, files


def _rehashed12(torch, oracle, f, stripe, pos):
    bad = f.clone()
    body = bad[stripe * REC12 + 32:(stripe + 1) * REC12].cpu().numpy().copy()
    body[pos] ^= 0x20
    bad[stripe * REC12 + 32:(stripe + 1) * REC12] = torch.from_numpy(body).cuda()
    bad[stripe * REC12:stripe * REC12 + 32] = torch.from_numpy(
        np.frombuffer(oracle.hh256s(body.tobytes()), dtype=np.uint8).copy()).cuda()
    return bad


def test_rs12_table_lists_every_pattern():
    """Every one- and two-shard loss of RS(12,4): 12 + 114 GET patterns (a
    data shard among the lost) and 16 + 120 heal patterns, plus the heal of
    all four parity shards (the encode's rows)."""
    assert len([x for x in LISTED12 if not x[0]]) == 12 + 114
    assert len([x for x in LISTED12 if x[0]]) == 16 + 120 + 1
    assert (1, (12, 13, 14, 15)) in LISTED12


@pytest.mark.parametrize("heal,lost", LISTED12, ids=lambda x: str(x))
def test_rs12_every_listed_pattern(gpu, oracle, records12, one_pass, heal, lost):
    """k_decode_records_net12 (four network waves over survivors 0-2 / 3-5 /
    6-8 / 9-11, each finishing one row), on a ragged walk: GET in both forms
    and heal, bit-exact against the oracle, with an altered surplus parity (in
    the ragged last step; which surplus — so which wave compares it — varies
    with the pattern) reported for its stripe alone."""
    import torch
    from rustfs_amd import Erasure, _lib
    shards, recs, files = records12
    e = Erasure(K12, 4, K12 * S12)
    present = [i for i in range(T12) if i not in lost]
    sur = present[K12:]
    if not heal:
        want = torch.from_numpy(shards[:, :K12].reshape(N12, K12 * S12).copy()).cuda()
        f = [None if i in lost else files[i] for i in range(T12)]
        for form in FORMS:
            out, status = decode_get(e, f, S12, N12, form)
            assert status == [0] * N12 and torch.equal(out, want), form
        if sur:
            stripe = sum(lost) % N12
            f2 = list(f)
            bad = sur[sum(lost) % len(sur)]
            f2[bad] = _rehashed12(torch, oracle, files[bad], stripe, 600 + sum(lost))
            for form in FORMS:
                out, status = decode_get(e, f2, S12, N12, form)
                assert [i for i, x in enumerate(status) if x] == [stripe], form
                assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
                ok = torch.ones(N12, dtype=torch.bool, device="cuda")
                ok[stripe] = False
                assert torch.equal(out[ok], want[ok])
        return
    src = [None if i in lost else files[i] for i in range(T12)]
    tgt = [torch.zeros(N12 * REC12, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T12)]
    assert e.heal_records_batch(src, tgt, S12, N12) == [0] * N12
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(N12, REC12), recs[i]), f"shard {i}"
    if sur:
        stripe = (5 * sum(lost) + 1) % N12
        src2 = list(src)
        bad = sur[(sum(lost) + 1) % len(sur)]
        src2[bad] = _rehashed12(torch, oracle, files[bad], stripe, 7 * sum(lost) % S12)
        tgt2 = [torch.zeros(N12 * REC12, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T12)]
        status = e.heal_records_batch(src2, tgt2, S12, N12)
        assert [i for i, x in enumerate(status) if x] == [stripe]
        assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
        keep = [s for s in range(N12) if s != stripe]
        for i in lost:
            assert np.array_equal(tgt2[i].cpu().numpy().reshape(N12, REC12)[keep], recs[i][keep]), f"shard {i}"


# ------------------------------------------------------- RS(6,4), RS(10,4)
# the default geometries of 10- and 14-drive sets (storageclass.rs:24-31) on
# ragged walks: RS(6,4) with S = 1001 (records at odd offsets), RS(10,4) with
# S = 1002 (records 2 mod 8, as at 1 MiB blocks)
GEOS = {(6, 4): (11, 1001), (10, 4): (9, 1002), (4, 4): (13, 1003),
        # the table kernel at odd k (round 5): RS(5,4) 9 drives, RS(11,4) 15
        # drives, RS(15,1) the reduced-redundancy class of 16 drives, RS(3,2),
        # RS(7,1), RS(13,3), RS(1,1) (2 drives) — ragged S, records at every
        # alignment mod 8
        (5, 4): (19, 1005), (11, 4): (9, 1006), (15, 1): (11, 1007), (3, 2): (17, 999), (7, 1): (19, 1011),
        (13, 3): (5, 1013), (1, 1): (9, 997), (9, 4): (7, 1019),
        # C = 14 heals with the target hashing merged into the last hash wave
        (14, 2): (7, 1021),
        # explicit classes EC:5..8 (m > 4, m <= k, k + m <= 16 drives,
        # storageclass.rs:480-498): the table kernel with 8 row slots
        (8, 8): (7, 1031), (10, 6): (5, 1033), (5, 5): (9, 1035), (11, 5): (5, 1037), (7, 7): (7, 1039),
        (9, 7): (5, 1041)}
LISTED6 = _listed("rs64_decode_nets.h", 10)
LISTED10 = _listed("rs104_decode_nets.h", 14)


def _geo_records(oracle, k, m=4):
    import torch
    n, S = GEOS[(k, m)]
    t, rec = k + m, 32 + S
    rng = np.random.default_rng(k * 7 + m)
    shards = np.zeros((n, t, S), dtype=np.uint8)
    recs = np.zeros((t, n, rec), dtype=np.uint8)
    for s in range(n):
        shards[s, :k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
        oracle.encode(k, m, shards[s])
        for i in range(t):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    return shards, recs, [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(t)]


@pytest.fixture(scope="module")
def records6(gpu, oracle):
    return _geo_records(oracle, 6, 4)


@pytest.fixture(scope="module")
def records10(gpu, oracle):
    return _geo_records(oracle, 10, 4)


def test_rs6_rs10_tables_list_every_pattern():
    """Every one- and two-shard loss: RS(6,4) 6 + 39 GET patterns (a data
    shard among the lost) and 10 + 45 heal patterns; RS(10,4) 10 + 85 and
    14 + 91; each + the heal of all four parity shards (the fused encode's)."""
    assert len([x for x in LISTED6 if not x[0]]) == 6 + 39 and len([x for x in LISTED6 if x[0]]) == 10 + 45 + 1
    assert len([x for x in LISTED10 if not x[0]]) == 10 + 85 and len([x for x in LISTED10 if x[0]]) == 14 + 91 + 1


def _geo_case(oracle, k, data, heal, lost, m=4):
    """GET in both forms and heal of one pattern, bit-exact against the
    oracle, with an altered surplus parity reported for its stripe alone."""
    import torch
    from rustfs_amd import Erasure, _lib
    n, S = GEOS[(k, m)]
    t, rec = k + m, 32 + S
    shards, recs, files = data
    e = Erasure(k, m, k * S)
    present = [i for i in range(t) if i not in lost]
    sur = present[k:]

    def rehashed(f, stripe, pos):
        bad = f.clone()
        body = bad[stripe * rec + 32:(stripe + 1) * rec].cpu().numpy().copy()
        body[pos] ^= 0x40
        bad[stripe * rec + 32:(stripe + 1) * rec] = torch.from_numpy(body).cuda()
        bad[stripe * rec:stripe * rec + 32] = torch.from_numpy(
            np.frombuffer(oracle.hh256s(body.tobytes()), dtype=np.uint8).copy()).cuda()
        return bad

    if not heal:
        want = torch.from_numpy(shards[:, :k].reshape(n, k * S).copy()).cuda()
        f = [None if i in lost else files[i] for i in range(t)]
        for form in FORMS:
            out, status = decode_get(e, f, S, n, form)
            assert status == [0] * n and torch.equal(out, want), form
        if sur:
            stripe = sum(lost) % n
            bad = sur[sum(lost) % len(sur)]
            f2 = list(f)
            f2[bad] = rehashed(files[bad], stripe, 700 + sum(lost))
            for form in FORMS:
                out, status = decode_get(e, f2, S, n, form)
                assert [i for i, x in enumerate(status) if x] == [stripe], form
                assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
        return
    src = [None if i in lost else files[i] for i in range(t)]
    tgt = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(t)]
    assert e.heal_records_batch(src, tgt, S, n) == [0] * n
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(n, rec), recs[i]), f"shard {i}"
    if sur:
        stripe = (3 * sum(lost) + 2) % n
        bad = sur[(sum(lost) + 1) % len(sur)]
        src2 = list(src)
        src2[bad] = rehashed(files[bad], stripe, 5 * sum(lost) % S)
        tgt2 = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(t)]
        status = e.heal_records_batch(src2, tgt2, S, n)
        assert [i for i, x in enumerate(status) if x] == [stripe]
        assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES


@pytest.mark.parametrize("heal,lost", LISTED6, ids=lambda x: str(x))
def test_rs6_every_listed_pattern(gpu, oracle, records6, one_pass, heal, lost):
    """k_decode_records_net6 (rs_decode_net.hip over 6 survivors)."""
    _geo_case(oracle, 6, records6, heal, lost, 4)


@pytest.mark.parametrize("heal,lost", LISTED10, ids=lambda x: str(x))
def test_rs10_every_listed_pattern(gpu, oracle, records10, one_pass, heal, lost):
    """k_decode_records_net10 (rs_decode_netq.hip, parts of 3, 3, 2, 2
    survivors; GET on a 2-slot ring with two workgroups per CU, heal one
    workgroup on a 4-slot ring)."""
    _geo_case(oracle, 10, records10, heal, lost, 4)


TABLE_GEOS = [(5, 4), (11, 4), (15, 1), (3, 2), (7, 1), (13, 3), (1, 1), (9, 4), (14, 2), (4, 4),
              (8, 8), (10, 6), (5, 5), (11, 5), (7, 7), (9, 7)]
TABLE_CASES = [(k, m, heal, lost) for k, m in TABLE_GEOS for heal, lost in _every_pattern(k, m)]


@pytest.fixture(scope="module")
def table_records(gpu, oracle):
    cache = {}

    def get(k, m):
        if (k, m) not in cache:
            cache[(k, m)] = _geo_records(oracle, k, m)
        return cache[(k, m)]
    return get


def _multi_loss_patterns(k, m, count, seed, losses=(3, 4)):
    """`count` patterns of RS(k, m) per loss count in `losses` (seeded
    sample, every one with a data shard among the lost for the GET), each as
    a GET and as the heal of every lost shard — EC:5..8's one-pass kernels
    for three to m lost drives (round 6)."""
    rng = np.random.default_rng(seed)
    t, out = k + m, []
    for e in losses:
        seen = set()
        while len(seen) < count:
            lost = tuple(sorted(int(x) for x in rng.choice(t, e, replace=False)))
            if min(lost) < k:
                seen.add(lost)
        for lost in sorted(seen):
            out += [(k, m, 0, lost), (k, m, 1, lost)]
    return out


MULTI_CASES = (_multi_loss_patterns(8, 8, 12, 88) + _multi_loss_patterns(10, 6, 12, 106) +
               _multi_loss_patterns(5, 5, 6, 55) + _multi_loss_patterns(9, 7, 6, 97))


@pytest.mark.parametrize("k,m,heal,lost", MULTI_CASES, ids=str)
@pytest.mark.parametrize("engine", ["one_pass", "two_pass"])
def test_ec58_three_four_lost(gpu, oracle, table_records, engine, k, m, heal, lost):
    """EC:5..8 (m = 5..8 parity shards, storageclass.rs:480-498) with three
    and four shards lost: GET in both forms and the heal of every lost shard,
    bit-exact against the oracle's shards and digests, an altered surplus
    parity reported for its stripe alone — through the one-pass table kernel
    (8 row slots: missing + surplus <= m) and through the two-pass path."""
    from rustfs_amd import _lib
    L = _lib.load()
    code = _lib.RSG_RECORD_ENGINE_ONE_PASS if engine == "one_pass" else _lib.RSG_RECORD_ENGINE_TWO_PASS
    _lib.check(L.rsg_set_record_engine(gpu.handle, code))
    try:
        _geo_case(oracle, k, table_records(k, m), heal, lost, m)
    finally:
        _lib.check(L.rsg_set_record_engine(gpu.handle, _lib.RSG_RECORD_ENGINE_AUTO))


MANY_CASES = (_multi_loss_patterns(8, 8, 12, 808, range(5, 9)) + _multi_loss_patterns(10, 6, 10, 1006, (5, 6)) +
              _multi_loss_patterns(7, 7, 10, 707, range(5, 8)) + _multi_loss_patterns(11, 5, 10, 1105, (5,)) +
              _multi_loss_patterns(9, 7, 8, 907, (5, 6, 7)))


@pytest.mark.parametrize("k,m,heal,lost", MANY_CASES, ids=str)
@pytest.mark.parametrize("engine", ["one_pass", "two_pass"])
def test_ec58_five_or_more_lost(gpu, oracle, table_records, engine, k, m, heal, lost):
    """EC:5..8 with five to m shards lost (seeded samples of RS(8,8), RS(10,6),
    RS(7,7), RS(11,5), RS(9,7); every parity shard spent at RS(8,8) with 8
    lost: no surplus to compare): GET in both forms and the heal of
    every lost shard, bit-exact against the oracle, through the one-pass
    table kernel (round 6) and through the two-pass path."""
    test_ec58_three_four_lost(gpu, oracle, table_records, engine, k, m, heal, lost)


EC5_MANY = [(heal, lost) for e in (3, 4, 5) for lost in itertools.combinations(range(10), e) for heal in (0, 1)
            if heal or min(lost) < 5]


@pytest.mark.parametrize("heal,lost", EC5_MANY, ids=str)
def test_ec5_every_three_to_five_loss_pattern(gpu, oracle, table_records, heal, lost):
    """RS(5,5) (EC:5 on 10 drives) with every choice of three, four and five
    lost shards (five: the most the class survives; one and two are in
    test_table_kernel_every_pattern): GET (every pattern with a data shard
    lost) and the heal of all of them, through the one-pass table kernel
    (round 6: R = lost data + surplus rows a step, gf_rows for R = 5, the
    per-row loop below; an altered surplus parity reported where one is
    left)."""
    test_ec58_three_four_lost(gpu, oracle, table_records, "one_pass", 5, 5, heal, lost)


def test_table_patterns_cover_every_loss():
    """RS(5,4): 5 + (36 - 6) GET (every pair but the 6 all-parity ones) and
    9 + 36 heal patterns; RS(15,1): 15 GET and 16 heal (one parity shard: one
    loss at most); RS(11,4) 11 + (105 - 6) and 15 + 105; RS(8,8) (EC:8 on
    16 drives) 8 + (120 - 28) and 16 + 120."""
    def count(k, m, heal):
        return len([x for x in _every_pattern(k, m) if x[0] == heal])
    assert (count(5, 4, 0), count(5, 4, 1)) == (5 + 30, 9 + 36)
    assert (count(15, 1, 0), count(15, 1, 1)) == (15, 16)
    assert (count(11, 4, 0), count(11, 4, 1)) == (11 + 99, 15 + 105)
    assert (count(8, 8, 0), count(8, 8, 1)) == (8 + 92, 16 + 120)


@pytest.mark.parametrize("k,m,heal,lost", TABLE_CASES, ids=str)
def test_table_kernel_every_pattern(gpu, oracle, table_records, one_pass, k, m, heal, lost):
    """The run-time-table one-pass kernel (k_decode_records_dma, one part per
    survivor count) at the data counts without networks and at m > 4 (8 row
    slots): every one- and two-shard loss, GET in both forms and heal, ragged
    S."""
    _geo_case(oracle, k, table_records(k, m), heal, lost, m)


def test_rs16_heal_three_lost(gpu, oracle, records16, one_pass):
    """A heal of three lost shards at RS(16,4) (the two-pass path: no
    one-pass kernel covers 20 shards, even with the one-pass engine forced):
    bit-exact."""
    import torch
    from rustfs_amd import Erasure
    shards, recs, files = records16
    e = Erasure(K16, 4, K16 * S)
    lost = (2, 9, 17)
    src = [None if i in lost else files[i] for i in range(T16)]
    tgt = [torch.zeros(N16 * REC, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(T16)]
    assert e.heal_records_batch(src, tgt, S, N16) == [0] * N16
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(N16, REC), recs[i]), f"shard {i}"


_TABLE_SNIPPET = r"""
import sys, numpy as np, torch
sys.path.insert(0, {root!r})
from rustfs_amd import Erasure, _lib
from oracle import oracle as O
L = _lib.load()
_lib.check(L.rsg_set_record_engine(_lib.context(0).handle, _lib.RSG_RECORD_ENGINE_ONE_PASS))
S = 1024
REC = 32 + S
for k, n, gets, heals in ((8, 19, [(0, 3), (2, 9), (5,)], [(1, 8), (0, 11), (4,)]), (16, 11, [(0, 3)], [(1, 16)]),
                          (12, 7, [(0, 3), (1,)], [(2, 13)])):
    t = k + 4
    rng = np.random.default_rng(k)
    shards = np.zeros((n, t, S), dtype=np.uint8)
    recs = np.zeros((t, n, REC), dtype=np.uint8)
    for s in range(n):
        shards[s, :k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
        O.encode(k, 4, shards[s])
        for i in range(t):
            recs[i, s, :32] = np.frombuffer(O.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    files = [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(t)]
    e = Erasure(k, 4, k * S)
    want = torch.from_numpy(shards[:, :k].reshape(n, k * S).copy()).cuda()
    for lost in gets:
        out, status = e.decode_records_batch([None if i in lost else files[i] for i in range(t)], S, n)
        assert status == [0] * n and torch.equal(out, want), (k, lost)
    for lost in heals:
        tgt = [torch.zeros(n * REC, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(t)]
        assert e.heal_records_batch([None if i in lost else files[i] for i in range(t)], tgt, S, n) == [0] * n
        for i in lost:
            assert np.array_equal(tgt[i].cpu().numpy().reshape(n, REC), recs[i]), (k, lost, i)
print("ok")
"""


@pytest.mark.parametrize("env", [{"RSG_DECODE_NET": "0"}, {"RSG_GET_CACHED": "0"}])
def test_network_knobs(gpu, oracle, env):
    """The A/B knobs of the network GET/heal path, set through rsg_set_tuning
    for this test alone: RSG_DECODE_NET=0 sends listed RS(8,4) / RS(12,4)
    patterns to the run-time-table one-pass kernel; RSG_GET_CACHED=0 makes the
    RS(8,4) network kernel's stores non-temporal.  Bit-exact against the
    oracle either way.  (RSG_NET12_RD=4 exists in measurement builds only.)"""
    from rustfs_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        with _lib.tuned(**env):
            exec(_TABLE_SNIPPET.format(root=root), {})
    finally:  # the snippet forces the one-pass engine on the shared context
        _lib.check(_lib.load().rsg_set_record_engine(gpu.handle, _lib.RSG_RECORD_ENGINE_AUTO))


# ------------------------------------------------- long shards (the ring wraps)
SL = 4096  # 8 steps of 512 B: the 3-slot ring, the A/B exchange and the trailing target hashers wrap


def _long_records(oracle, k, n, seed, S=SL):
    import torch
    t = k + 4
    rng = np.random.default_rng(seed)
    shards = np.zeros((n, t, S), dtype=np.uint8)
    recs = np.zeros((t, n, 32 + S), dtype=np.uint8)
    for s in range(n):
        shards[s, :k] = rng.integers(0, 256, (k, S), dtype=np.uint8)
        oracle.encode(k, 4, shards[s])
        for i in range(t):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    return shards, recs, [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(t)]


# one pattern of each distinct kernel shape (present files, targets, stored and compared rows)
LONG = [(8, 19, 0, (0,)), (8, 19, 0, (0, 3)), (8, 19, 0, (2, 9)), (8, 19, 0, (6, 11)),
        (8, 19, 1, (8,)), (8, 19, 1, (5,)), (8, 19, 1, (1, 8)), (8, 19, 1, (0, 5)), (8, 19, 1, (9, 11)),
        (16, 11, 0, (3,)), (16, 11, 0, (2, 11)), (16, 11, 0, (4, 17)),
        (16, 11, 1, (17,)), (16, 11, 1, (1, 16)), (16, 11, 1, (0, 5)), (16, 11, 1, (7,))]
# ragged walks at the production shard sizes: RS(12,4) at 1 MiB (S = 87382,
# 170 steps + 342 bytes), RS(10,4) (104858) and RS(6,4) (174763, records at
# odd offsets), and RS(8,4) with a ragged tail (S = 4100)
LONG_RAGGED = [(12, 5, 0, (0,), 87382), (12, 5, 0, (2, 13), 87382), (12, 5, 1, (3, 14), 87382),
               (12, 5, 1, (15,), 87382), (12, 6, 0, (5, 7), 4100), (8, 9, 0, (0, 3), 4100), (8, 9, 1, (1, 8), 4100),
               (8, 9, 0, (2,), 4100), (16, 5, 0, (4, 17), 65540), (16, 5, 1, (1, 16), 65540),
               (10, 5, 0, (0, 3), 104858), (10, 5, 1, (2, 11), 104858), (6, 5, 0, (1, 4), 174763),
               (6, 5, 1, (0, 7), 174763), (4, 9, 0, (0, 5), 262144), (4, 9, 1, (2, 6), 262144)]


@pytest.mark.parametrize("k,n,heal,lost,S", LONG_RAGGED, ids=str)
def test_long_ragged_walks(gpu, oracle, one_pass, k, n, heal, lost, S):
    """Ragged record walks (S not a multiple of the 512-byte step, records at
    every alignment) through the network kernels: GET in both forms and heal,
    bit-exact; an inconsistent surplus flagged in the last stripe."""
    _long_case(oracle, k, n, heal, lost, S)


@pytest.mark.parametrize("k,n,heal,lost", LONG, ids=str)
def test_long_shards_every_shape(gpu, oracle, one_pass, k, n, heal, lost):
    """the per-pattern tests use 2 steps per shard, fewer than the
    3-slot ring; here one pattern of each kernel shape runs 8 steps, GET in
    both forms and heal, bit-exact against the oracle, with an inconsistent
    surplus caught for its stripe alone."""
    _long_case(oracle, k, n, heal, lost, SL)


def _long_case(oracle, k, n, heal, lost, SL):
    import torch
    from rustfs_amd import Erasure, _lib
    t = k + 4
    shards, recs, files = _long_records(oracle, k, n, seed=k * 100 + sum(lost), S=SL)
    e = Erasure(k, 4, k * SL)
    rec = 32 + SL
    present = [i for i in range(t) if i not in lost]
    sur = present[k:]
    if not heal:
        want = torch.from_numpy(shards[:, :k].reshape(n, k * SL).copy()).cuda()
        f = [None if i in lost else files[i] for i in range(t)]
        for form in FORMS:
            out, status = decode_get(e, f, SL, n, form)
            assert status == [0] * n and torch.equal(out, want), form
        if sur:
            stripe = n - 1
            f2 = list(f)
            bad = files[sur[-1]].clone()
            body = bad[stripe * rec + 32:(stripe + 1) * rec].cpu().numpy().copy()
            body[SL - 5] ^= 0x04  # in the last step
            bad[stripe * rec + 32:(stripe + 1) * rec] = torch.from_numpy(body).cuda()
            bad[stripe * rec:stripe * rec + 32] = torch.from_numpy(
                np.frombuffer(oracle.hh256s(body.tobytes()), dtype=np.uint8).copy()).cuda()
            f2[sur[-1]] = bad
            for form in FORMS:
                out, status = decode_get(e, f2, SL, n, form)
                assert [i for i, x in enumerate(status) if x] == [stripe], form
                assert status[stripe] == _lib.RSG_ERR_INCONSISTENT_SOURCES
                assert torch.equal(out[:stripe], want[:stripe])
        return
    src = [None if i in lost else files[i] for i in range(t)]
    tgt = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(t)]
    assert e.heal_records_batch(src, tgt, SL, n) == [0] * n
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(n, rec), recs[i]), f"shard {i}"
