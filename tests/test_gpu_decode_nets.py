"""Every RS(8,4) erasure pattern of one or two lost shards through the one-pass
GET / heal kernel with its compile-time XOR network (k_decode_records_net,
one kernel per pattern; rs84_decode_nets.h): GET (a data shard lost) and heal
(every lost shard a target), on oracle-built BitrotWriter records, over a
ragged batch (19 stripes: two full 8-stripe workgroups and a partial one, so
every 4-stripe network group meets live and dead stripes), bit-exact against
the oracle's shards and digests; then the same pattern with one surplus
parity record of one stripe altered and re-hashed must report
"inconsistent sources" for that stripe only (erasure.rs:935-973,
heal.rs:179-197).  The CPU test test_decode_nets.py pins the networks
themselves."""
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K, M, T = 8, 4, 12
S, N = 1024, 19
REC = 32 + S


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


@pytest.mark.parametrize("lost", [x for x in LOSSES if min(x) < K], ids=str)
def test_get_every_pattern(gpu, oracle, records, one_pass, lost):
    import torch
    from rustfs_amd import Erasure, _lib
    shards, recs, files = records
    e = Erasure(K, M, K * S)
    want = torch.from_numpy(shards[:, :K].reshape(N, K * S).copy()).cuda()
    f = [None if i in lost else files[i] for i in range(T)]
    out, status = e.decode_records_batch(f, S, N)
    assert status == [0] * N and torch.equal(out, want)
    sur = _surplus(lost)
    if sur:
        stripe = sum(lost) % N
        f2 = list(f)
        f2[sur[-1]] = _rehashed(torch, oracle, files[sur[-1]], stripe, 3 * sum(lost) % S)
        out, status = e.decode_records_batch(f2, S, N)
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
