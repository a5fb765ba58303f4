"""ReedSolomonEncoder::reconstruct semantics on the device-batch path, and
compare mode (verify, GET surplus check, heal parity check) for k > 16.

reconstruct (erasure.rs:425-428) = reconstruct_data from the first k present
shards, then encode_parity_shards (erasure.rs:505-561) re-encodes EVERY parity
shard from the data.  The oracle restates exactly that: reconstruct with
data_only, then encode.  The batch entry point works in place, so these tests
also pin that no launch reads a shard an earlier launch of the same product
overwrote (k > 16 chains launches over the inputs).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle_reconstruct_reencode(oracle, k, m, stripe, present):
    ref = stripe.copy()
    oracle.reconstruct(k, m, ref, present, data_only=True)
    oracle.encode(k, m, ref)
    return ref


def _batch(torch, oracle, k, m, S, n, seed):
    rng = np.random.default_rng(seed)
    host = np.zeros((n, k + m, S), dtype=np.uint8)
    host[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    for s in range(n):
        oracle.encode(k, m, host[s])
    return host


@pytest.mark.parametrize("k,m,S,n,missing,stale", [
    (20, 4, 4096, 3, (0,), ()),              # k > 16: parity 20 is a survivor and an input of the chain
    (20, 4, 1000, 2, (0, 5, 21), ()),
    (8, 8, 4096, 4, (3,), (10,)),             # parity 10 present, not a survivor, stale bytes
    (8, 8, 2048, 2, (0, 1), (9, 15)),
    (8, 4, 131072, 3, (0,), ()),
    (8, 4, 131072, 3, (0, 3), ()),
    (8, 4, 131072, 3, (0, 3, 5), ()),
    (8, 4, 131072, 3, (0, 3, 5, 7), ()),
    (8, 4, 4096, 3, (2, 9), ()),
    (8, 4, 4096, 3, (), (8, 11)),             # nothing missing: every parity re-encoded
    (17, 3, 777, 2, (16, 17), ()),
    (192, 64, 96, 2, tuple(range(0, 192, 6)) + (193, 200), ()),  # R > 8 rows and C > 16 inputs
])
def test_batch_reconstruct_reencode_parity(gpu, oracle, k, m, S, n, missing, stale):
    import torch
    from rustfs_amd import Erasure, RSG_RECONSTRUCT_REENCODE_PARITY
    host = _batch(torch, oracle, k, m, S, n, seed=k * 31 + m + len(missing))
    rng = np.random.default_rng(S)
    for s in range(n):
        for i in stale:  # a present parity that disagrees with the data
            host[s, i, rng.integers(0, S)] ^= 0xA5
        for i in missing:
            host[s, i] = 0x3C  # garbage in the missing slots
    present = [i not in missing for i in range(k + m)]
    want = np.stack([_oracle_reconstruct_reencode(oracle, k, m, host[s], present) for s in range(n)])
    st = torch.from_numpy(host).cuda()
    Erasure(k, m, k * S).reconstruct_batch(st, present, RSG_RECONSTRUCT_REENCODE_PARITY)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    for s in range(n):
        for i in range(k + m):
            assert np.array_equal(got[s, i], want[s, i]), (s, i)


@pytest.mark.parametrize("k,m,S", [(20, 4, 1000), (8, 8, 512)])
def test_host_reconstruct_reencode_matches_batch(gpu, oracle, k, m, S):
    """The host-buffer rsg_reconstruct in REENCODE mode agrees with the oracle
    (and so with the batch path) for a stale non-survivor parity."""
    from rustfs_amd import ReedSolomonEncoder
    host = _batch(None, oracle, k, m, S, 1, seed=99)[0]
    host[k + m - 1, 3] ^= 0x11
    present = [i != 1 for i in range(k + m)]
    want = _oracle_reconstruct_reencode(oracle, k, m, host, present)
    shards = [None if not present[i] else host[i].tobytes() for i in range(k + m)]
    ReedSolomonEncoder(k, m).reconstruct(shards)
    for i in range(k + m):
        assert bytes(shards[i]) == want[i].tobytes(), i


@pytest.mark.parametrize("k,m,S,n", [(20, 4, 52429, 5), (192, 64, 96, 4), (17, 3, 4099, 6)])
def test_verify_batch_wide(gpu, oracle, k, m, S, n):
    """rsg_verify_batch_dev for k > 16 (erasure.rs:430-441): per-stripe flags."""
    import torch
    from rustfs_amd import Erasure
    host = _batch(torch, oracle, k, m, S, n, seed=k + S)
    host[1, k + m - 1, S - 1] ^= 0x01   # last parity, last byte
    host[n - 2, k, 0] ^= 0x80           # first parity, first byte
    st = torch.from_numpy(host).cuda()
    ok = Erasure(k, m, k * S).verify_batch(st).cpu().tolist()
    want = [1] * n
    want[1] = want[n - 2] = 0
    assert ok == want


def _records(torch, oracle, k, m, S, n, seed):
    host = _batch(torch, oracle, k, m, S, n, seed)
    recs = np.zeros((k + m, n, 32 + S), dtype=np.uint8)
    for s in range(n):
        for i in range(k + m):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(host[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = host[s, i]
    return host, recs, [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(k + m)]


@pytest.mark.parametrize("k,m,S,n", [(20, 4, 2048, 4), (200, 8, 64, 3)])
def test_decode_records_surplus_check_wide(gpu, oracle, k, m, S, n):
    """GET engine, k > 16, data lost with surplus parity present: rebuilt data
    exact, and an inconsistent surplus parity (valid digest) is InvalidData
    (erasure.rs:935-973) for its stripe only."""
    import torch
    from rustfs_amd import Erasure, _lib
    host, recs, files = _records(torch, oracle, k, m, S, n, seed=k * 3 + S)
    e = Erasure(k, m, k * S)
    want = torch.from_numpy(host[:, :k].reshape(n, k * S).copy()).cuda()
    f = [None if i in (0, 7) else files[i] for i in range(k + m)]
    out, status = e.decode_records_batch(f, S, n)
    assert status == [0] * n and torch.equal(out, want)
    # surplus parity k+m-1 of stripe 1 re-hashed after a flip: digest valid, bytes wrong
    bad = recs[k + m - 1].copy()
    bad[1, 32 + S // 2] ^= 0x02
    bad[1, :32] = np.frombuffer(oracle.hh256s(bad[1, 32:].tobytes()), dtype=np.uint8)
    f[k + m - 1] = torch.from_numpy(bad.reshape(-1).copy()).cuda()
    out, status = e.decode_records_batch(f, S, n)
    assert status == [0, _lib.RSG_ERR_INCONSISTENT_SOURCES] + [0] * (n - 2)
    assert torch.equal(out[0], want[0]) and torch.equal(out[2:], want[2:])


@pytest.mark.parametrize("k,m,S,n", [(20, 4, 2048, 4), (200, 8, 64, 3)])
def test_heal_parity_check_wide(gpu, oracle, k, m, S, n):
    """Heal, k > 16: targets rebuilt exactly; a source parity that disagrees
    with the re-encoded parity (heal.rs:180-196) fails its stripe, and the
    failed stripe's target records carry a zero digest (never verify)."""
    import torch
    from rustfs_amd import Erasure, _lib
    host, recs, files = _records(torch, oracle, k, m, S, n, seed=k * 5 + S)
    e = Erasure(k, m, k * S)
    rec = 32 + S
    lost = [2, k + 1]
    src = [None if i in lost else files[i] for i in range(k + m)]
    tgt = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(k + m)]
    assert e.heal_records_batch(src, tgt, S, n) == [0] * n
    for i in lost:
        assert np.array_equal(tgt[i].cpu().numpy().reshape(n, rec), recs[i]), i
    bad = recs[k].copy()
    bad[n - 1, 32 + 5] ^= 0x40
    bad[n - 1, :32] = np.frombuffer(oracle.hh256s(bad[n - 1, 32:].tobytes()), dtype=np.uint8)
    src[k] = torch.from_numpy(bad.reshape(-1).copy()).cuda()
    status = e.heal_records_batch(src, tgt, S, n)
    assert status == [0] * (n - 1) + [_lib.RSG_ERR_INCONSISTENT_SOURCES]
    for i in lost:
        got = tgt[i].cpu().numpy().reshape(n, rec)
        assert np.array_equal(got[:n - 1], recs[i][:n - 1]), i
        assert not got[n - 1, :32].any(), i  # poisoned digest header


def test_heal_failed_stripe_digest_poisoned(gpu, oracle):
    """Read quorum lost in one stripe: its target records' digests are zeroed
    (a caller that ignores h_status must not get verifiable records)."""
    import torch
    from rustfs_amd import Erasure, _lib
    k, m, S, n = 4, 2, 1024, 3
    host, recs, files = _records(torch, oracle, k, m, S, n, seed=4)
    rec = 32 + S
    f = [x.clone() for x in files]
    for i in (1, 2, 3):  # stripe 0 loses 3 > m shards (digest bytes)
        f[i][5] ^= 0xFF
    tgt = [None] * (k + m)
    tgt[0] = torch.zeros(n * rec, dtype=torch.uint8, device="cuda")
    status = Erasure(k, m, k * S).heal_records_batch([None] + f[1:], tgt, S, n)
    assert status == [_lib.RSG_ERR_TOO_FEW_SHARDS, 0, 0]
    got = tgt[0].cpu().numpy().reshape(n, rec)
    assert not got[0, :32].any()
    assert np.array_equal(got[1:], recs[0][1:])
