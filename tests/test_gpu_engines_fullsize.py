"""The record engines at the bench line's full sizes (the pattern
tests run n <= 19 stripes; the line checked one stripe): RS(8,4) at S = 131072
RS(12,4) at S = 87382 and RS(11,4) at S = 95326 (ragged walks, records at
every even offset), n =
4096 BitrotWriter records per file, through the one-pass kernels the engine
picks at that scale.

Parity and digests of a sample of stripes are checked against the oracle;
then every stripe of every output is compared on the device with the bytes it
must equal (size-independent properties): the in-place GET's rebuilt slots
with the encoded data shards, the healed record files with the encoder's
record files (digest headers included), and a lost disk plus one rotten
record per stripe of another file (the redo path) likewise."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _records(torch, k, m, S, n, seed):
    from rustfs_amd import Erasure
    e = Erasure(k, m, 1 << 20)
    assert e.shard_size() == S
    g = torch.Generator(device="cuda").manual_seed(seed)
    st = torch.empty((n, k + m, S), dtype=torch.uint8, device="cuda")
    for s0 in range(0, n, 256):
        s1 = min(n, s0 + 256)
        st[s0:s1, :k] = torch.randint(0, 256, (s1 - s0, k, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.empty((n, k + m, 32), dtype=torch.uint8, device="cuda")
    e.encode_batch(st, dig)
    files = []
    for i in range(k + m):
        f = torch.empty((n, 32 + S), dtype=torch.uint8, device="cuda")
        f[:, :32] = dig[:, i]
        f[:, 32:] = st[:, i]
        files.append(f.reshape(-1))
    return e, st, dig, files


# RS(11,4): the run-time-table kernel on the 2-slot ring (two workgroups a CU),
# its heal hashing the targets in the last hash wave; RS(8,8) (EC:8 on 16
# drives): the table kernel with 8 row slots (round 5)
@pytest.mark.parametrize("k,m,S", [(8, 4, 131072), (12, 4, 87382), (11, 4, 95326), (8, 8, 131072)])
def test_engines_every_stripe_at_bench_size(gpu, oracle, k, m, S):
    import torch
    n = 4096
    t, rec = k + m, 32 + S
    e, st, dig, files = _records(torch, k, m, S, n, seed=k)
    for s in (0, 1777, n - 1):  # the encoder's parity and digests against the oracle
        ref = st[s].cpu().numpy().copy()
        ref[k:] = 0
        oracle.encode(k, m, ref)
        assert np.array_equal(st[s].cpu().numpy(), ref), s
        d = dig[s].cpu().numpy()
        for i in range(t):
            assert d[i].tobytes() == oracle.hh256s(ref[i]), (s, i)
    # GET with two data disks lost: every stripe's rebuilt shards equal the data
    lost = (0, 3)
    slots = torch.full((n, k * S), 0xA5, dtype=torch.uint8, device="cuda")
    _, src, status = e.decode_records_into_batch([None if i in lost else files[i] for i in range(t)], S, n,
                                                 targets=slots)
    assert status == [0] * n
    for i in range(k):
        assert (not src[i].any()) if i in lost else src[i].all(), i
    got = slots.view(n, k, S)
    for i in lost:
        assert torch.equal(got[:, i], st[:, i]), f"rebuilt shard {i}"
    # heal of one data + one parity disk: the target files equal the encoder's
    tg_idx = (1, k)
    tg = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in tg_idx else None for i in range(t)]
    assert e.heal_records_batch([None if i in tg_idx else files[i] for i in range(t)], tg, S, n) == [0] * n
    for i in tg_idx:
        assert torch.equal(tg[i], files[i]), f"healed file {i}"
    # a lost disk and a rotten record in every 97th stripe of data file 5: the
    # rotten records count as missing for their stripes (redone), all exact
    bad = files[5].clone().view(n, rec)
    rot = torch.arange(0, n, 97, device="cuda")
    bad[rot, 32 + S // 2] ^= 0x5A
    f2 = [None if i == 0 else files[i] for i in range(t)]
    f2[5] = bad.reshape(-1)
    slots.fill_(0xA5)
    _, src, status = e.decode_records_into_batch(f2, S, n, targets=slots)
    assert status == [0] * n
    assert not src[0].any() and not src[5][rot.cpu().numpy()].any() and int(src[5].sum()) == n - rot.numel()
    got = slots.view(n, k, S)
    assert torch.equal(got[:, 0], st[:, 0])
    assert torch.equal(got[rot, 5], st[rot, 5])


@pytest.mark.parametrize("k,m,S,lost", [(8, 8, 131072, (0, 3, 5)), (10, 6, 104858, (1, 4, 7, 12))])
def test_ec58_multi_loss_every_stripe_at_bench_size(gpu, k, m, S, lost):
    """EC:5..8 (storageclass.rs:480-498) at n = 4096 records of 1 MiB blocks
    with three / four shards lost (round 6: the one-pass table kernel with 8
    row slots): the GET's rebuilt data shards equal the encoded data and the
    heal of every lost shard writes the encoder's record files, digest
    headers included, in every stripe."""
    import torch
    n = 4096
    t, rec = k + m, 32 + S
    e, st, dig, files = _records(torch, k, m, S, n, seed=k * 31 + m)
    slots = torch.full((n, k * S), 0xA5, dtype=torch.uint8, device="cuda")
    _, src, status = e.decode_records_into_batch([None if i in lost else files[i] for i in range(t)], S, n,
                                                 targets=slots)
    assert status == [0] * n
    got = slots.view(n, k, S)
    for i in lost:
        if i < k:
            assert not src[i].any() and torch.equal(got[:, i], st[:, i]), f"rebuilt shard {i}"
    tg = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None for i in range(t)]
    assert e.heal_records_batch([None if i in lost else files[i] for i in range(t)], tg, S, n) == [0] * n
    for i in lost:
        assert torch.equal(tg[i], files[i]), f"healed file {i}"
