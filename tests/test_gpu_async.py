"""Asynchronous record engines (rsg_decode_records_submit /
rsg_heal_records_submit, ABI 5): tickets shared with the host-batch PUT,
per-call scratch (no context-wide lock), so GETs and heals from several
threads on one context run concurrently — the shape of the reference's
decode pipeline, where many tokio tasks read and decode blocks at once
(decode.rs:1702-1968) — each bit-exact against oracle-built records."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K, M, T = 8, 4, 12


def _oracle_records(torch, oracle, S, n, seed):
    rng = np.random.default_rng(seed)
    shards = np.zeros((n, T, S), dtype=np.uint8)
    recs = np.zeros((T, n, 32 + S), dtype=np.uint8)
    for s in range(n):
        shards[s, :K] = rng.integers(0, 256, (K, S), dtype=np.uint8)
        oracle.encode(K, M, shards[s])
        for i in range(T):
            recs[i, s, :32] = np.frombuffer(oracle.hh256s(shards[s, i].tobytes()), dtype=np.uint8)
            recs[i, s, 32:] = shards[s, i]
    return shards, recs, [torch.from_numpy(recs[i].reshape(-1).copy()).cuda() for i in range(T)]


def test_submit_then_wait_and_poll(gpu, oracle):
    """Several GETs in flight on one stream before any wait; waited out of
    order; a polled ticket completes; results identical to the synchronous
    forms."""
    import torch
    from rustfs_amd import Erasure
    S, n = 4096, 37
    shards, recs, files = _oracle_records(torch, oracle, S, n, seed=1)
    e = Erasure(K, M, K * S)
    want = torch.from_numpy(shards[:, :K].reshape(n, K * S).copy()).cuda()
    lost = [None if i in (1, 6) else files[i] for i in range(T)]
    tickets = [e.decode_records_submit(files, S, n), e.decode_records_submit(lost, S, n),
               e.decode_records_submit(lost, S, n, inplace=True), e.decode_records_submit(files, S, n, inplace=True)]
    out, status = tickets[1].wait()
    assert status == [0] * n and torch.equal(out, want)
    slots, src, status = tickets[2].wait()
    assert status == [0] * n and not src[1].any() and not src[6].any() and src[[0, 2, 3, 4, 5, 7]].all()
    assert torch.equal(slots.view(n, K, S)[:, 1], want.view(n, K, S)[:, 1])
    while not tickets[3].poll():
        pass
    _, src, status = tickets[3].wait()
    assert status == [0] * n and src.all()
    out, status = tickets[0].wait()
    assert status == [0] * n and torch.equal(out, want)
    from rustfs_amd import _lib
    assert _lib.load().rsg_wait(gpu.handle, tickets[0].ticket) == _lib.RSG_ERR_INVALID_ARG  # released
    assert tickets[0].wait()[1] == [0] * n  # the ticket object keeps its result


def test_four_threads_decode_and_heal(gpu, oracle):
    """4 threads, each on its own stream, each submitting GETs (both forms,
    lost disks) and heals on the one shared context and waiting on them:
    every result bit-exact against the oracle's shards and records."""
    import torch
    from rustfs_amd import Erasure
    S, n = 4096, 64
    shards, recs, files = _oracle_records(torch, oracle, S, n, seed=2)
    want = torch.from_numpy(shards[:, :K].reshape(n, K * S).copy()).cuda()
    errors = []

    def worker(w):
        try:
            e = Erasure(K, M, K * S)
            stream = torch.cuda.Stream()
            rec = 32 + S
            for it in range(6):
                lost = ((w + it) % K, K + (w % M))
                f = [None if i in lost else files[i] for i in range(T)]
                with torch.cuda.stream(stream):  # the targets' fill is ordered before the heal on this stream
                    tg = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in lost else None
                          for i in range(T)]
                    t1 = e.decode_records_submit(f, S, n, stream=stream)
                    t2 = e.decode_records_submit(f, S, n, inplace=True, stream=stream)
                    t3 = e.heal_records_submit(f, tg, S, n, stream=stream)
                out, status = t1.wait()
                assert status == [0] * n and torch.equal(out, want), ("gather", w, it)
                slots, src, status = t2.wait()
                assert status == [0] * n, ("into", w, it)
                d = lost[0]
                assert not src[d].any() and torch.equal(slots.view(n, K, S)[:, d], want.view(n, K, S)[:, d])
                assert t3.wait() == [0] * n, ("heal", w, it)
                for i in lost:
                    assert np.array_equal(tg[i].cpu().numpy().reshape(n, rec), recs[i]), ("heal", w, it, i)
        except Exception as exc:  # pragma: no cover - reported below
            errors.append(exc)

    ths = [threading.Thread(target=worker, args=(w,)) for w in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[0]


def _rot(torch, f, stripe, S, pos):
    """The record's body altered, its digest left: a bitrot mismatch."""
    bad = f.clone()
    off = stripe * (32 + S) + 32 + pos
    bad[off] = bad[off] ^ 0x10
    return bad


def test_rotten_records_redone_async(gpu, oracle):
    """a submitted GET and heal that each meet a rotten record
    (verify-before-use, bitrot.rs:227-247: the record counts as missing for its
    stripe, which the finishing step redoes) with a second job queued behind
    them on the same stream, waited out of order; then the same calls again,
    reusing the returned scratch.  Outputs, h_src and statuses bit-exact."""
    import torch
    from rustfs_amd import Erasure, _lib
    S, n = 1024, 1100  # >= 1024 stripes: the one-pass kernels, as the engine picks at scale
    shards, recs, files = _oracle_records(torch, oracle, S, n, seed=3)
    e = Erasure(K, M, K * S)
    rec = 32 + S
    want = torch.from_numpy(shards[:, :K].reshape(n, K * S).copy()).cuda()
    get_src = [None if i in (1, 6) else files[i] for i in range(T)]
    get_src[3] = _rot(torch, files[3], 5, S, 77)            # stripe 5: data shard 3 rotten too
    heal_src = [None if i in (1, 8) else files[i] for i in range(T)]
    heal_src[4] = _rot(torch, files[4], 1099, S, S - 1)      # stripe 1099: data shard 4 rotten
    stream = torch.cuda.Stream()
    for rnd in range(2):
        with torch.cuda.stream(stream):
            tg = [torch.zeros(n * rec, dtype=torch.uint8, device="cuda") if i in (1, 8) else None for i in range(T)]
            t_get = e.decode_records_submit(get_src, S, n, inplace=True, stream=stream)
            t_heal = e.heal_records_submit(heal_src, tg, S, n, stream=stream)
            t_after = e.decode_records_submit(files, S, n, stream=stream)  # queued behind both
        out, status = t_after.wait()
        assert status == [0] * n and torch.equal(out, want), rnd
        assert t_heal.wait() == [0] * n, rnd
        for i in (1, 8):
            assert np.array_equal(tg[i].cpu().numpy().reshape(n, rec), recs[i]), (rnd, i)
        slots, src, status = t_get.wait()
        assert status == [0] * n, rnd
        assert not src[1].any() and not src[6].any()
        assert not src[3][5] and src[3][:5].all() and src[3][6:].all(), rnd
        got = slots.view(n, K, S)
        for i in (1, 6):
            assert torch.equal(got[:, i], want.view(n, K, S)[:, i]), (rnd, i)
        assert torch.equal(got[5, 3], want.view(n, K, S)[5, 3]), rnd  # the rotten record's shard, rebuilt
    assert _lib.load().rsg_sync(gpu.handle, stream.cuda_stream) == 0


def test_in_place_slots_must_not_alias(gpu, oracle):
    """one buffer passed as two slots whose stripe windows collide
    (target_stride == S, slot j = slot i + S: stripe s of slot j is stripe s+1
    of slot i) is refused — two rebuilt shards would overwrite each other; the
    documented block layout (slot i = base + i*S, stride k*S) is accepted."""
    import ctypes
    import torch
    from rustfs_amd import _lib
    S, n = 1024, 4
    shards, recs, files = _oracle_records(torch, oracle, S, n, seed=4)
    L = _lib.load()
    buf = torch.zeros((n + K) * S, dtype=torch.uint8, device="cuda")
    ptrs = (ctypes.c_void_p * T)(*[None if i in (0, 1) else files[i].data_ptr() for i in range(T)])
    status = (ctypes.c_int * n)()
    src = (ctypes.c_uint8 * (K * n))()

    def call(slots, stride):
        tg = (ctypes.c_void_p * K)(*slots)
        return L.rsg_decode_records_into_dev(gpu.handle, K, M, S, n, ptrs, _lib.RSG_HASH_HIGHWAY256S, 1, tg, stride,
                                             src, status, None)
    base = buf.data_ptr()
    alias = [base + i * S for i in range(K)]  # stride S: every slot's stripe s is slot 0's stripe s+i
    assert call(alias, S) == _lib.RSG_ERR_INVALID_ARG
    same = [base] * K
    assert call(same, K * S) == _lib.RSG_ERR_INVALID_ARG
    block = torch.zeros(n * K * S, dtype=torch.uint8, device="cuda")
    assert call([block.data_ptr() + i * S for i in range(K)], K * S) == 0
    torch.cuda.synchronize()
    assert list(status) == [0] * n
    got = block.view(n, K, S).cpu().numpy()
    assert np.array_equal(got[:, 0], shards[:, 0]) and np.array_equal(got[:, 1], shards[:, 1])
