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
