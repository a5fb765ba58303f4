"""Asynchronous host-batch encode (rsg_encode_batch_host_submit / rsg_poll /
rsg_wait): the PUT producer's bounded in-flight queue (encode_batched,
encode.rs:64-72, 795-919) in front of the GPU.  Every job's parity and
digests are checked against the oracle."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pinned(torch, shape):
    return torch.zeros(shape, dtype=torch.uint8).pin_memory().numpy()


def _check(oracle, k, m, st, dig, stripes):
    for s in stripes:
        ref = st[s].copy()
        ref[k:] = 0
        oracle.encode(k, m, ref)
        assert np.array_equal(ref, st[s]), s
        if dig is not None:
            for i in range(k + m):
                assert dig[s, i].tobytes() == oracle.hh256s(ref[i]), (s, i)


@pytest.mark.parametrize("k,m,S,n,jobs", [(8, 4, 131072, 40, 5), (2, 2, 524288, 9, 3), (6, 3, 3001, 17, 4),
                                          (16, 4, 65536, 100, 3)])
def test_submit_poll_many_jobs_in_flight(gpu, oracle, k, m, S, n, jobs):
    import torch
    from rustfs_amd import Erasure
    e = Erasure(k, m, k * S)
    rng = np.random.default_rng(S + n)
    bufs, digs, tickets = [], [], []
    for j in range(jobs):
        st = _pinned(torch, (n, k + m, S))
        st[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
        st[:, k:] = 0xEE
        dig = np.zeros((n, k + m, 32), dtype=np.uint8) if j % 2 == 0 else None
        bufs.append(st)
        digs.append(dig)
        tickets.append(e.encode_batch_host_submit(st, dig))
    # poll every job to completion (in any order), then check each
    pending = list(range(jobs))
    t0 = time.time()
    while pending and time.time() - t0 < 60:
        pending = [j for j in pending if not tickets[j].poll()]
        time.sleep(0.001)
    assert not pending
    for j in range(jobs):
        _check(oracle, k, m, bufs[j], digs[j], sorted({0, n // 2, n - 1}))


def test_wait_and_ticket_release(gpu, oracle):
    import ctypes
    import torch
    from rustfs_amd import Erasure, _lib
    k, m, S, n = 8, 4, 4096, 33
    e = Erasure(k, m, k * S)
    st = _pinned(torch, (n, k + m, S))
    st[:, :k] = np.random.default_rng(1).integers(0, 256, (n, k, S), dtype=np.uint8)
    t = e.encode_batch_host_submit(st)
    t.wait()
    _check(oracle, k, m, st, None, range(n))
    # a released ticket is unknown to the library
    done = ctypes.c_int(0)
    ctx = _lib.context(0)
    assert _lib.load().rsg_poll(ctx.handle, t.ticket, ctypes.byref(done)) == _lib.RSG_ERR_INVALID_ARG
    assert _lib.load().rsg_wait(ctx.handle, 123456789) == _lib.RSG_ERR_INVALID_ARG


def test_pageable_buffers_still_correct(gpu, oracle):
    """Pageable memory works (the copies are then staged by the runtime)."""
    from rustfs_amd import Erasure
    k, m, S, n = 4, 2, 8192, 11
    st = np.zeros((n, k + m, S), dtype=np.uint8)
    st[:, :k] = np.random.default_rng(2).integers(0, 256, (n, k, S), dtype=np.uint8)
    dig = np.zeros((n, k + m, 32), dtype=np.uint8)
    Erasure(k, m, k * S).encode_batch_host_submit(st, dig).wait()
    _check(oracle, k, m, st, dig, range(n))


def test_zero_parity_still_hashes(gpu, oracle):
    """m == 0 with digests requested: every data shard is hashed (ADVICE r1:
    the digests used to be left untouched)."""
    from rustfs_amd import Erasure
    k, S, n = 3, 1000, 4
    st = np.random.default_rng(3).integers(0, 256, (n, k, S), dtype=np.uint8)
    dig = np.zeros((n, k, 32), dtype=np.uint8)
    Erasure(k, 0, k * S).encode_batch_host(st, dig)
    for s in range(n):
        for i in range(k):
            assert dig[s, i].tobytes() == oracle.hh256s(st[s, i]), (s, i)


def test_empty_shards_hash_as_empty_message(gpu, oracle):
    from rustfs_amd import Erasure
    for k, m in ((4, 2), (2, 0)):
        st = np.zeros((3, k + m, 0), dtype=np.uint8)
        dig = np.full((3, k + m, 32), 0x77, dtype=np.uint8)
        Erasure(k, m, 1024).encode_batch_host(st, dig)
        assert all(dig[s, i].tobytes() == oracle.hh256s(b"") for s in range(3) for i in range(k + m))


def test_concurrent_submitters(gpu, oracle):
    """Several producer threads submitting to one context: jobs interleave in
    the slot pipeline, every result stays exact."""
    import threading
    import torch
    from rustfs_amd import Erasure
    k, m, S, n = 8, 4, 16384, 24
    e = Erasure(k, m, k * S)
    errors = []

    def producer(seed):
        try:
            rng = np.random.default_rng(seed)
            for _ in range(4):
                st = _pinned(torch, (n, k + m, S))
                st[:, :k] = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
                dig = np.zeros((n, k + m, 32), dtype=np.uint8)
                e.encode_batch_host_submit(st, dig).wait()
                _check(oracle, k, m, st, dig, (0, n - 1))
        except Exception as exc:  # surfaced below
            errors.append(repr(exc))

    th = [threading.Thread(target=producer, args=(s,)) for s in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:2]
