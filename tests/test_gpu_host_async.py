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


def test_ticket_waited_from_many_threads(gpu, oracle):
    """Several threads waiting on and polling one ticket all see it finish
    (the job's events live until the last waiter returns); afterwards the
    ticket is released."""
    import ctypes
    import threading
    import torch
    from rustfs_amd import Erasure, _lib
    k, m, S, n = 8, 4, 131072, 96
    e = Erasure(k, m, k * S)
    L, ctx = _lib.load(), _lib.context(0).handle
    st = _pinned(torch, (n, k + m, S))
    st[:, :k] = np.random.default_rng(9).integers(0, 256, (n, k, S), dtype=np.uint8)
    dig = _pinned(torch, (n, k + m, 32))
    for rep in range(3):
        t = ctypes.c_uint64(0)
        _lib.check(L.rsg_encode_batch_host_submit(ctx, k, m, S, n, st.ctypes.data, S, (k + m) * S,
                                                  dig.ctypes.data, _lib.RSG_HASH_HIGHWAY256S, ctypes.byref(t)))
        res = []

        def waiter(poll):
            if poll:
                done = ctypes.c_int(0)
                while True:
                    rc = L.rsg_poll(ctx, t.value, ctypes.byref(done))
                    if rc != 0 or done.value:
                        res.append((rc, done.value))
                        return
            else:
                res.append((L.rsg_wait(ctx, t.value), 1))

        th = [threading.Thread(target=waiter, args=(i % 2 == 1,)) for i in range(6)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=60)
        # every caller either saw the job finish or, arriving after another
        # released it, got INVALID_ARG; at least one saw it finish
        assert all(rc in (_lib.RSG_OK, _lib.RSG_ERR_INVALID_ARG) for rc, _ in res), res
        assert any(rc == _lib.RSG_OK and d == 1 for rc, d in res), res
        assert L.rsg_wait(ctx, t.value) == _lib.RSG_ERR_INVALID_ARG
    _check(oracle, k, m, st, dig, [0, n - 1])


def test_submit_failure_drains_queued_subbatches(tmp_path):
    """rsg_encode_batch_host_submit failing on a later sub-batch (fault
    injected with the test-only rsg_test_fail_subbatch, in a child process) returns the
    error only after the sub-batches it had queued have landed: their parity
    and digests are in the caller's buffers when the call returns, nothing is
    left in flight, and no ticket is issued."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "child.py"
    script.write_text(f'''
import ctypes, sys
sys.path.insert(0, {root!r})
import numpy as np, torch
from oracle import oracle as O
from rustfs_amd import _lib
L = _lib.load(); ctx = _lib.context(0).handle
assert L.rsg_test_fail_subbatch(ctx, 1) == _lib.RSG_OK
k, m, S = 8, 4, 131072
n = 3 * ((96 << 20) // ((k + m) * S))  # three ~96 MiB sub-batches
st = torch.zeros((n, k + m, S), dtype=torch.uint8).pin_memory().numpy()
st[:, :k] = np.random.default_rng(4).integers(0, 256, (n, k, S), dtype=np.uint8)
st[:, k:] = 0xEE
dig = torch.zeros((n, k + m, 32), dtype=torch.uint8).pin_memory().numpy()
t = ctypes.c_uint64(77)
rc = L.rsg_encode_batch_host_submit(ctx, k, m, S, n, st.ctypes.data, S, (k + m) * S, dig.ctypes.data,
                                    _lib.RSG_HASH_HIGHWAY256S, ctypes.byref(t))
assert rc == _lib.RSG_ERR_DEVICE and t.value == 0, (rc, t.value)
# sub-batch 0 completed before the call returned: no synchronisation here
ref = st[0].copy(); ref[k:] = 0; O.encode(k, m, ref)
assert np.array_equal(ref, st[0]) and dig[0, 0].tobytes() == O.hh256s(ref[0])
assert (st[n - 1, k:] == 0xEE).all()  # the failed and later sub-batches wrote nothing
# the context still works afterwards
t2 = ctypes.c_uint64(0)
assert L.rsg_encode_batch_host_submit(ctx, k, m, S, 4, st.ctypes.data, S, (k + m) * S, None, 0,
                                      ctypes.byref(t2)) == _lib.RSG_OK  # one sub-batch: index 1 never comes
assert L.rsg_wait(ctx, t2.value) == _lib.RSG_OK
assert L.rsg_test_fail_subbatch(ctx, -1) == _lib.RSG_OK
print("child ok")
''')
    p = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=150)
    assert p.returncode == 0 and "child ok" in p.stdout, p.stderr[-3000:]
