"""GET-side engine (rsg_decode_records_dev): verify-before-use of BitrotWriter
records + batched reconstruct + surplus-parity verification, on the GPU,
against the CPU oracle and the reference's semantics (bridge.rs:274-307,
bitrot.rs:227-247, erasure.rs:935-973)."""
import numpy as np
import pytest

from conftest import decode_get

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("engine_path")]


@pytest.fixture(params=["gather", "into"])
def form(request):
    """Both output forms of the GET engine: the contiguous gather
    (rsg_decode_records_dev) and reconstruct_into's in-place form
    (rsg_decode_records_into_dev)."""
    return request.param


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


def _records(torch, k, m, S, n, seed):
    from rustfs_amd import Erasure
    e = Erasure(k, m, k * S)
    g = torch.Generator(device="cuda").manual_seed(seed)
    st = torch.zeros((n, k + m, S), dtype=torch.uint8, device="cuda")
    st[:, :k] = torch.randint(0, 256, (n, k, S), dtype=torch.uint8, device="cuda", generator=g)
    dig = torch.zeros((n, k + m, 32), dtype=torch.uint8, device="cuda")
    e.encode_batch(st, dig)
    files = [torch.cat([dig[:, i], st[:, i]], dim=1).contiguous().reshape(-1) for i in range(k + m)]
    return e, st, files


@pytest.mark.parametrize("k,m,S,n", [(8, 4, 4096, 9), (4, 2, 3001, 5), (12, 4, 87382, 3), (2, 2, 524288, 2)])
def test_decode_records_paths(gpu, oracle, form, k, m, S, n):
    import torch
    from rustfs_amd import _lib
    e, st, files = _records(torch, k, m, S, n, seed=S)
    want = st[:, :k].reshape(n, k * S)
    rec = 32 + S
    # all present: copy path
    out, status = decode_get(e, files, S, n, form)
    assert status == [0] * n and torch.equal(out, want)
    # whole files lost (up to m): reconstruct path, common pattern
    lost = [0, k] if m >= 2 else [0]
    f2 = [None if i in lost else files[i] for i in range(k + m)]
    out, status = decode_get(e, f2, S, n, form)
    assert status == [0] * n and torch.equal(out, want)
    # a corrupted data record in one stripe: that stripe alone treats the shard as missing
    f3 = [f.clone() for f in files]
    f3[1][1 * rec + 32 + 17] ^= 0x40
    out, status = decode_get(e, f3, S, n, form)
    assert status == [0] * n and torch.equal(out, want)
    # more than m bad records in one stripe: read quorum lost for that stripe only
    f4 = [f.clone() for f in files]
    for i in range(m + 1):
        f4[i][(n - 1) * rec + 3] ^= 0x01  # digest byte
    out, status = decode_get(e, f4, S, n, form)
    assert status[:-1] == [0] * (n - 1) and status[-1] == _lib.RSG_ERR_TOO_FEW_SHARDS
    assert torch.equal(out[:-1], want[:-1])


def test_decode_records_detects_inconsistent_parity(gpu, oracle, form):
    """A parity record whose digest matches but whose bytes disagree with the
    data: InvalidData 'inconsistent read source shards' when data must be rebuilt."""
    import torch
    from rustfs_amd import _lib
    k, m, S, n = 8, 4, 4096, 4
    e, st, files = _records(torch, k, m, S, n, seed=5)
    rec = 32 + S
    bad = files[k + 2].clone()
    body = bad[2 * rec + 32: 3 * rec].cpu().numpy().copy()
    body[100] ^= 0xFF
    bad[2 * rec + 32: 3 * rec] = torch.from_numpy(body).cuda()
    bad[2 * rec: 2 * rec + 32] = torch.from_numpy(np.frombuffer(oracle.hh256s(body), dtype=np.uint8).copy()).cuda()
    f = [None] + files[1:k + 2] + [bad] + files[k + 3:]
    out, status = decode_get(e, f, S, n, form)
    assert status == [0, 0, _lib.RSG_ERR_INCONSISTENT_SOURCES, 0]
    want = st[:, :k].reshape(n, k * S)
    assert torch.equal(out[0], want[0]) and torch.equal(out[3], want[3])
    # without surplus verification the rebuilt data is still exact (the parity is not a survivor)
    out, status = decode_get(e, f, S, n, form, verify_surplus=False)
    assert status == [0] * n and torch.equal(out, want)


@pytest.mark.parametrize("k,m,S,n,lost", [
    (8, 4, 131072, 5, (0,)), (8, 4, 131072, 6, (0, 3)), (8, 4, 4096, 9, (1, 4, 6)), (8, 4, 4096, 7, (0, 2, 5, 7)),
    (8, 4, 4096, 7, (3, 9)), (8, 4, 4096, 5, (2, 8, 11)), (4, 2, 65536, 4, (1,)), (6, 3, 4096, 3, (0, 5, 7)),
    (2, 2, 1024, 3, (0,)), (1, 3, 512, 2, (0, 2)), (5, 4, 2048, 9, (4,)),
    (8, 4, 512, 17, (0,)), (8, 4, 512, 3, (1, 2, 3, 4)), (8, 4, 1024, 8, (7, 8, 9)), (8, 4, 4608, 11, (6,)),
    (16, 4, 4096, 9, (0,)), (16, 4, 4096, 5, (3, 17)), (16, 4, 512, 13, (0, 5, 9, 15)), (16, 2, 1024, 4, (15,)),
    (16, 4, 65536, 6, (2, 11)), (2, 4, 2048, 6, (0, 1)), (4, 4, 1024, 5, (1, 2, 6)), (2, 2, 524288, 3, (1,)),
    # ragged walks (S not a multiple of 512) at rustfs's default set geometries, 1 MiB blocks
    (12, 4, 87382, 5, (0, 13)), (12, 4, 87382, 3, (4, 5, 6)), (10, 4, 104858, 3, (1,)), (6, 4, 174763, 3, (0, 2)),
    (6, 3, 3001, 4, (5,)), (8, 4, 100, 9, (0,)), (8, 4, 1, 5, (7,)), (4, 2, 31, 7, (0,)),
])
def test_decode_records_lost_disk_one_pass(gpu, oracle, form, k, m, S, n, lost):
    """A lost disk (whole data shard files missing) takes the one-pass GET
    kernel (verify + gather + rebuild + surplus check): bit-exact output."""
    import torch
    e, st, files = _records(torch, k, m, S, n, seed=S + len(lost))
    want = st[:, :k].reshape(n, k * S)
    f = [None if i in lost else files[i] for i in range(k + m)]
    out, status = decode_get(e, f, S, n, form)
    assert status == [0] * n and torch.equal(out, want)
    out, status = decode_get(e, f, S, n, form, verify_surplus=False)
    assert status == [0] * n and torch.equal(out, want)


def test_decode_records_lost_disk_with_rotten_record(gpu, oracle, form):
    """Lost disk plus a rotten record elsewhere: the one-pass result is not
    trusted (a digest mismatched), the general path picks other survivors for
    that stripe and still returns the exact data."""
    import torch
    k, m, S, n = 8, 4, 4096, 6
    e, st, files = _records(torch, k, m, S, n, seed=11)
    rec = 32 + S
    want = st[:, :k].reshape(n, k * S)
    f = [None if i == 2 else files[i].clone() for i in range(k + m)]
    f[5][3 * rec + 32 + 100] ^= 0x08  # data record body of stripe 3
    f[k][1 * rec + 7] ^= 0x01  # parity digest of stripe 1
    out, status = decode_get(e, f, S, n, form)
    assert status == [0] * n and torch.equal(out, want)


def test_decode_records_lost_disk_inconsistent_surplus(gpu, oracle, form):
    """Lost disk, every digest valid, one surplus parity record re-hashed after
    a bit flip: the one-pass kernel reports InvalidData for that stripe only."""
    import torch
    from rustfs_amd import _lib
    k, m, S, n = 8, 4, 4096, 5
    e, st, files = _records(torch, k, m, S, n, seed=13)
    rec = 32 + S
    bad = files[k + 3].clone()
    body = bad[4 * rec + 32: 5 * rec].cpu().numpy().copy()
    body[7] ^= 0x10
    bad[4 * rec + 32: 5 * rec] = torch.from_numpy(body).cuda()
    bad[4 * rec: 4 * rec + 32] = torch.from_numpy(np.frombuffer(oracle.hh256s(body), dtype=np.uint8).copy()).cuda()
    f = [None if i == 0 else files[i] for i in range(k + m)]
    f[k + 3] = bad
    out, status = decode_get(e, f, S, n, form)
    assert status == [0, 0, 0, 0, _lib.RSG_ERR_INCONSISTENT_SOURCES]
    want = st[:, :k].reshape(n, k * S)
    assert torch.equal(out[:4], want[:4])


@pytest.mark.parametrize("k,m,lost", [(8, 4, (0, 5)), (16, 4, (0, 5)), (16, 4, (9,)), (4, 4, (1, 2))])
def test_decode_records_lost_disk_many_workgroups(gpu, oracle, form, k, m, lost):
    """One-pass GET kernel over many workgroups (8 stripes each, 4 for
    RS(16,4)) and a ragged last one: rotten records and an inconsistent
    surplus parity scattered over the batch are each caught for their own
    stripe only."""
    import torch
    from rustfs_amd import _lib
    S, n = 4096, 2051
    e, st, files = _records(torch, k, m, S, n, seed=17 + k)
    rec = 32 + S
    want = st[:, :k].reshape(n, k * S)
    f = [None if i in lost else files[i].clone() for i in range(k + m)]
    f[3][2050 * rec + 32 + 9] ^= 0x02       # data record body, last stripe
    f[k + 1][8 * rec + 1] ^= 0x80           # survivor parity digest, stripe 8
    body = f[k + 3][1234 * rec + 32: 1235 * rec].cpu().numpy().copy()
    body[4000] ^= 0x01                      # surplus parity of stripe 1234, re-hashed: inconsistent
    f[k + 3][1234 * rec + 32: 1235 * rec] = torch.from_numpy(body).cuda()
    f[k + 3][1234 * rec: 1234 * rec + 32] = torch.from_numpy(
        np.frombuffer(oracle.hh256s(body), dtype=np.uint8).copy()).cuda()
    out, status = decode_get(e, f, S, n, form)
    bad = [i for i, s in enumerate(status) if s != 0]
    assert bad == [1234] and status[1234] == _lib.RSG_ERR_INCONSISTENT_SOURCES
    ok = torch.ones(n, dtype=torch.bool, device="cuda")
    ok[1234] = False
    assert torch.equal(out[ok], want[ok])


def test_kernel_timing_hook(gpu, oracle, engine_path):
    """rsg_set_kernel_timing / rsg_last_kernel_ms (bench.py's measurement
    hook): off by default (-1), a positive kernel time after a timed GET with
    a lost disk, after an all-present GET and after a whole-file
    bitrot_verify, unchanged results."""
    import ctypes
    import torch
    from rustfs_amd import _lib
    k, m, S, n = 8, 4, 4096, 16
    e, st, files = _records(torch, k, m, S, n, seed=77)
    want = st[:, :k].reshape(n, k * S)
    L, ctx = _lib.load(), _lib.context(0).handle
    v = ctypes.c_float(0)
    _lib.check(L.rsg_set_kernel_timing(ctx, 0))
    decode_get(e, files, S, n, "gather")
    _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
    assert v.value == -1.0
    _lib.check(L.rsg_set_kernel_timing(ctx, 1))
    try:
        for form in ("gather", "into"):
            for lost in ((), (0, 3)):
                fl = [None if i in lost else files[i] for i in range(k + m)]
                out, status = decode_get(e, fl, S, n, form)
                assert status == [0] * n and torch.equal(out, want)
                _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
                assert v.value > 0, (form, lost)
        # whole-file bitrot_verify is timed the same way
        from rustfs_amd.bitrot import HashAlgorithm, bitrot_verify_batch
        rec = 32 + S
        assert bitrot_verify_batch(files, n * rec, n * S, HashAlgorithm.HighwayHash256S, S) == [0] * (k + m)
        _lib.check(L.rsg_last_kernel_ms(ctx, ctypes.byref(v)))
        assert v.value > 0
    finally:
        _lib.check(L.rsg_set_kernel_timing(ctx, 0))


@pytest.mark.parametrize("S", [4096, 4102, 4099])
def test_into_serves_verified_records_in_place(gpu, oracle, S):
    """reconstruct_into's contract (bridge.rs:274-307, :52-54): with every data
    shard present nothing is written; a rotten data record is the only shard
    rebuilt, into its slot, and reported as not served from its record.
    Records at 0 mod 16 (the quad hash kernel's verify), 6 mod 16 and odd
    pitches (the LDS-DMA ring's, rs_verify.hip; 5 stripes: a partial
    workgroup)."""
    import torch
    from conftest import SLOT_FILL
    k, m, n = 8, 4, 5
    e, st, files = _records(torch, k, m, S, n, seed=21)
    rec = 32 + S
    slots = torch.full((n, k * S), SLOT_FILL, dtype=torch.uint8, device="cuda")
    _, src, status = e.decode_records_into_batch(files, S, n, targets=slots)
    assert status == [0] * n and src.all()
    assert bool((slots == SLOT_FILL).all()), "an all-present GET wrote a slot"
    f = [x.clone() for x in files]
    f[1][3 * rec + 32 + 77] ^= 0x10  # data record 1 of stripe 3 rots
    _, src, status = e.decode_records_into_batch(f, S, n, targets=slots)
    assert status == [0] * n
    want_src = np.ones((k, n), dtype=bool)
    want_src[1, 3] = False
    assert np.array_equal(src, want_src)
    got = slots.view(n, k, S)
    assert torch.equal(got[3, 1], st[3, 1])
    untouched = torch.ones((n, k), dtype=torch.bool, device="cuda")
    untouched[3, 1] = False
    assert bool((got[untouched] == SLOT_FILL).all())


def test_into_lost_disk_strided_slots(gpu, oracle):
    """Slots as k separate buffers with a stride larger than the shard: only
    the lost shards' slots are written, at that stride."""
    import torch
    k, m, S, n = 8, 4, 4096, 9
    e, st, files = _records(torch, k, m, S, n, seed=23)
    stride = S + 64
    slots = [torch.full((n * stride,), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(k)]
    f = [None if i in (0, 3) else files[i] for i in range(k + m)]
    _, src, status = e.decode_records_into_batch(f, S, n, targets=slots, target_stride=stride)
    assert status == [0] * n
    for i in range(k):
        v = slots[i].view(n, stride)
        if i in (0, 3):
            assert not src[i].any() and torch.equal(v[:, :S], st[:, i]) and bool((v[:, S:] == 0x5A).all())
        else:
            assert src[i].all() and bool((v == 0x5A).all())


def test_into_rejects_bad_slots(gpu, oracle):
    """A slot overlapping a source record file, a stride shorter than the
    shard, or both output forms at once: RSG_ERR_INVALID_ARG, nothing run."""
    import ctypes
    import torch
    from rustfs_amd import _lib
    k, m, S, n = 4, 2, 1024, 3
    e, st, files = _records(torch, k, m, S, n, seed=25)
    f = [None] + files[1:]
    with pytest.raises(_lib.RsgError) as ei:
        e.decode_records_into_batch(f, S, n, targets=[files[2]] * k, target_stride=S)
    assert ei.value.code == _lib.RSG_ERR_INVALID_ARG
    slots = [torch.empty(n * S, dtype=torch.uint8, device="cuda") for _ in range(k)]
    with pytest.raises(_lib.RsgError) as ei:
        e.decode_records_into_batch(f, S, n, targets=[torch.empty(n * S, dtype=torch.uint8, device="cuda")
                                                      for _ in range(k)], target_stride=S - 1)
    assert ei.value.code == _lib.RSG_ERR_INVALID_ARG
    L = _lib.load()
    ptrs = (ctypes.c_void_p * (k + m))(*[x.data_ptr() if x is not None else None for x in f])
    tp = (ctypes.c_void_p * k)(*[x.data_ptr() for x in slots])
    out = torch.empty(n * k * S, dtype=torch.uint8, device="cuda")
    status = (ctypes.c_int * n)()
    tk = ctypes.c_uint64(0)
    assert L.rsg_decode_records_submit(gpu.handle, k, m, S, n, ptrs, 1, 1, out.data_ptr(), tp, S, None, status,
                                       None, ctypes.byref(tk)) == _lib.RSG_ERR_INVALID_ARG
    assert L.rsg_decode_records_submit(gpu.handle, k, m, S, n, ptrs, 1, 1, None, None, 0, None, status,
                                       None, ctypes.byref(tk)) == _lib.RSG_ERR_INVALID_ARG
